#!/bin/bash
# SQ counter passes over the bench_layer convs (f16x3) + layer timings.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LAYERS=${LAYERS:-0,1,2,3,4}
timeout -k 10 120 python scripts_gpu/layers.py 32 20 fp32,f16x3 $LAYERS > gpurun_out/layers.log 2>&1
rc=$?; cat gpurun_out/layers.log; [ $rc -ne 0 ] && exit $rc
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE FETCH_SIZE"; do
  rm -rf gpurun_out/pmc_l$i
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_l$i -o run --output-format csv -- python scripts_gpu/layers.py 32 3 f16x3 $LAYERS > gpurun_out/pmc_l$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_l$i.log; exit $rc; }
  i=$((i+1))
done
python scripts_gpu/pmc_table.py gpurun_out/pmc_l0 gpurun_out/pmc_l1
