#!/bin/bash
# SQ stall breakdown + instruction mix of one bench layer of CONFIG's denoiser (cfg_handle.py):
# two separate --pmc passes (8 SQ counters max per pass; GRBM in its own block). CONFIG / LAYER /
# TAG from env; summary by scripts_gpu/pmc_table.py.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=${LAYER:-1}; CONFIG=${CONFIG:-bair}; TAG=${TAG:-sq}
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_MFMA"; do
  rm -rf gpurun_out/${TAG}_l${L}_p$i
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_l${L}_p$i -o run --output-format csv -- python scripts_gpu/pmc_layer_run.py $CONFIG $L 5 > gpurun_out/${TAG}_l${L}_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_l${L}_p$i.log; exit $rc; }
  i=$((i+1))
done
python scripts_gpu/pmc_table.py gpurun_out/${TAG}_l${L}_p0 gpurun_out/${TAG}_l${L}_p1
find gpurun_out/${TAG}_l${L}_p* -name "*trace*.csv" -delete
