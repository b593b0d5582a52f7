#!/bin/bash
# STW / temporal attention diagnosis: s_memtime phase stamps (EXTDM_X3_DBG=32), then the SQ
# counters of the in-tree kernels (two --pmc passes)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03b_ad}
EXTDM_X3_DBG=32 timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 2 > gpurun_out/${TAG}_stamps.log 2>&1
echo "stamps rc=$?"; grep -E "attn_x3<|lib=" gpurun_out/${TAG}_stamps.log | cut -c1-600
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_MFMA"; do
  rm -rf gpurun_out/${TAG}_p$i
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_p$i -o run --output-format csv -- python scripts_gpu/attn_dbg.py 64 5 > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_p$i.log; exit $rc; }
  i=$((i+1))
done
python scripts_gpu/pmc_table.py gpurun_out/${TAG}_p0 gpurun_out/${TAG}_p1 > gpurun_out/${TAG}_table.txt
find gpurun_out/${TAG}_p0 gpurun_out/${TAG}_p1 -name "*kernel_trace.csv" -delete
cat gpurun_out/${TAG}_table.txt
