#!/bin/bash
# SQ counters of the level-0 STW attention kernels, in-tree vs $BASE (two --pmc passes each)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03b_pa}
BASE=${BASE:-_variants/base/libextdm_hip.so}
for arm in new base; do
  i=0
  for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_MFMA"; do
    rm -rf gpurun_out/${TAG}_${arm}_p$i
    if [ $arm = base ]; then export EXTDM_LIB=$BASE; else unset EXTDM_LIB; fi
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_${arm}_p$i -o run --output-format csv -- python scripts_gpu/attn_dbg.py 64 5 > gpurun_out/${TAG}_${arm}_p$i.log 2>&1
    rc=$?; echo "$arm pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_${arm}_p$i.log; exit $rc; }
    i=$((i+1))
  done
  python scripts_gpu/pmc_table.py gpurun_out/${TAG}_${arm}_p0 gpurun_out/${TAG}_${arm}_p1 > gpurun_out/${TAG}_${arm}_table.txt
  find gpurun_out/${TAG}_${arm}_p0 gpurun_out/${TAG}_${arm}_p1 -name "*kernel_trace.csv" -delete
done
grep -A17 "attn_x3_kernelILi64ELi0ELi32ELi8ELb1" gpurun_out/${TAG}_new_table.txt gpurun_out/${TAG}_base_table.txt
