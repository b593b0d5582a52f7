#!/bin/bash
# Round 3: the f16x3 attention kernels — layer tests, A/B layer timing of the in-tree
# library against $BASE (default _variants/base, HEAD sources), and a rocprofv3 kernel trace
# (per-launch durations) of the in-tree layers at B = 64.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03a}
BASE=${BASE:-_variants/base/libextdm_hip.so}
timeout -k 10 400 python -u -m pytest tests/test_gpu_attn.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 || exit 1
  EXTDM_LIB=$BASE timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 || exit 1
done
rm -rf gpurun_out/${TAG}_kt
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_kt -o run --output-format csv -- python scripts_gpu/attn_dbg.py 64 20 > gpurun_out/${TAG}_kt.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_kt.log; exit $rc; }
python scripts_gpu/kernel_launches.py gpurun_out/${TAG}_kt attn_x3_kernel > gpurun_out/${TAG}_launches.txt
cat gpurun_out/${TAG}_launches.txt
