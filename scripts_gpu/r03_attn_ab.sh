#!/bin/bash
# A/B layer timing of the in-tree library against $BASE (default _variants/base), after the
# attention layer tests; output under gpurun_out/${TAG}_*.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03b}
BASE=${BASE:-_variants/base/libextdm_hip.so}
timeout -k 10 400 python -u -m pytest tests/test_gpu_attn.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 >> gpurun_out/${TAG}_ab.txt || exit 1
  EXTDM_LIB=$BASE timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 >> gpurun_out/${TAG}_ab.txt || exit 1
done
cat gpurun_out/${TAG}_ab.txt
