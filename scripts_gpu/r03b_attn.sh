#!/bin/bash
# Round 3 session 2: attention layer tests + A/B layer timing (in-tree vs _variants/base),
# then the activation-scale precision tests and the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03b}
BASE=${BASE:-_variants/base/libextdm_hip.so}
timeout -k 10 400 python -u -m pytest tests/test_gpu_attn.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_attn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_attn_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 || exit 1
  EXTDM_LIB=$BASE timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 || exit 1
done
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 600 python -u -m pytest tests/test_gpu_precision.py -x -v -s --timeout 300 --timeout-method thread -k "scales or fp64" > gpurun_out/${TAG}_prec.log 2>&1
echo "prec rc=$?"; grep -E "s=|vs fp64|passed|failed" gpurun_out/${TAG}_prec.log | tail -12
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/${TAG}_bench.json; exit $rc
