#!/bin/bash
# session-2 check: parity of the res_conv GroupNorm fusion, the attention timing-only
# switches, bench at B = 64 and B = 128
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_precision.py tests/test_gpu_attn.py -x -q --timeout 300 --timeout-method thread > gpurun_out/s2a_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s2a_tests.log; [ $rc -ne 0 ] && exit $rc
for d in 0 4 8 12; do
  EXTDM_X3_DBG=$d timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 >> gpurun_out/s2a_attn.log 2>&1 || exit $?
done
cat gpurun_out/s2a_attn.log | grep dbg
for B in 64 128; do
  timeout -k 10 300 python bench.py --sampling-steps 50 --steps 50 --warmup 5 --batch $B --no-cpu-baseline > gpurun_out/s2a_b$B.json 2> gpurun_out/s2a_b$B.err || exit $?
  tail -c 300 gpurun_out/s2a_b$B.json | head -c 200; echo
done
