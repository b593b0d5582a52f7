#!/bin/bash
# Fence-free sampler step: the radix bins read with device-scope atomic loads and zeroed with
# device-scope atomic stores, the step advance in a one-workgroup launch. First the tests that caught
# the plain-load version (two ranks vs one, bitwise) with the sampler / chain parity tests; if green,
# the closing PMC passes + DDIM-20 stats (measure.sh) on this library.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_ranks.py tests/test_gpu_parity.py tests/test_gpu_wrappers.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/coherent_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/coherent_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts_gpu/measure.sh
