#!/bin/bash
# Sampler update with four elements per thread (one Philox block, two Box-Muller pairs per four
# normals; the same values): the sampler / chain parity tests, then the closing PMC passes and the
# DDIM-20 BAIR kernel stats on this library (measure.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wrappers.py tests/test_gpu_bench_ranks.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/sampler4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/sampler4_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts_gpu/measure.sh
