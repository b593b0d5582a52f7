#!/bin/bash
# Round 3 session 2: HEAD re-check on a fresh box — the activation-scale precision tests,
# the attention layer tests, and the default bench line (BAIR, B = 64, DDPM-1000).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_precision.py -x -v -s --timeout 300 --timeout-method thread -k "scales or fp64" > gpurun_out/${TAG}_prec.log 2>&1
echo "prec rc=$?"; grep -E "s=|vs fp64|passed|failed" gpurun_out/${TAG}_prec.log | tail -12
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/${TAG}_bench.json; exit $rc
