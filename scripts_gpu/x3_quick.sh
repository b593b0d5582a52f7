#!/bin/bash
# quick loop: f16x3 precision tests + conv layer timings
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_precision.py -x -q -s --timeout 200 --timeout-method thread ${PYTEST_K} > gpurun_out/x3_tests.log 2>&1
rc=$?; echo "x3 tests rc=$rc"; grep -E "FAIL|Error|vs fp64|passed|failed" gpurun_out/x3_tests.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts_gpu/layers.py 32 20 ${PRECS:-f16x3} ${LAYERS:-0,1,2,3,4}
