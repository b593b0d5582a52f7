#!/bin/bash
# conv_x3 stage-barrier A/B: parity + precision tests, then bench_layer timings with the
# spanning barriers (default) and with EXTDM_X3_NOSPAN=1
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "$TESTS" != none ]; then
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_precision.py tests/test_gpu_parity.py} -x -q --timeout 200 --timeout-method thread > gpurun_out/span_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/span_tests.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 120 python scripts_gpu/layers.py 64 20 f16x3 ${LAYERS:-0,1,2,3,4} && [ -z "$NO_AB" ] && \
EXTDM_X3_NOSPAN=1 timeout -k 10 120 python scripts_gpu/layers.py 64 20 f16x3 ${LAYERS:-0,1,2,3,4}
