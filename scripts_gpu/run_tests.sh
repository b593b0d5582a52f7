#!/bin/bash
# GPU validation: smoke, then the gpu-marked tests. Stops after any crash-class exit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout 600 ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc2=$?
echo "tests rc=$rc2"
tail -30 gpurun_out/gpu_tests.log
exit $rc2
