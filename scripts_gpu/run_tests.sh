#!/bin/bash
# GPU validation: smoke, then the gpu-marked tests with every parity check's error on record
# (tests/parity_log.py -> gpurun_out/parity_errors.jsonl -> gpurun_out/parity_errors.json).
# Stops after any crash-class exit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
rm -f gpurun_out/parity_errors.jsonl
EXTDM_PARITY_LOG=$PWD/gpurun_out/parity_errors.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s -x --timeout 600 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc2=$?
echo "tests rc=$rc2"
grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -3
python scripts_gpu/parity_errors.py gpurun_out/parity_errors.jsonl gpurun_out/parity_errors.json \
  $(sha256sum 140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd/libextdm_hip.so | cut -c1-16)
exit $rc2
