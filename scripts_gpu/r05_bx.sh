#!/bin/bash
# A/B of the compile-time buffer-load X staging (BX) in conv_x3: parity subset, layer times, steps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
sha256sum 140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd/libextdm_hip.so | cut -c1-16
true && rc=0 && echo > gpurun_out/r05_bx_tests.log
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05_bx_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 0,1,5,4,13 || exit 1
  EXTDM_X3_NO_BX=1 timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 0,1,5,4,13 || exit 1
done
S=20 AB="EXTDM_X3_NO_BX=1" bash scripts_gpu/ab_step.sh
