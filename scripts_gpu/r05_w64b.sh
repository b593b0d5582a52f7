#!/bin/bash
# stw64_x3 tile path: window-64 attention tests, then layer-6 timings tile vs per-lane.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
sha256sum 140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd/libextdm_hip.so | cut -c1-16
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_attn.py -k window64 > gpurun_out/r05_w64b_tests.log 2>&1
rc=$?; echo "w64 tests rc=$rc"; grep -E "parity|passed|failed" gpurun_out/r05_w64b_tests.log | tail -14; [ $rc -ne 0 ] && exit $rc
for c in kth cityscapes ucf; do
  timeout -k 10 120 python scripts_gpu/layers_cfg.py $c 6 || exit 1
  EXTDM_STW64_NO_TILE=1 timeout -k 10 120 python scripts_gpu/layers_cfg.py $c 6 || exit 1
done
