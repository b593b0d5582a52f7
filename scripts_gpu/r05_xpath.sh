#!/bin/bash
# xpath frame-group-major tile order: unet goldens, layer-9 time and PMC WRITE, A/B against the
# class-major order (EXTDM_XP_FG=0).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
sha256sum 140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd/libextdm_hip.so | cut -c1-16
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "golden or oracle" > gpurun_out/r05_xp_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05_xp_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for fg in 8 0 4 16; do EXTDM_XP_FG=$fg timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 9 | sed "s/^/FG=$fg /" || exit 1; done; done
for fg in 8 0; do
  EXTDM_XP_FG=$fg LAYERS=9 bash scripts_gpu/pmc_layers.sh > gpurun_out/r05_xp_pmc_$fg.log 2>&1 || { tail -5 gpurun_out/r05_xp_pmc_$fg.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/pmc_layer9.json')); print('FG=$fg', 'FETCH raw MB', d['fetch_bytes_raw_per_launch']/1e6, 'WRITE MB', d['write_bytes_per_launch']/1e6)"
  cp gpurun_out/pmc_layer9.json gpurun_out/pmc_layer9_fg$fg.json
done
