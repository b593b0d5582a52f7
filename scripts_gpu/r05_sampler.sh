#!/bin/bash
# Multi-workgroup sampler step: parity (quantile bit-exactness, chains, graph == eager), then
# whole-step A/B against the one-workgroup kernel (EXTDM_SAMPLER_1WG=1), BAIR and UCF.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
sha256sum 140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd/libextdm_hip.so | cut -c1-16
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_wrappers.py tests/test_gpu_chain_precision.py > gpurun_out/r05_sampler_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05_sampler_tests.log; [ $rc -ne 0 ] && exit $rc
S=20 AB="EXTDM_SAMPLER_1WG=1" bash scripts_gpu/ab_step.sh || exit 1
for arm in 0 1; do
  EXTDM_SAMPLER_1WG=$arm timeout -k 10 300 python bench.py --config ucf --no-cpu-baseline --no-roofline > gpurun_out/r05_ucf_$arm.json 2>gpurun_out/r05_ucf_$arm.err || exit 1
  tail -1 gpurun_out/r05_ucf_$arm.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ucf 1WG=$arm', d['value'], d['ms_per_step'])"
done
