#!/bin/bash
# Occupancy hints (amdgpu_waves_per_eu): noise_pool_x3 at four waves per SIMD (142 -> 120 registers,
# no AGPR accumulators) and the FAST 128-row implicit-GEMM tiles (Downsample / ConvTranspose /
# 1x1) at four. Parity tests, then noise_pool's layer time and whole BAIR DDIM-20 steps against the
# previous library (_variants/base), interleaved twice on one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_e2e_configs.py tests/test_gpu_lfae.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/occ_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/occ_tests.log; [ $rc -ne 0 ] && exit $rc
OLD=$PWD/_variants/base/libextdm_hip.so
for rep in 1 2; do
  for lib in old new; do
    if [ $lib = old ]; then L="EXTDM_LIB=$OLD"; else L=""; fi
    env $L timeout -k 10 120 python scripts_gpu/layers.py 128 20 f16x3 10,9 | sed "s/^/$lib /" || exit 1
    env $L timeout -k 10 300 python bench.py --sampling-steps 20 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline \
      > gpurun_out/occ_$lib$rep.json 2> gpurun_out/occ_$lib$rep.err || { tail -5 gpurun_out/occ_$lib$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/occ_$lib$rep.json').read().strip().splitlines()[-1]); print('$lib$rep bair', d['ms_per_step'], d['value'])"
  done
done
