# phase-composed fea conv: parity subset + layer timings (0 = 5x5 phase conv, 11 = edges) + kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "unet_forward_vs_reference_golden or batch_independence or range_guard" > gpurun_out/r04_fea_tests.log 2>&1 || exit 1
for v in "" "EXTDM_FEA_XBUF=1" "EXTDM_FEA_TILE=256"; do
  echo "== $v" >> gpurun_out/r04_fea_layers.log
  env $v timeout -k 10 300 python scripts_gpu/layers.py 64 20 f16x3 0,11 >> gpurun_out/r04_fea_layers.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_fea -o run -- python scripts_gpu/layers.py 64 5 f16x3 0,11 > gpurun_out/prof_fea.log 2>&1 || exit 1
