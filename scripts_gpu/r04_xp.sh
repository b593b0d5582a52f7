# pre-split xpad: parity + precision suites, layers 9 / 10, then the per-config profiles
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_precision.py tests/test_gpu_e2e_configs.py tests/test_gpu_pw.py > gpurun_out/xp_tests.log 2>&1 || { tail -30 gpurun_out/xp_tests.log; exit 1; }
tail -2 gpurun_out/xp_tests.log
for rep in 1 2; do timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 9,10 2>&1 | grep -v amdgpu || exit 1; done
bash scripts_gpu/r04_cfgprof.sh
