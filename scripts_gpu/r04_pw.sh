# register-resident-weight 1x1 (pw_x3): parity suites, layer 12 A/B, whole-step A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_precision.py tests/test_gpu_e2e_configs.py > gpurun_out/pw_tests.log 2>&1 || { tail -30 gpurun_out/pw_tests.log; exit 1; }
tail -3 gpurun_out/pw_tests.log
for rep in 1 2; do
  for arm in 0 1; do
    echo "== NO_PW=$arm"; EXTDM_NO_PW=$arm timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 12 2>&1 | grep -v amdgpu || exit 1
  done
done
ARMS="- EXTDM_NO_PW=1" bash scripts_gpu/ab_multi.sh || exit 1
