# conflict-free lane order for 16-wide images (EXTDM_X3_ROT): parity, layers, whole-step A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_precision.py tests/test_gpu_pw.py > gpurun_out/rot_tests.log 2>&1 || { tail -30 gpurun_out/rot_tests.log; exit 1; }
tail -2 gpurun_out/rot_tests.log
for rep in 1 2; do for V in cur norot; do
  unset EXTDM_LIB; [ $V = cur ] || export EXTDM_LIB=_variants/$V/libextdm_hip.so
  echo "== $V"; timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 0,1,5,2,3 2>&1 | grep -v amdgpu || exit 1
done; done
unset EXTDM_LIB
ARMS="- EXTDM_LIB=_variants/norot/libextdm_hip.so" bash scripts_gpu/ab_multi.sh
