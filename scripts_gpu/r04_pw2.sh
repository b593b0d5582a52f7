# pw_x3 with the LDS-DMA raw ring + counted waits: bitwise test, parity, layer 12 variants, step A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pw.py tests/test_gpu_parity.py tests/test_gpu_e2e_configs.py > gpurun_out/pw2_tests.log 2>&1 || { tail -30 gpurun_out/pw2_tests.log; exit 1; }
tail -3 gpurun_out/pw2_tests.log
for rep in 1 2; do
for V in cur pwR pwS pwL nopw; do
  echo "== $V"
  unset EXTDM_LIB EXTDM_NO_PW
  case $V in cur) ;; nopw) export EXTDM_NO_PW=1;; *) export EXTDM_LIB=_variants/$V/libextdm_hip.so;; esac
  timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 12 2>&1 | grep -v amdgpu || exit 1
done
done
unset EXTDM_LIB EXTDM_NO_PW
ARMS="- EXTDM_NO_PW=1" bash scripts_gpu/ab_multi.sh || exit 1
