# pw_x3 variants: register staging (in-tree), load-first (pwR2), LDS-DMA ring (pwD), conv_x3 (nopw)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 240 --timeout-method thread tests/test_gpu_pw.py 2>&1 | grep -v amdgpu | tail -3
for rep in 1 2; do
for V in cur pwR2 pwD nopw; do
  echo "== $V"
  unset EXTDM_LIB EXTDM_NO_PW
  case $V in cur) ;; nopw) export EXTDM_NO_PW=1;; *) export EXTDM_LIB=_variants/$V/libextdm_hip.so;; esac
  timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 12 2>&1 | grep -v amdgpu || exit 1
done
done
