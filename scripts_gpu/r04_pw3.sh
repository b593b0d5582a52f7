cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for V in cur pwR; do
  unset EXTDM_LIB; [ $V = cur ] || export EXTDM_LIB=_variants/$V/libextdm_hip.so
  echo "== $V"; timeout -k 10 300 python -u -m pytest -x -s -q --timeout 240 --timeout-method thread tests/test_gpu_pw.py 2>&1 | grep -v amdgpu | tail -4 || exit 1
done
