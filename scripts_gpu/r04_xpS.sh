cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do for V in cur xpS; do
  unset EXTDM_LIB; [ $V = cur ] || export EXTDM_LIB=_variants/$V/libextdm_hip.so
  echo "== $V"; timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 9,10,0 2>&1 | grep -v amdgpu || exit 1
done; done
