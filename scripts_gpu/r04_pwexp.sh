# pw_x3 diagnostics: layer 12 for the in-tree lib, the no-store / no-load variants, conv_x3 (NO_PW)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for V in cur pwS pwL nopw; do
  echo "== $V"
  unset EXTDM_LIB EXTDM_NO_PW
  case $V in cur) ;; nopw) export EXTDM_NO_PW=1;; *) export EXTDM_LIB=_variants/$V/libextdm_hip.so;; esac
  timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 12 2>&1 | grep -v amdgpu || exit 1
done
done
unset EXTDM_LIB EXTDM_NO_PW
LAYERS=12 TAG=pwsq bash scripts_gpu/r04_sq.sh && python scripts_gpu/sq_summary.py gpurun_out/pwsq_table.txt
