# conv_x3 knock-out diagnostics: layer times of the in-tree lib, bufx, and the EXP variants
# (1 = no MFMA, 2 = no X loads, 4 = no output stores, 8 = no weight DMA); timings only
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for V in cur bufx exp1 exp2 exp4 exp8 bufx; do
  echo "== $V"
  if [ $V = cur ]; then unset EXTDM_LIB; else export EXTDM_LIB=_variants/$V/libextdm_hip.so; fi
  timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 ${LAYERS:-0,1,5,2,3,12,13} 2>&1 | grep -v amdgpu || exit 1
done
echo "== cur EXTDM_X3_BM1=128"; unset EXTDM_LIB
EXTDM_X3_BM1=128 timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 12,13 2>&1 | grep -v amdgpu || exit 1
echo "== cur EXTDM_X3_BM1=128 EXTDM_X3_NO_MFAST=1"
EXTDM_X3_BM1=128 EXTDM_X3_NO_MFAST=1 timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 12,13 2>&1 | grep -v amdgpu || exit 1
