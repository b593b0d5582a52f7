#!/bin/bash
# A/B of bench layers ($LAYERS, default the cross-attention core 8) between the in-tree
# library and _variants/$VAR, then the GPU tests $TESTS on the variant (EXTDM_LIB).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
VAR=${VAR:-cross}; LAYERS=${LAYERS:-8}
for rep in 1 2; do
  for arm in cur $VAR; do
    if [ $arm = cur ]; then unset EXTDM_LIB; else export EXTDM_LIB=_variants/$arm/libextdm_hip.so; fi
    echo "== $arm"; timeout -k 10 180 python scripts_gpu/layers.py 64 20 f16x3 $LAYERS || exit 1
  done
done
unset EXTDM_LIB
[ -z "$TESTS" ] && exit 0
EXTDM_LIB=_variants/$VAR/libextdm_hip.so timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/ab_${VAR}_tests.log 2>&1
rc=$?; echo "variant tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/ab_${VAR}_tests.log | tail -12; exit $rc
