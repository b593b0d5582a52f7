#!/bin/bash
# layer timings, alternating the in-tree library (A) and $VARIANT (B), twice each
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=${VARIANT:-_variants/nopipe/libextdm_hip.so}
for rep in 1 2; do
  echo "A$rep"; timeout -k 10 120 python scripts_gpu/layers.py 64 20 f16x3 ${LAYERS:-1,5,2,3,4} || exit 1
  echo "B$rep"; EXTDM_LIB=$V timeout -k 10 120 python scripts_gpu/layers.py 64 20 f16x3 ${LAYERS:-1,5,2,3,4} || exit 1
done
