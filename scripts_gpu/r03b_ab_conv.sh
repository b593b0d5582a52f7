#!/bin/bash
# Conv layer A/B (bench_layer ids 1, 5, 0, 4 at B = 64, f16x3) in-tree vs $BASE, plus the
# in-tree x-branch gathers (9, 10), then the precision diagnosis at s = 1e-3
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
BASE=${BASE:-_variants/base/libextdm_hip.so}
for rep in 1 2; do
  timeout -k 10 180 python scripts_gpu/layers.py 64 20 f16x3 1,5,0,4,9,10 | sed 's/^/new  /' || exit 1
  EXTDM_LIB=$BASE timeout -k 10 180 python scripts_gpu/layers.py 64 20 f16x3 1,5,0,4 | sed 's/^/base /' || exit 1
done
[ -n "$NOPREC" ] && exit 0
timeout -k 10 600 python scripts_gpu/prec_diag.py 1e-3
