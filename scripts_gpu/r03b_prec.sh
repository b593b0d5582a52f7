#!/bin/bash
# precision diagnosis at small scale + the attention / precision test files + attention A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03b}
BASE=${BASE:-_variants/base/libextdm_hip.so}
timeout -k 10 600 python scripts_gpu/prec_diag.py 1e-3 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_attn.py tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_prec.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${TAG}_prec.log | tail -8; grep -E "s=|vs fp64" gpurun_out/${TAG}_prec.log | tail -6
[ $rc -gt 1 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 || exit 1
  EXTDM_LIB=$BASE timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 || exit 1
done
