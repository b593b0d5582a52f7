#!/bin/bash
# Round 3 session 2: smoke + the full GPU suite (verbose, per-test timing), the attention
# layer A/B timing against $BASE, then the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03b}
BASE=${BASE:-_variants/base/libextdm_hip.so}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --durations=15 --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/${TAG}_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}_suite.log | grep -E "FAILED|ERROR|passed|failed" | tail -15
grep -E "s=|vs fp64" gpurun_out/${TAG}_suite.log | tail -6
[ $rc -gt 1 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 || exit 1
  EXTDM_LIB=$BASE timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 || exit 1
done
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().split('\n')[-1]); r=d['roofline']
print(d['value'], d['ms_per_step'], r['kernel'][:40], r['launch_ms'], r['frac'], [(o['kernel'][:30], o['launch_ms'], o['frac']) for o in r['others']])"
exit $rc
