#!/bin/bash
# Round 3 session 4: smoke + the full GPU suite, the default bench line, then the DDIM-20
# kernel stats of the same library (r03_measure.sh, PMC passes skipped unless PMC=1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03c}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}_smoke.log; [ $rc -ne 0 ] && exit $rc
if [ -z "$NOSUITE" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --durations=15 --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/${TAG}_suite.log 2>&1
  rc=$?; echo "suite rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${TAG}_suite.log | tail -15
  [ $rc -gt 1 ] && exit $rc
fi
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/${TAG}_bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_bench.err; exit $rc; }
if [ -n "$PMC" ]; then TAG=$TAG bash scripts_gpu/r03_measure.sh; else TAG=$TAG SKIP_PMC=1 bash scripts_gpu/r03_measure.sh; fi
