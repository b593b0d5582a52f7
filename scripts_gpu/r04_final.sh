#!/bin/bash
# Round-4 closing measurement on the in-tree library: PMC FETCH / WRITE passes of every bench
# roofline kernel into profiles/ (bench.py reads them: same library sha, same template), smoke,
# the default bench line, and the DDIM-20 kernel stats + per-launch groups (r03_measure.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04}
# heartbeat: the profiled / CPU-baseline phases print nothing for minutes (gpurun's silence guard)
( while sleep 45; do echo "heartbeat $(date +%T)" >> gpurun_out/${TAG}_heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
if [ -z "$SKIP_PMC" ]; then
  B=64 bash scripts_gpu/pmc_layers.sh || exit 1
  cp gpurun_out/pmc_layer*.json profiles/ || exit 1
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/${TAG}_bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_bench.err; exit $rc; }
TAG=$TAG SKIP_PMC=1 bash scripts_gpu/r03_measure.sh
