#!/bin/bash
# One bench line per BASELINE workload (bench.py --config; each config's own lead kernel heads its
# roofline) with the CPU baseline, each under its own limit: gpurun_out/${TAG}_bench_<config>.json.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05}
( while sleep 45; do echo "heartbeat $(date +%T)" >> gpurun_out/${TAG}_bench_heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
for c in ${CONFIGS:-bair smmnist kth ucf cityscapes}; do
  timeout -k 10 ${TL:-700} python -u bench.py --config $c ${EXTRA} > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err
  rc=$?; echo "$c rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_bench_$c.err; exit $rc; }
  tail -1 gpurun_out/${TAG}_bench_$c.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; print(d['config']['bench_config'], d['value'], 'frames/s', d['ms_per_step'], 'ms/step', 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'lead', r.get('kernel', '')[:60], r.get('frac'), 'traffic', r.get('traffic'))"
done
