#!/bin/bash
# One bench line per BASELINE workload (bench.py --config; each config's own lead kernel heads
# its roofline), each under its own time limit; results in gpurun_out/r04_bench_<config>.json.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
( while sleep 45; do echo "heartbeat $(date +%T)" >> gpurun_out/r04_bench_all_heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
for c in ${CONFIGS:-smmnist kth ucf cityscapes}; do
  timeout -k 10 ${TL:-600} python bench.py --config $c > gpurun_out/r04_bench_$c.json 2> gpurun_out/r04_bench_$c.err
  rc=$?; echo "$c rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/r04_bench_$c.err; exit $rc; }
  tail -1 gpurun_out/r04_bench_$c.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; print(d['config']['bench_config'], d['value'], 'frames/s', d['ms_per_step'], 'ms/step', 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'lead', r.get('kernel', '')[:60], r.get('frac'))"
done
