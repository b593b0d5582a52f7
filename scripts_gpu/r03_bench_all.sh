#!/bin/bash
# One bench line per BASELINE workload (bench.py --config; BAIR last = the driver's default
# command), each under its own time limit; results in gpurun_out/r03_bench_<config>.json.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in ${CONFIGS:-smmnist kth ucf cityscapes bair}; do
  timeout -k 10 ${TL:-600} python bench.py --config $c > gpurun_out/r03_bench_$c.json 2> gpurun_out/r03_bench_$c.err
  rc=$?; echo "$c rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/r03_bench_$c.err; exit $rc; }
  tail -1 gpurun_out/r03_bench_$c.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['bench_config'], d['value'], 'frames/s', d['ms_per_step'], 'ms/step', 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'roofline', (d.get('roofline') or {}).get('frac'))"
done
