#!/bin/bash
# Closing evidence, part 2: one bench line per non-BAIR BASELINE workload (bench.py --config, with
# its CPU baseline and its own lead kernel's roofline) -> gpurun_out/r05_bench_<config>.json.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in ucf cityscapes smmnist kth; do
  timeout -k 10 500 python -u bench.py --config $c > gpurun_out/r05_bench_$c.json 2> gpurun_out/r05_bench_$c.err
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05_bench_$c.err; exit $rc; }
  tail -1 gpurun_out/r05_bench_$c.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; print(d['config']['bench_config'], d['value'], d['ms_per_step'], (d.get('cpu_baseline') or {}).get('value'), r.get('kernel', '')[:50], r.get('frac'), r.get('traffic'))"
done
