#!/bin/bash
# DDIM-20 kernel stats of each non-BAIR BASELINE workload at its bench batch (one generation), to
# name each config's dominant kernel: gpurun_out/cfgprof_<config>/ + top-kernel summary; then the
# level-0 attention layer timings of each config (layers 6, 7).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05}
for c in ${CONFIGS:-kth cityscapes ucf smmnist}; do
  rm -rf gpurun_out/cfgprof_$c
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/cfgprof_$c -o run --output-format csv -- python bench.py --config $c --sampling-steps 20 --warmup 0 --no-cpu-baseline --no-roofline > gpurun_out/cfgprof_$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/cfgprof_$c.log; exit $rc; }
  f=$(find gpurun_out/cfgprof_$c -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/${TAG}_cfgprof_${c}_kernel_stats.csv
  python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:10]:
    print(f"  {100*float(r['TotalDurationNs'])/tot:5.1f}%  n={r['Calls']:>6}  avg={float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:110]}")
PY
  find gpurun_out/cfgprof_$c -name "*kernel_trace.csv" -delete
done
for c in kth cityscapes ucf; do timeout -k 10 120 python scripts_gpu/layers_cfg.py $c 6,7 || exit 1; done
