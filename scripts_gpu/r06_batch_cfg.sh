#!/bin/bash
# r06: per-clip step cost of the small-batch BASELINE workloads at larger per-GPU batches
# (bench.py --config c --batch B at DDIM-20, one generation), to choose each config's bench batch
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cb in ${CB:-cityscapes:8 cityscapes:16 cityscapes:32 ucf:4 ucf:8 ucf:16 kth:16 kth:32}; do
  c=${cb%%:*}; b=${cb##*:}
  timeout -k 10 300 python bench.py --config $c --batch $b --sampling-steps 20 --steps 20 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/bcfg_${c}_$b.json 2> gpurun_out/bcfg_${c}_$b.err || { echo "$c $b failed"; tail -3 gpurun_out/bcfg_${c}_$b.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bcfg_${c}_$b.json').read().strip().splitlines()[-1]); print('$c', $b, 'ms/step', d['ms_per_step'], 'ms/clip-step', round(d['ms_per_step']/$b, 4), 'frames/s', d['value'], 'ws GB', d['config']['workspace_gb'])"
done
