#!/bin/bash
# Per-GPU clip batch sweep of the BAIR bench (DDIM-20 generation, no CPU baseline): frames/s.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for B in ${BATCHES:-64 128 192 256}; do
  timeout -k 10 300 python bench.py --batch $B --sampling-steps 20 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/r05_batch_$B.json 2> gpurun_out/r05_batch_$B.err || { tail -3 gpurun_out/r05_batch_$B.err; exit 1; }
  tail -1 gpurun_out/r05_batch_$B.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B', d['value'], 'frames/s', d['ms_per_step'], 'ms/step', d['config']['workspace_gb'], 'GB')"
done
