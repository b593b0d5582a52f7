#!/bin/bash
# One extra bench arm with an environment switch: ENVSET="NAME=value" ($S steps, B = $B).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
S=${S:-50}; B=${B:-64}
env $ENVSET timeout -k 10 300 python bench.py --sampling-steps $S --steps $S --warmup 5 --batch $B --no-cpu-baseline > gpurun_out/envarm.json 2> gpurun_out/envarm.err || { tail -5 gpurun_out/envarm.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/envarm.json').read().strip().splitlines()[-1]); print('$ENVSET', 'ms/step', d['ms_per_step'], 'layers', d['roofline']['launch_ms'], [o['launch_ms'] for o in d['roofline']['others']])"
