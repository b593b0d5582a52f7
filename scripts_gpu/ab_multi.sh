#!/bin/bash
# Whole-step comparison over several settings: bench.py at a short DDIM schedule per arm,
# arms from $ARMS (space-separated; "-" = no setting, else VAR=VALUE[,VAR=VALUE]), REPS rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
S=${S:-20}; REPS=${REPS:-2}
for rep in $(seq 1 $REPS); do
  for arm in $ARMS; do
    if [ "$arm" = "-" ]; then envs=""; else envs="${arm//,/ }"; fi
    tag=$(echo "$arm" | tr -c 'A-Za-z0-9' '_')
    env $envs timeout -k 10 300 python bench.py --sampling-steps $S --steps $S --warmup 3 --no-cpu-baseline > gpurun_out/abm_$tag$rep.json 2> gpurun_out/abm_$tag$rep.err || { tail -5 gpurun_out/abm_$tag$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abm_$tag$rep.json').read().strip().splitlines()[-1]); print('$rep', '$arm', d['ms_per_step'], d['value'])"
  done
done
