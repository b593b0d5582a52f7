#!/bin/bash
# A/B: init_conv's cond_fea branch hoisted into the cond cache (default) vs per step
# (EXTDM_NO_FEA_HOIST=1) for the non-BAIR workloads (DDIM-20, interleaved twice on one box).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in ${CONFIGS:-ucf smmnist kth cityscapes}; do
  for rep in 1 2; do
    for arm in A B; do
      if [ $arm = A ]; then envs=""; else envs="EXTDM_NO_FEA_HOIST=1"; fi
      env $envs timeout -k 10 300 python bench.py --config $c --sampling-steps 20 --warmup 1 --no-cpu-baseline --no-roofline \
        > gpurun_out/hoist_${c}_$arm$rep.json 2> gpurun_out/hoist_${c}_$arm$rep.err || { tail -5 gpurun_out/hoist_${c}_$arm$rep.err; exit 1; }
      python -c "import json; d=json.loads(open('gpurun_out/hoist_${c}_$arm$rep.json').read().strip().splitlines()[-1]); print('$c $arm$rep', '$envs', d['ms_per_step'], d['value'])"
    done
  done
done
