#!/bin/bash
# GPU suite with the parity log (run_tests.sh), then A/B of KTH's C = 256 dim-16 windows on the f16x3
# attention core (default) vs the fp32 fused kernel (EXTDM_NO_X3_CORE=1): whole DDIM-20 steps,
# interleaved twice on one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts_gpu/run_tests.sh || exit 1
for rep in 1 2; do
  for arm in A B; do
    if [ $arm = A ]; then envs=""; else envs="EXTDM_NO_X3_CORE=1"; fi
    env $envs timeout -k 10 300 python bench.py --config kth --sampling-steps 20 --warmup 1 --no-cpu-baseline --no-roofline \
      > gpurun_out/core16_$arm$rep.json 2> gpurun_out/core16_$arm$rep.err || { tail -5 gpurun_out/core16_$arm$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/core16_$arm$rep.json').read().strip().splitlines()[-1]); print('kth $arm$rep', '$envs', d['ms_per_step'], d['value'])"
  done
done
