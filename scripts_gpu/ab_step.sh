#!/bin/bash
# A/B of whole sampler steps: bench.py at a short DDIM schedule, alternating the
# environment setting in $AB (e.g. AB="EXTDM_NO_GN_FUSE=1"), twice each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
S=${S:-50}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do
  for arm in A B; do
    if [ $arm = A ]; then envs=""; else envs="$AB"; fi
    env $envs timeout -k 10 300 python bench.py --sampling-steps $S --steps $S --warmup 3 --no-cpu-baseline > gpurun_out/ab_$arm$rep.json 2> gpurun_out/ab_$arm$rep.err || { tail -5 gpurun_out/ab_$arm$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$arm$rep.json').read().strip().splitlines()[-1]); print('$arm$rep', '$envs', d['ms_per_step'], d['value'])"
  done
done
