#!/bin/bash
# A/B of whole DDIM-$S steps of bench.py --config c (CONFIGS) with the environment setting $AB
# (arm B) against none (arm A), interleaved twice; optional $TESTS first.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
S=${S:-20}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/abe_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/abe_tests.log; [ $rc -ne 0 ] && exit $rc
fi
for c in ${CONFIGS:-cityscapes}; do
  for rep in 1 2; do
    for arm in A B; do
      if [ $arm = A ]; then envs="X=0"; else envs="$AB"; fi
      env $envs timeout -k 10 300 python bench.py --config $c --sampling-steps $S --steps $S --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/abe_${c}_$arm$rep.json 2> gpurun_out/abe_${c}_$arm$rep.err || { tail -5 gpurun_out/abe_${c}_$arm$rep.err; exit 1; }
      python -c "import json; d=json.loads(open('gpurun_out/abe_${c}_$arm$rep.json').read().strip().splitlines()[-1]); print('$c', '$arm$rep', '$envs', d['ms_per_step'], d['value'])"
    done
  done
done
