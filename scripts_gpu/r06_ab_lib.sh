#!/bin/bash
# A/B of whole sampler steps between two libraries: arm A = $LIBA (default _variants/noslp: the round-6
# base build), arm B = the in-tree library; bench.py --config c at DDIM-$S, per config in $CONFIGS,
# interleaved twice. Optional $TESTS first (pytest, stops on failure).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
S=${S:-20}
LIBA=${LIBA:-_variants/noslp/libextdm_hip.so}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
fi
for c in ${CONFIGS:-ucf cityscapes smmnist}; do
  for rep in 1 2; do
    for arm in A B; do
      if [ $arm = A ]; then envs="EXTDM_LIB=$PWD/$LIBA"; else envs="X=0"; fi
      env $envs timeout -k 10 300 python bench.py --config $c --sampling-steps $S --steps $S --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/ab_${c}_$arm$rep.json 2> gpurun_out/ab_${c}_$arm$rep.err || { tail -5 gpurun_out/ab_${c}_$arm$rep.err; exit 1; }
      python -c "import json; d=json.loads(open('gpurun_out/ab_${c}_$arm$rep.json').read().strip().splitlines()[-1]); print('$c', '$arm$rep', d['ms_per_step'], d['value'])"
    done
  done
done
