#!/bin/bash
# Interleaved A/B of whole-step time: the in-tree library ("cur") against each
# _variants/<name>/libextdm_hip.so in $LIBS, DDPM-$S at B = $B, $R rounds; optional
# $TESTS pytest selection first, $ATTN=1 adds the attention layer timings per arm.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
S=${S:-50}; B=${B:-64}; R=${R:-2}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
fi
for i in $(seq $R); do
  for arm in cur $LIBS; do
    if [ $arm = cur ]; then unset EXTDM_LIB; else export EXTDM_LIB=_variants/$arm/libextdm_hip.so; fi
    if [ -n "$ATTN" ]; then timeout -k 10 120 python scripts_gpu/attn_dbg.py $B > gpurun_out/ab_attn_$arm.log 2>&1 || exit $?; echo "$arm $(cat gpurun_out/ab_attn_$arm.log | grep dbg)"; fi
    timeout -k 10 300 python bench.py --sampling-steps $S --steps $S --warmup 5 --batch $B --no-cpu-baseline --no-roofline > gpurun_out/ab_$arm.json 2> gpurun_out/ab_$arm.err || { tail -5 gpurun_out/ab_$arm.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$arm.json').read().strip().splitlines()[-1]); print('$arm', '$i', 'ms/step', d['ms_per_step'])"
  done
done
