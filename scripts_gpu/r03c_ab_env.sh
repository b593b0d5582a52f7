#!/bin/bash
# Interleaved whole-step A/B over environment settings: arm 0 = no setting, then each
# ";"-separated entry of $ARMS (e.g. ARMS="EXTDM_X3_W128=8;EXTDM_X3_SPLIT4=128,256"),
# DDPM-$S at B = $B, $R rounds; optional $TESTS pytest selection first.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
S=${S:-50}; B=${B:-64}; R=${R:-2}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
fi
IFS=';' read -ra AR <<< "$ARMS"
for i in $(seq $R); do
  for k in $(seq 0 ${#AR[@]}); do
    envs=""; [ $k -gt 0 ] && envs="${AR[$((k-1))]}"
    env $envs timeout -k 10 300 python bench.py --sampling-steps $S --steps $S --warmup 5 --batch $B --no-cpu-baseline --no-roofline > gpurun_out/abe_$k.json 2> gpurun_out/abe_$k.err || { tail -5 gpurun_out/abe_$k.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abe_$k.json').read().strip().splitlines()[-1]); print('arm $k', '$envs', $i, 'ms/step', d['ms_per_step'])"
  done
done
