#!/bin/bash
# GPU suite (parity log) then per-config bench lines without the CPU baseline.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
sha256sum 140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd/libextdm_hip.so | cut -c1-16
bash scripts_gpu/run_tests.sh || exit $?
for c in ${CONFIGS:-kth cityscapes ucf}; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > gpurun_out/r05_bench_$c.json 2> gpurun_out/r05_bench_$c.err
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05_bench_$c.err; exit $rc; }
  tail -1 gpurun_out/r05_bench_$c.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; print(d['config']['bench_config'], d['value'], 'frames/s', d['ms_per_step'], 'ms/step', 'lead', r.get('kernel', '')[:70], r.get('frac'))"
done
