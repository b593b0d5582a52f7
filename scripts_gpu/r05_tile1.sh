#!/bin/bash
# Temporal attention's LDS tile path extended from D = 16 to any D <= 32 (16 or 32 frame slots per
# pixel; KTH 30, SMMNIST 19, Cityscapes 7 frames): parity tests, then layer 7 of each config against
# the previous library (_variants/base, per-lane loads for D != 16), interleaved twice on one box,
# then whole DDIM-20 steps of kth / smmnist / cityscapes against it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_attn.py tests/test_gpu_e2e_configs.py tests/test_gpu_wrappers.py -x -q -s \
  --timeout 600 --timeout-method thread > gpurun_out/tile1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error|D=" gpurun_out/tile1_tests.log | tail -6; [ $rc -ne 0 ] && exit $rc
OLD=$PWD/_variants/base/libextdm_hip.so
for rep in 1 2; do
  for lib in old new; do
    if [ $lib = old ]; then L="EXTDM_LIB=$OLD"; else L=""; fi
    for c in kth smmnist cityscapes; do
      env $L timeout -k 10 120 python scripts_gpu/layers_cfg.py $c 7 | sed "s/^/$lib /" || exit 1
      env $L timeout -k 10 300 python bench.py --config $c --sampling-steps 20 --warmup 1 --no-cpu-baseline --no-roofline \
        > gpurun_out/tile1_${c}_$lib$rep.json 2> gpurun_out/tile1_${c}_$lib$rep.err || { tail -5 gpurun_out/tile1_${c}_$lib$rep.err; exit 1; }
      python -c "import json; d=json.loads(open('gpurun_out/tile1_${c}_$lib$rep.json').read().strip().splitlines()[-1]); print('$lib$rep $c step', d['ms_per_step'], d['value'])"
    done
  done
done
