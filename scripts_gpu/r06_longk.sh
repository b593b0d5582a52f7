#!/bin/bash
# KTH's long-K Tmodulators split-K by the per-sample cost model (_variants/split) against the shipped
# library: KTH parity / batch-invariance tests on the variant, layer 13 interleaved, whole KTH
# DDIM-20 steps interleaved, then BAIR / SMMNIST steps on both (their convs are unchanged).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
VL=$PWD/_variants/${VAR:-split}/libextdm_hip.so
EXTDM_LIB=$VL timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e_configs.py tests/test_gpu_parity.py -k "kth" -x -v --timeout 300 --timeout-method thread > gpurun_out/longk_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|ERROR|err" gpurun_out/longk_tests.log | tail -12; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 120 python -u scripts_gpu/layers_cfg.py kth 13 2>&1 | grep layer | sed "s/^/A$rep /" || exit 1
  EXTDM_LIB=$VL timeout -k 10 120 python -u scripts_gpu/layers_cfg.py kth 13 2>&1 | grep layer | sed "s/^/B$rep /" || exit 1
done
for c in ${CONFIGS:-kth bair}; do
  for rep in 1 2; do
    for arm in A B; do
      if [ $arm = A ]; then envs="X=0"; else envs="EXTDM_LIB=$VL"; fi
      env $envs timeout -k 10 300 python bench.py --config $c --sampling-steps 20 --steps 20 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/longk_${c}_$arm$rep.json 2> gpurun_out/longk_${c}_$arm$rep.err || { tail -5 gpurun_out/longk_${c}_$arm$rep.err; exit 1; }
      python -c "import json; d=json.loads(open('gpurun_out/longk_${c}_$arm$rep.json').read().strip().splitlines()[-1]); print('$c', '$arm$rep', d['ms_per_step'], d['value'])"
    done
  done
done
