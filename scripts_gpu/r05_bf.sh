#!/bin/bash
# Round 5: the bf16 attention core inside the fused kernels (BF16_ATTN): attention-layer and
# forward tests, UCF / Cityscapes e2e goldens, then layer timings for UCF and Cityscapes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_attn.py tests/test_gpu_bf16_attn.py tests/test_gpu_e2e_configs.py > gpurun_out/r05_bf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "max\|err|passed|failed|Error" gpurun_out/r05_bf_tests.log | tail -40; [ $rc -ne 0 ] && exit $rc
for c in ucf cityscapes kth; do
  timeout -k 10 120 python scripts_gpu/layers_cfg.py $c 6,7 || exit 1
done
