#!/bin/bash
# Round 5: the fused 64-token-window STW route (stw64_x3.hip): its attention-layer tests, the ada /
# ada_u22 goldens, then layer-6 timings per config with the route on and off.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_attn.py -k window64 > gpurun_out/r05_w64_tests.log 2>&1
rc=$?; echo "w64 tests rc=$rc"; grep -E "max\|err|PASS|FAIL|Error" gpurun_out/r05_w64_tests.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "variant" tests/test_gpu_bf16_attn.py > gpurun_out/r05_w64_goldens.log 2>&1
rc=$?; echo "goldens rc=$rc"; tail -5 gpurun_out/r05_w64_goldens.log; [ $rc -ne 0 ] && exit $rc
for c in kth cityscapes ucf; do
  timeout -k 10 120 python scripts_gpu/layers_cfg.py $c 6,7 || exit 1
  EXTDM_NO_STW64=1 timeout -k 10 120 python scripts_gpu/layers_cfg.py $c 6 || exit 1
done
