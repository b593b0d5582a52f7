#!/bin/bash
# tests for the current tree, then conv_x3 pipelining A/B (layers) and conv_gemm A/B (kernel stats)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_precision.py tests/test_gpu_bf16_attn.py tests/test_gpu_metrics.py -x -q -s --timeout 400 --timeout-method thread > gpurun_out/batch_tests.log 2>&1
rc=$?; grep -E "bf16_attn max|passed|failed|Error" gpurun_out/batch_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
VARIANT=_variants/nopipe/libextdm_hip.so LAYERS=1,5,2,4 bash scripts_gpu/lib_ab.sh > gpurun_out/pipe_ab.log 2>&1 || exit 1
cat gpurun_out/pipe_ab.log
AB="EXTDM_LIB=_variants/gemmold/libextdm_hip.so" bash scripts_gpu/ab_prof.sh
