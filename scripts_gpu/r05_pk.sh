#!/bin/bash
# Packed-fp32 attention VALU (and the cross kernel's), xpath at 128 px per wave (EXTDM_XP_NT=4), (v_pk_fma / v_pk_add / v_pk_mul in the softmax, LN prologue, V scale,
# tile epilogue; rcp for the normaliser) and the hoisted cond_fea branch: parity tests, then the
# attention layer times against the previous library (_variants/hoist, hoisted branch only),
# interleaved twice on one box, then the hoist A/B per config (EXTDM_NO_FEA_HOIST=1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_attn.py tests/test_gpu_e2e_configs.py tests/test_gpu_wrappers.py \
  tests/test_gpu_parity.py tests/test_gpu_precision.py tests/test_gpu_bf16_attn.py -x -q -s --timeout 600 \
  --timeout-method thread > gpurun_out/pk_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/pk_tests.log | tail -3; [ $rc -ne 0 ] && exit $rc
EXTDM_XP_NT=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "unet_forward" -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/pk_tests_nt4.log 2>&1
rc=$?; echo "NT=4 forward tests rc=$rc"; tail -1 gpurun_out/pk_tests_nt4.log; [ $rc -ne 0 ] && exit $rc
OLD=$PWD/_variants/hoist/libextdm_hip.so
for rep in 1 2; do
  for lib in old new; do
    if [ $lib = old ]; then L="EXTDM_LIB=$OLD"; else L=""; fi
    env $L timeout -k 10 120 python scripts_gpu/layers.py 128 20 f16x3 6,7,8,9 | sed "s/^/$lib /" || exit 1
    [ $lib = new ] && { EXTDM_XP_NT=4 timeout -k 10 120 python scripts_gpu/layers.py 128 20 f16x3 9 | sed "s/^/new-NT4 /" || exit 1; }
    for c in kth cityscapes ucf smmnist; do
      env $L timeout -k 10 120 python scripts_gpu/layers_cfg.py $c 6,7 | sed "s/^/$lib /" || exit 1
    done
  done
done
CONFIGS="ucf smmnist kth cityscapes" bash scripts_gpu/r05_hoist_ab.sh
