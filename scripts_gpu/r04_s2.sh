# session-2 check: parity subset incl. sharding invariance, edge-kernel timings, forward trace, 1x1 A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "unet_forward_vs_reference_golden or batch_independence or graph_equals or ddpm10_chain" > gpurun_out/s2_tests.log 2>&1 || exit 1
timeout -k 10 300 python scripts_gpu/layers.py 64 20 f16x3 0,11 > gpurun_out/s2_layers.log 2>&1 || exit 1
rm -rf gpurun_out/s2_trace
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s2_trace -o run --output-format csv -- python scripts_gpu/forward_trace.py 64 > gpurun_out/s2_trace.log 2>&1 || exit 1
f=$(find gpurun_out/s2_trace -name "*kernel_trace.csv" | head -1); python scripts_gpu/trace_order.py $f 3 > gpurun_out/s2_forward.txt || exit 1
S=20 AB="EXTDM_X3_NO_MFAST=1 EXTDM_X3_SPLIT256=0" bash scripts_gpu/ab_step.sh > gpurun_out/s2_ab_1x1.log 2>&1 || exit 1
# X-tile layout A/B (in-tree swizzled vs _variants/lin): parity of the variant, then layer timings interleaved
for V in linbufx bufx lin; do
  EXTDM_LIB=_variants/$V/libextdm_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "unet_forward_vs_reference_golden or batch_independence" > gpurun_out/s2_${V}_tests.log 2>&1 || exit 1
  VARIANT=_variants/$V/libextdm_hip.so LAYERS=0,1,2,3,4 bash scripts_gpu/lib_ab.sh > gpurun_out/s2_${V}_ab.log 2>&1 || exit 1
done
