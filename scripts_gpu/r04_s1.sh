# round-4 session-1 check: GPU parity subset, layer timings, an eager forward trace (B = 64),
# whole-step A/B of the phase-composed fea conv and of split-K / MFAST on the 1x1 convs, SQ passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_attn.py -k "unet_forward_vs_reference_golden or batch_independence or ddpm1000 or heads6 or range_guard or graph_equals" > gpurun_out/s1_tests.log 2>&1 || exit 1
timeout -k 10 300 python scripts_gpu/layers.py 64 20 f16x3 0,11,1,5 > gpurun_out/s1_layers.log 2>&1 || exit 1
rm -rf gpurun_out/s1_trace
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s1_trace -o run --output-format csv -- python scripts_gpu/forward_trace.py 64 > gpurun_out/s1_trace.log 2>&1 || exit 1
f=$(find gpurun_out/s1_trace -name "*kernel_trace.csv" | head -1); python scripts_gpu/trace_order.py $f 3 > gpurun_out/s1_forward.txt || exit 1
S=20 AB="EXTDM_NO_FEA_PHASE=1" bash scripts_gpu/ab_step.sh > gpurun_out/s1_ab_fea.log 2>&1 || exit 1
S=20 AB="EXTDM_X3_NO_MFAST=1 EXTDM_X3_SPLIT256=0" bash scripts_gpu/ab_step.sh > gpurun_out/s1_ab_1x1.log 2>&1 || exit 1
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_MFMA"; do
  rm -rf gpurun_out/sq5_p$i
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/sq5_p$i -o run --output-format csv -- python scripts_gpu/layers.py 64 3 f16x3 0,1 > gpurun_out/sq5_p$i.log 2>&1 || exit 1
  i=$((i+1))
done
