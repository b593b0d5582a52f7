# parity subset (+ DDPM-1000 chain, heads-6 core), layer 0 / 11 timings, kernel trace, SQ counter passes of layers 0 / 1
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_attn.py -k "unet_forward_vs_reference_golden or batch_independence or ddpm1000 or heads6" > gpurun_out/r04_fea_tests.log 2>&1 || exit 1
timeout -k 10 300 python scripts_gpu/layers.py 64 20 f16x3 0,11,1 > gpurun_out/r04_fea_layers.log 2>&1 || exit 1
rm -rf gpurun_out/prof_fea
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_fea -o run -- python scripts_gpu/layers.py 64 5 f16x3 0,11 > gpurun_out/prof_fea.log 2>&1 || exit 1
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_MFMA"; do
  rm -rf gpurun_out/sq5_p$i
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/sq5_p$i -o run --output-format csv -- python scripts_gpu/layers.py 64 3 f16x3 0,1 > gpurun_out/sq5_p$i.log 2>&1 || exit 1
  i=$((i+1))
done
