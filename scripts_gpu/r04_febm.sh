# phase conv with 128-row two-phase tiles (EXTDM_FEA_BM=128): parity, layers 0 / 11, whole-step A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
EXTDM_FEA_BM=128 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_e2e_configs.py -k "unet_forward_vs_reference or batch_independence or graph_equals or bair or ddpm10" > gpurun_out/febm_tests.log 2>&1 || { tail -30 gpurun_out/febm_tests.log; exit 1; }
tail -2 gpurun_out/febm_tests.log
for rep in 1 2; do for bm in 64 128; do
  echo "== FEA_BM=$bm"; EXTDM_FEA_BM=$bm timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 0,11 2>&1 | grep -v amdgpu || exit 1
done; done
ARMS="- EXTDM_FEA_BM=128" bash scripts_gpu/ab_multi.sh
