# wave-specialised staging (EXTDM_X3_WS=1): parity, interleaved layer A/B, whole-step A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
EXTDM_X3_WS=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_precision.py -k "unet_forward_vs_reference_golden or batch_independence or graph_equals or ddpm10_chain or variant_unet or scales" > gpurun_out/ws_tests.log 2>&1 || { tail -30 gpurun_out/ws_tests.log; exit 1; }
for rep in 1 2; do
  for arm in 0 1; do
    echo "== WS=$arm"; EXTDM_X3_WS=$arm timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 0,1,5,2,11 2>&1 | grep -v amdgpu || exit 1
  done
done
S=20 AB="EXTDM_X3_WS=1" bash scripts_gpu/ab_step.sh || exit 1
