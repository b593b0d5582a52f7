# 1x1 256-row convs: 256 x 256 tiles where they fill the chip (x3_bn256) against 256 x 128
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
echo "== default"; timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 13 2>&1 | grep -v amdgpu || exit 1
echo "== BN1=128"; EXTDM_X3_BN1=128 timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 13 2>&1 | grep -v amdgpu || exit 1
ARMS="- EXTDM_X3_BN1=128" REPS=2 bash scripts_gpu/ab_multi.sh || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_pw.py > gpurun_out/bn1_tests.log 2>&1; rc=$?; tail -5 gpurun_out/bn1_tests.log; exit $rc
