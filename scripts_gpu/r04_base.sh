cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 || exit 1
timeout -k 10 300 python scripts_gpu/layers.py 64 20 f16x3 0,1,5,6,7,8,9,10 > gpurun_out/r04_layers_base.log 2>&1 || exit 1
