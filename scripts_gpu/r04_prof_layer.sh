# kernel trace of bench layers ($1 = comma list) at B = 64: per-kernel stats under gpurun_out/prof_layer/
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_layer -o run --output-format csv -- python scripts_gpu/layers.py 64 5 f16x3 "$1" > gpurun_out/prof_layer.log 2>&1 || exit 1
find gpurun_out/prof_layer -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/prof_layer_stats.csv
