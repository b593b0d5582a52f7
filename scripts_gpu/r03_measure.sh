#!/bin/bash
# Round-3 measurement set on the HEAD library: the PMC FETCH / WRITE passes of every bench
# roofline kernel (pmc_layers.sh -> gpurun_out/pmc_layer<id>.json), then one rocprofv3
# kernel-trace of a DDIM-20 bench generation with the roofline timing, summarised as
# --stats plus per-launch groups (kernel_launches.py) of the attention and conv kernels.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03}
if [ -z "$SKIP_PMC" ]; then B=${B:-64} bash scripts_gpu/pmc_layers.sh || exit 1; fi
rm -rf gpurun_out/prof_$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --sampling-steps 20 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_$TAG.log; [ $rc -ne 0 ] && exit $rc
for p in attn_x3_kernel cross_attn_x3p conv_x3_kernel; do python scripts_gpu/kernel_launches.py gpurun_out/prof_$TAG $p; done > gpurun_out/prof_${TAG}_launches.txt
find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -delete
cat gpurun_out/prof_${TAG}_launches.txt | grep -E "attn|cross" 
