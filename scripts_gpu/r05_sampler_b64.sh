#!/bin/bash
# The sampler step at the reference's 64 clips per GPU on the shipped build: rocprofv3 kernel stats of
# a DDIM-20 BAIR generation at --batch 64 -> gpurun_out/r05_bair_b64_ddim20_kernel_stats.csv.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/prof_b64
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b64 -o run --output-format csv -- python bench.py --batch 64 --sampling-steps 20 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/prof_b64.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -3 gpurun_out/prof_b64.log; exit $rc; }
cp "$(find gpurun_out/prof_b64 -name '*kernel_stats.csv' | head -1)" gpurun_out/r05_bair_b64_ddim20_kernel_stats.csv
find gpurun_out/prof_b64 -name "*kernel_trace.csv" -delete
grep -E "sampler|radix" gpurun_out/r05_bair_b64_ddim20_kernel_stats.csv | cut -d, -f2-5
