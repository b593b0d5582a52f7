#!/bin/bash
# Closing measurement on the in-tree library (TAG, default r05), each step under its own limit:
#   1. PMC FETCH / WRITE passes of every BAIR roofline kernel and of each other config's lead
#      (pmc_layers.sh -> gpurun_out/pmc_layer<id>.json, pmc_<config>_layer<id>.json; copied to
#      profiles/ by the caller: bench.py reports traffic only from PMC files of the same library sha)
#   2. one rocprofv3 kernel trace of a DDIM-20 BAIR generation (same kernels and shapes as DDPM-1000,
#      whose 2000 graph replays crash the profiler) -> ${TAG}_bair_ddim20_kernel_stats.csv + the
#      per-launch groups of the attention and conv kernels (kernel_launches.py)
# SKIP_PMC=1 skips 1; SKIP_PROF=1 skips 2.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05}
( while sleep 45; do echo "heartbeat $(date +%T)" >> gpurun_out/${TAG}_heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
sha256sum 140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd/libextdm_hip.so | cut -c1-16
if [ -z "$SKIP_PMC" ]; then
  CONFIG=bair bash scripts_gpu/pmc_layers.sh || exit 1
  for c in kth cityscapes ucf smmnist; do CONFIG=$c LAYERS=6 bash scripts_gpu/pmc_layers.sh || exit 1; done
fi
if [ -z "$SKIP_PROF" ]; then
  rm -rf gpurun_out/prof_$TAG
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --sampling-steps 20 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_$TAG.log; [ $rc -ne 0 ] && exit $rc
  cp "$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)" gpurun_out/${TAG}_bair_ddim20_kernel_stats.csv
  for p in attn_x3_kernel cross_attn_x3p conv_x3_kernel xpath_x3 sampler; do python scripts_gpu/kernel_launches.py gpurun_out/prof_$TAG $p; done > gpurun_out/${TAG}_bair_ddim20_launches.txt
  find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -delete
fi
