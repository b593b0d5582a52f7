#!/bin/bash
# Round-6 closing, part B: PMC FETCH / WRITE passes of every roofline entry of the non-BAIR bench
# lines (their own denoiser, batch and precision: cfg_handle.py) -> gpurun_out/pmc_<config>_layer<id>.json
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
( while sleep 45; do echo "heartbeat $(date +%T)" >> gpurun_out/pmc_cfg_heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
CONFIG=kth LAYERS="6 1 5 7 4 9 13" bash scripts_gpu/pmc_layers.sh || exit 1
for c in ${CFGS:-smmnist ucf cityscapes}; do CONFIG=$c LAYERS="6 1 5 7 4 13" bash scripts_gpu/pmc_layers.sh || exit 1; done
