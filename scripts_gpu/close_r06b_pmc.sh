#!/bin/bash
# Round-6 closing on the final library (after the long-K split), PMC part: FETCH / WRITE passes of
# every roofline entry of the bench lines of CFGS (bair: its LAYERS; kth: 6 1 5 7 4 9 13; the others:
# 6 1 5 7 4 13) -> gpurun_out/pmc_layer<id>.json / pmc_<config>_layer<id>.json (committed to profiles/).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
( while sleep 45; do echo "heartbeat $(date +%T)" >> gpurun_out/pmc_close_heartbeat.log; done ) &
HB=$!
trap 'kill $HB' EXIT
sha256sum 140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd/libextdm_hip.so | cut -c1-16
for c in ${CFGS:-bair kth}; do
  case $c in
    bair) L="" ;;
    kth) L="6 1 5 7 4 9 13" ;;
    *) L="6 1 5 7 4 13" ;;
  esac
  CONFIG=$c LAYERS="$L" bash scripts_gpu/pmc_layers.sh || exit 1
done
