#!/bin/bash
# r06 diagnosis: pairs of GPU processes started together (file barrier), each looping 25 s:
# the sampler step alone (fixed inputs, repeated; every repeat bitwise equal to the first) beside
# a process running sampling calls, once per library in LIBS (default: the in-tree one)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run2() {  # name, cmdA, cmdB
  rm -f /tmp/r06sync*
  timeout -k 10 150 $2 --sync /tmp/r06sync --peers 2 --seconds ${SECS:-25} > gpurun_out/pair_$1_A.log 2>&1 &
  local pa=$!
  timeout -k 10 150 $3 --sync /tmp/r06sync --peers 2 --seconds ${SECS:-25} > gpurun_out/pair_$1_B.log 2>&1 &
  local pb=$!
  wait $pa; local ra=$?; wait $pb; local rb=$?
  echo "$1: rc $ra $rb"
  grep -h "DONE" gpurun_out/pair_$1_A.log gpurun_out/pair_$1_B.log
  grep -h "elements differ" gpurun_out/pair_$1_A.log gpurun_out/pair_$1_B.log | head -3
  [ $ra -eq 0 ] && [ $rb -eq 0 ]
}
P="python -u scripts_gpu"
for lib in ${LIBS:-140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd/libextdm_hip.so}; do
  tag=$(echo $lib | tr '/' '_')
  EXTDM_LIB=$PWD/$lib run2 "$tag" "$P/r06_samplercheck.py --tag chk" "$P/r06_stress.py --stages sample --tag loop" || exit 1
done
