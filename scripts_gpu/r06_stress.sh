#!/bin/bash
# r06 diagnosis: the sampling call's run-to-run determinism with two processes on the GPU,
# per variant: VARIANTS="tag|args|env ..." (default: graph + multi-workgroup sampler; eager;
# one-workgroup sampler); commas inside args / env stand for spaces
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ITERS=${ITERS:-30}
pair() {  # tag, extra args, env
  env $3 timeout -k 10 200 python -u scripts_gpu/r06_stress.py --iters $ITERS --stages sample --tag $1A $2 > gpurun_out/stress_$1A.log 2>&1 &
  local pa=$!
  env $3 timeout -k 10 200 python -u scripts_gpu/r06_stress.py --iters $ITERS --stages sample --tag $1B --batch 2 $2 > gpurun_out/stress_$1B.log 2>&1 &
  local pb=$!
  wait $pa; local ra=$?
  wait $pb; local rb=$?
  echo "$1: rc A=$ra B=$rb"
  grep -h "DONE\|first at" gpurun_out/stress_$1A.log gpurun_out/stress_$1B.log
  [ $ra -eq 0 ] && [ $rb -eq 0 ]
}
VARIANTS=${VARIANTS:-"graph||EXTDM_SAMPLER_1WG=0 eager|--eager|EXTDM_SAMPLER_1WG=0 onewg||EXTDM_SAMPLER_1WG=1"}
for v in $VARIANTS; do
  IFS='|' read -r tag args envs <<< "$v"
  args=${args//,/ }; envs=${envs//,/ }
  pair "$tag" "$args" "${envs:-X=0}" || exit 1
done
