#!/bin/bash
# Round-3 closing measurement on the in-tree library: PMC FETCH / WRITE passes of every
# bench roofline kernel (pmc_layers.sh), copied into profiles/ so the bench line's
# `traffic` fields read them, then smoke + the default bench line + the DDIM-20 kernel
# stats (r03c_head.sh; the GPU suite too unless NOSUITE=1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
B=64 bash scripts_gpu/pmc_layers.sh || exit 1
cp gpurun_out/pmc_layer*.json profiles/ || exit 1
TAG=${TAG:-r03e} bash scripts_gpu/r03c_head.sh
