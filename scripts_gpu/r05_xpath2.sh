#!/bin/bash
# xpath frame-group size sweep (layer 9) and the whole-step A/B of the best against class-major.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do for fg in 16 32 64 112 0; do EXTDM_XP_FG=$fg timeout -k 10 200 python scripts_gpu/layers.py 64 20 f16x3 9 | sed "s/^/FG=$fg /" || exit 1; done; done
S=20 AB="EXTDM_XP_FG=0" bash scripts_gpu/ab_step.sh
