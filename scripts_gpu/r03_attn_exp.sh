#!/bin/bash
# Round 3 attention experiments: NW = 4 vs 8 workgroups (EXTDM_X3_ATTN_NW) and the SQ
# counters of the in-tree kernels (scripts_gpu/pmc_attn.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 || exit 1
  EXTDM_X3_ATTN_NW=4 timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 || exit 1
done
TAG=${TAG:-r03pa} bash scripts_gpu/pmc_attn.sh
