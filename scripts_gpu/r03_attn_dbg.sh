#!/bin/bash
# Timing-only breakdown of the fused attention layers (EXTDM_X3_DBG: 8 = no epilogue
# loads / stores, 16 = no unit loop, 24 = neither), in-tree library, B = 64.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03c}
for rep in 1 2; do
  for d in 0 8 16 24; do
    EXTDM_X3_DBG=$d timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 >> gpurun_out/${TAG}_dbg.txt || exit 1
  done
done
cat gpurun_out/${TAG}_dbg.txt
