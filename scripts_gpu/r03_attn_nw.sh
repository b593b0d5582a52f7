#!/bin/bash
# NW = 8 (one 8-wave workgroup per CU) vs NW = 4 (two 4-wave workgroups per CU) for the
# fused attention layers, with and without the unit loop (EXTDM_X3_DBG=16).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03d}
for rep in 1 2; do
  for nw in 8 4; do
    for d in 0 16; do
      EXTDM_X3_ATTN_NW=$nw EXTDM_X3_DBG=$d timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 | sed "s/^/nw=$nw /" >> gpurun_out/${TAG}_nw.txt || exit 1
    done
  done
done
cat gpurun_out/${TAG}_nw.txt
