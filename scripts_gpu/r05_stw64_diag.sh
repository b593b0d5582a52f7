#!/bin/bash
# stw64_x3 diagnostics: layer-6 time with the unit loop / the epilogue knocked out
# (EXTDM_STW64_DBG), then the SQ instruction mix / stall passes for KTH and UCF.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in kth ucf; do
  for d in 0 16 8 24; do
    EXTDM_STW64_DBG=$d timeout -k 10 120 python scripts_gpu/layers_cfg.py $c 6 || exit 1
  done
done
CONFIG=kth LAYER=6 TAG=sqkth bash scripts_gpu/pmc_sq.sh > gpurun_out/r05_sq_kth6.txt 2>&1 || exit 1
CONFIG=ucf LAYER=6 TAG=squcf bash scripts_gpu/pmc_sq.sh > gpurun_out/r05_sq_ucf6.txt 2>&1 || exit 1
grep -A20 stw64 gpurun_out/r05_sq_kth6.txt | head -22
