#!/bin/bash
# Launch groups (kernel, grid) of a DDIM-20 generation per config on the shipped library, to find
# launches that run fewer workgroups than CUs; then SQ passes of BAIR bench layers 0 1 5 6 7.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in ${CONFIGS:-kth cityscapes}; do
  rm -rf gpurun_out/grid_$c
  timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/grid_$c -o run --output-format csv -- python bench.py --config $c --sampling-steps 20 --warmup 0 --no-cpu-baseline --no-roofline > gpurun_out/grid_$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/grid_$c.log; exit $rc; }
  python scripts_gpu/launch_groups.py gpurun_out/grid_$c 45 > gpurun_out/r06_grids_$c.txt
  find gpurun_out/grid_$c -name "*kernel_trace.csv" -delete
done
for L in ${SQ_LAYERS:-0 1 5 6 7}; do
  LAYER=$L TAG=r06sq bash scripts_gpu/pmc_sq.sh > gpurun_out/r06_sq_l$L.txt 2>&1 || { tail -5 gpurun_out/r06_sq_l$L.txt; exit 1; }
done
