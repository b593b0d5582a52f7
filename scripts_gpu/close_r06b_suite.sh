#!/bin/bash
# Round-6 closing on the final library, part 2: smoke + the whole GPU suite with the parity log
# (run_tests.sh), the SQ passes of BAIR bench layers 0 1 5 6 7, the DDIM-20 BAIR kernel stats
# (measure.sh, SKIP_PMC=1), each step under its own limit, stopping at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts_gpu/run_tests.sh || exit 1
for L in 0 1 5 6 7; do
  LAYER=$L TAG=r06sq bash scripts_gpu/pmc_sq.sh > gpurun_out/r06_sq_l$L.txt 2>&1 || { tail -5 gpurun_out/r06_sq_l$L.txt; exit 1; }
done
SKIP_PMC=1 TAG=r06 bash scripts_gpu/measure.sh
