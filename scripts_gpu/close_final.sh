#!/bin/bash
# Closing evidence on the final library: sampler / chain parity tests, the PMC passes + DDIM-20 BAIR
# kernel stats (measure.sh), the SQ passes of the shipped level-0 3x3 conv templates and attention
# layers (bench layers 1, 5, 6, 7), then the BAIR bench line with this library's PMC traffic (the
# fresh pmc_*.json copied into this snapshot's profiles/ first; the caller commits the same files).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wrappers.py tests/test_gpu_bench_ranks.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/final_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/final_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts_gpu/measure.sh || exit 1
for l in 1 5 6 7; do
  CONFIG=bair LAYER=$l TAG=r05sq bash scripts_gpu/pmc_sq.sh > gpurun_out/r05_sq_l$l.txt 2>&1 || { tail -5 gpurun_out/r05_sq_l$l.txt; exit 1; }
done
cp gpurun_out/pmc_layer*.json gpurun_out/pmc_*_layer6.json profiles/
CONFIGS=bair bash scripts_gpu/bench_all.sh
