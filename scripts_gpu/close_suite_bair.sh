#!/bin/bash
# Closing evidence on the shipped library: the GPU suite with the parity log (run_tests.sh), then the
# BAIR bench line (its roofline traffic from the committed PMC files of the same library).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
bash scripts_gpu/run_tests.sh && CONFIGS=bair bash scripts_gpu/bench_all.sh
