#!/bin/bash
# Closing evidence, part 1: the GPU suite with the parity log (run_tests.sh), then each non-BAIR
# workload's DDIM-20 kernel shares and level-0 attention layer times (cfgprof.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
bash scripts_gpu/run_tests.sh && bash scripts_gpu/cfgprof.sh
