#!/bin/bash
# full GPU suite (no bench), then the whole-step A/B (DDPM-50, B = 64) in-tree vs $LIBS
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03b_suite2.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r03b_suite2.log; [ $rc -ne 0 ] && exit $rc
LIBS=${LIBS:-c3e} R=2 bash scripts_gpu/ab_bench.sh
