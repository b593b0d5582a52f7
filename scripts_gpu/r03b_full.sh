#!/bin/bash
# conv layer A/B against $BASE, then smoke + full GPU suite + attention A/B + bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
NOPREC=1 bash scripts_gpu/r03b_ab_conv.sh || exit $?
bash scripts_gpu/r03b_suite.sh
