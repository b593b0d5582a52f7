#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts_gpu/run_tests.sh
rc=$?
if [ $rc -ne 0 ]; then echo "tests failed rc=$rc"; exit $rc; fi
BATCHES="${BATCHES:-16 32}" bash scripts_gpu/profile.sh
