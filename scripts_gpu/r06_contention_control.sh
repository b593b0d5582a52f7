#!/bin/bash
# r06: the two-process determinism test on the control library (_variants/slp: the sampler built
# WITH SLP vectorisation, everything else as shipped) — expected to FAIL — then on the shipped one
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
EXTDM_LIB=$PWD/_variants/slp/libextdm_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread \
  tests/test_gpu_sampler.py -k second_gpu_process > gpurun_out/contention_slp.log 2>&1
echo "control (SLP sampler) rc=$? (1 = the test caught it)"
grep -h "mismatches" gpurun_out/contention_slp.log | head -3 | cut -c1-300
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread \
  tests/test_gpu_sampler.py -k second_gpu_process > gpurun_out/contention_shipped.log 2>&1
rc=$?
echo "shipped rc=$rc"; tail -2 gpurun_out/contention_shipped.log
exit $rc
