#!/bin/bash
# The tile prologue / epilogue of the level-0 STW kernel: layer tests, layer timing against
# EXTDM_X3_NO_TILE=1 (per-lane path) and HEAD (_variants/base), then the phase stamps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03g}
timeout -k 10 400 python -u -m pytest tests/test_gpu_attn.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 | sed "s/^/tile /" >> gpurun_out/${TAG}_ab.txt || exit 1
  EXTDM_X3_NO_TILE=1 timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 | sed "s/^/notile /" >> gpurun_out/${TAG}_ab.txt || exit 1
  EXTDM_LIB=_variants/base/libextdm_hip.so timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 | sed "s/^/base /" >> gpurun_out/${TAG}_ab.txt || exit 1
done
EXTDM_X3_DBG=32 timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 2 > gpurun_out/${TAG}_stamps.txt 2>&1 || exit 1
cat gpurun_out/${TAG}_ab.txt; grep "C=64,MODE=0" gpurun_out/${TAG}_stamps.txt | tail -2
