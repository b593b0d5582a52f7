#!/bin/bash
# Layer timing of the in-tree library against the variants named in $VARS (under _variants/),
# interleaved, twice; the attention layer tests first.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03v}
timeout -k 10 400 python -u -m pytest tests/test_gpu_attn.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 | sed "s/^/cur /" >> gpurun_out/${TAG}_ab.txt || exit 1
  for v in $VARS; do
    EXTDM_LIB=_variants/$v/libextdm_hip.so timeout -k 10 120 python scripts_gpu/attn_dbg.py 64 20 | sed "s/^/$v /" >> gpurun_out/${TAG}_ab.txt || exit 1
  done
done
cat gpurun_out/${TAG}_ab.txt | sed 's/lib=[^ ]* //'
