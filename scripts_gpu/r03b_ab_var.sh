#!/bin/bash
# conv layer A/B: in-tree vs $VAR (a _variants/<name>/libextdm_hip.so), two rounds, layers $LAYERS
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
LAYERS=${LAYERS:-1,5,0,4,9,10}
for rep in 1 2; do
  timeout -k 10 180 python scripts_gpu/layers.py 64 20 f16x3 $LAYERS | sed 's/^/tree /' || exit 1
  EXTDM_LIB=$VAR timeout -k 10 180 python scripts_gpu/layers.py 64 20 f16x3 $LAYERS | sed "s#^#$(basename $(dirname $VAR)) #" || exit 1
done
