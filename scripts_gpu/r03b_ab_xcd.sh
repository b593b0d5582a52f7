#!/bin/bash
# XCD-aware tile order A/B: conv layers + cross attention (bench_layer ids) in-tree vs $VAR,
# then the FETCH / WRITE PMC passes of the 7x7 (layer 0) and the cross kernel (layer 8) in-tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
VAR=${VAR:-_variants/h3/libextdm_hip.so}
for rep in 1 2; do
  timeout -k 10 180 python scripts_gpu/layers.py 64 20 f16x3 1,5,0,4,8,9,10 | sed 's/^/tree /' || exit 1
  EXTDM_LIB=$VAR timeout -k 10 180 python scripts_gpu/layers.py 64 20 f16x3 1,5,0,4,8,9,10 | sed "s#^#base #" || exit 1
done
for L in 0 8 1; do
  for C in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/pmcx_${L}_$C
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmcx_${L}_$C -o run --output-format csv -- python scripts_gpu/pmc_init_conv.py 64 10 $L > gpurun_out/pmcx_${L}_$C.log 2>&1 || exit 1
  done
  PAT=$(python -c "import bench; print([k for l, _, k, _ in bench.NativeWorkload.LAYERS if l == $L][0])")
  python scripts_gpu/pmc_summary.py gpurun_out/pmcx_${L}_FETCH_SIZE gpurun_out/pmcx_${L}_WRITE_SIZE "$PAT" 64 gpurun_out/pmcx_layer$L.json || exit 1
  find gpurun_out/pmcx_${L}_* -name "*trace*.csv" -delete
done
