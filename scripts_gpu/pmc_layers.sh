#!/bin/bash
# HBM bytes per launch of the bench's roofline kernels (bench.py LAYERS, names and ids
# taken from there): separate rocprofv3 --pmc passes for FETCH_SIZE and WRITE_SIZE over
# `extdm_bench_layer` launches, summarised (scripts_gpu/pmc_summary.py; the gfx950 FETCH_SIZE x2
# correction only for the layers in bench.py WIDE_READS) into gpurun_out/pmc_layer<id>.json.
# LAYERS_ONLY="0 12" restricts the passes to those ids.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
B=${B:-64}
python -c "import bench; [print(f'{l}:{int(l in bench.NativeWorkload.WIDE_READS)}:{k}') for l, _, k, _ in bench.NativeWorkload.LAYERS]" > gpurun_out/pmc_specs.txt || exit 1
while IFS= read -r spec; do
  L=${spec%%:*}; rest=${spec#*:}; WIDE=${rest%%:*}; PAT=${rest#*:}
  if [ -n "$LAYERS_ONLY" ] && ! echo " $LAYERS_ONLY " | grep -q " $L "; then continue; fi
  for C in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/pmc_${L}_$C
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_${L}_$C -o run --output-format csv -- python scripts_gpu/pmc_init_conv.py $B 10 $L > gpurun_out/pmc_${L}_$C.log 2>&1
    rc=$?; echo "layer $L $C rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_${L}_$C.log; exit $rc; }
  done
  python scripts_gpu/pmc_summary.py gpurun_out/pmc_${L}_FETCH_SIZE gpurun_out/pmc_${L}_WRITE_SIZE "$PAT" $B gpurun_out/pmc_layer$L.json $WIDE || exit 1
  find gpurun_out/pmc_${L}_* -name "*trace*.csv" -delete
done < gpurun_out/pmc_specs.txt
