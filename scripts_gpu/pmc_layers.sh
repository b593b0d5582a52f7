#!/bin/bash
# HBM bytes per launch of bench roofline kernels: separate rocprofv3 --pmc passes for FETCH_SIZE and
# WRITE_SIZE over `extdm_bench_layer` launches of CONFIG's denoiser (default bair; cfg_handle.py),
# summarised (scripts_gpu/pmc_summary.py; the gfx950 FETCH_SIZE x2 correction only for whole-line
# readers, bench.py NativeWorkload.wide_reads) into gpurun_out/pmc_layer<id>.json (bair) or
# gpurun_out/pmc_<config>_layer<id>.json. LAYERS="0 12" selects the ids (default: bair's LAYERS).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
CONFIG=${CONFIG:-bair}
if [ -z "$LAYERS" ]; then
  LAYERS=$(python -c "import bench; print(' '.join(str(l) for l, *_ in bench.NativeWorkload.LAYERS))") || exit 1
fi
for L in $LAYERS; do
  # the launched template, the read rule, the precision / batch (one untimed run outside the profiler)
  timeout -k 10 120 python scripts_gpu/pmc_layer_run.py $CONFIG $L 2 > gpurun_out/pmc_${CONFIG}_${L}_spec.txt 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "layer $L spec rc=$rc"; tail -3 gpurun_out/pmc_${CONFIG}_${L}_spec.txt; continue; }
  PAT=$(sed -n 's/^KERNEL://p' gpurun_out/pmc_${CONFIG}_${L}_spec.txt)
  WIDE=$(sed -n 's/^WIDE://p' gpurun_out/pmc_${CONFIG}_${L}_spec.txt)
  PRC=$(sed -n 's/^PREC:\([^ ]*\) .*/\1/p' gpurun_out/pmc_${CONFIG}_${L}_spec.txt)
  BB=$(sed -n 's/^PREC:.* B:\(.*\)/\1/p' gpurun_out/pmc_${CONFIG}_${L}_spec.txt)
  [ -z "$PAT" ] && { echo "layer $L: no kernel template"; continue; }
  for C in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/pmc_${CONFIG}_${L}_$C
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_${CONFIG}_${L}_$C -o run --output-format csv -- python scripts_gpu/pmc_layer_run.py $CONFIG $L 10 > gpurun_out/pmc_${CONFIG}_${L}_$C.log 2>&1
    rc=$?; echo "$CONFIG layer $L $C rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_${CONFIG}_${L}_$C.log; exit $rc; }
  done
  OUT=gpurun_out/pmc_layer$L.json; [ "$CONFIG" != bair ] && OUT=gpurun_out/pmc_${CONFIG}_layer$L.json
  PREC=$PRC python scripts_gpu/pmc_summary.py gpurun_out/pmc_${CONFIG}_${L}_FETCH_SIZE gpurun_out/pmc_${CONFIG}_${L}_WRITE_SIZE "$PAT" $BB $OUT $WIDE || exit 1
  find gpurun_out/pmc_${CONFIG}_${L}_* -name "*trace*.csv" -delete
done
