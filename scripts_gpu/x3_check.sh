#!/bin/bash
# f16x3 conv path: precision tests, DDIM-20 bench in both precisions, kernel stats of the f16x3 run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_precision.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/x3_tests.log 2>&1
rc=$?; echo "x3 tests rc=$rc"; grep -E "PASS|FAIL|Error|vs fp64|passed|failed" gpurun_out/x3_tests.log | tail -30
[ $rc -ne 0 ] && exit $rc
for P in fp32 f16x3; do
  timeout -k 10 300 python bench.py --sampling-steps 20 --batch 32 --no-cpu-baseline --precision $P > gpurun_out/x3_bench_$P.json 2> gpurun_out/x3_bench_$P.err
  rc=$?; echo "bench $P rc=$rc"; cat gpurun_out/x3_bench_$P.json
  [ $rc -ne 0 ] && { tail -20 gpurun_out/x3_bench_$P.err; exit $rc; }
done
rm -rf gpurun_out/prof_x3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_x3 -o run --output-format csv -- python bench.py --sampling-steps 20 --batch 32 --no-cpu-baseline --precision f16x3 > gpurun_out/prof_x3.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_x3.log
find gpurun_out/prof_x3 -name "*kernel_trace.csv" -delete
f=$(find gpurun_out/prof_x3 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python scripts_gpu/stats.py $f 30
exit $rc
