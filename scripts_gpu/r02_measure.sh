#!/bin/bash
# Round-2 measurement: parity subset, the driver's bench command, and rocprofv3 kernel
# stats of the same bench at DDIM-20 (the profiler segfaults on 2000 graph replays).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r02}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 600 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/${TAG}_bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_bench.err; exit $rc; }
fi
if [ -n "$PROF" ]; then
  rm -rf gpurun_out/${TAG}_prof
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --sampling-steps 20 --batch 64 --no-cpu-baseline --warmup 2 > gpurun_out/${TAG}_prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/${TAG}_prof.log
  find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -delete
  exit $rc
fi
