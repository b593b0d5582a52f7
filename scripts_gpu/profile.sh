#!/bin/bash
# Timing sweep over the per-GPU batch (short DDPM schedule) + rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in ${BATCHES:-8 16 32}; do
  timeout -k 10 300 python bench.py --sampling-steps ${SSTEPS:-20} --steps 1 --warmup 1 --batch $B --no-cpu-baseline > gpurun_out/sweep_b$B.json 2> gpurun_out/sweep_b$B.err
  rc=$?; echo "batch $B rc=$rc"; cat gpurun_out/sweep_b$B.json
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/sweep_b$B.err; exit $rc; fi
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --sampling-steps ${SSTEPS:-20} --steps 1 --warmup 0 --batch ${PBATCH:-16} --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -5 gpurun_out/prof.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
