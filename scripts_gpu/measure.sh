#!/bin/bash
# Round measurement set: (1) the default bench line (DDPM-1000, CPU baseline);
# (2) FETCH_SIZE / WRITE_SIZE passes over the init_conv kernel (separate runs);
# (3) rocprofv3 --kernel-trace --stats of the bench command at DDIM-20 (the profiler
# crashes on the 2000-replay DDPM-1000 command; same kernels and shapes).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${B:-32}
KP=${KP:-conv_x3_kernel<7, 64, 512}
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python bench.py --batch $B > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_full.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_full.err; exit $rc; }
fi
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/prof
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python scripts_gpu/pmc_init_conv.py $B 10 > gpurun_out/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; tail -2 gpurun_out/pmc_fetch.log; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python scripts_gpu/pmc_init_conv.py $B 10 > gpurun_out/pmc_write.log 2>&1
rc=$?; echo "pmc write rc=$rc"; tail -2 gpurun_out/pmc_write.log; [ $rc -ne 0 ] && exit $rc
python scripts_gpu/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write "$KP" $B gpurun_out/pmc_init_conv.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --sampling-steps 20 --batch $B --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof.log
find gpurun_out/prof -name "*kernel_trace.csv" -delete
exit $rc
