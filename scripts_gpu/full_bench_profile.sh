#!/bin/bash
# Round-end measurement set: the default bench line (DDPM-1000, CPU baseline),
# the rocprofv3 kernel stats of the same command, and the init_conv PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${B:-32}
[ -z "$SKIP_BENCH" ] && timeout -k 10 600 python bench.py --batch $B > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; [ -n "$SKIP_BENCH" ] && rc=0; echo "bench rc=$rc"; cat gpurun_out/bench_full.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_full.err; exit $rc; }
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python scripts_gpu/pmc_init_conv.py $B 10 > gpurun_out/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; tail -3 gpurun_out/pmc_fetch.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python scripts_gpu/pmc_init_conv.py $B 10 > gpurun_out/pmc_write.log 2>&1
rc=$?; echo "pmc write rc=$rc"; tail -3 gpurun_out/pmc_write.log; [ $rc -ne 0 ] && exit $rc
python scripts_gpu/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write "conv_halo_kernel<7, 64, 1" $B gpurun_out/pmc_init_conv.json
rm -rf gpurun_out/prof_full
timeout -k 10 600 rocprofv3 --kernel-trace --stats --collection-period ${PSTART:-40}:${PLEN:-15}:1 -d gpurun_out/prof_full -o run --output-format csv -- python bench.py --batch $B --no-cpu-baseline > gpurun_out/prof_full.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_full.log
find gpurun_out/prof_full -name "*kernel_trace.csv" -delete
[ $rc -ne 0 ] && exit $rc
