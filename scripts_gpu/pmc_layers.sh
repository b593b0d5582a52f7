#!/bin/bash
# HBM bytes per launch of the bench's roofline kernels (bench.py LAYERS): separate
# rocprofv3 --pmc passes for FETCH_SIZE and WRITE_SIZE over `extdm_bench_layer` launches,
# summarised with the gfx950 FETCH_SIZE x2 correction (scripts_gpu/pmc_summary.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
B=${B:-64}
for spec in "1:conv_x3_kernel<3, 1, 64, 256, 1, 4, 4, 2, true, 2, false>" "5:conv_x3_kernel<3, 1, 64, 256, 1, 4, 4, 2, true, 1, true>" "0:conv_x3_kernel<7, 1, 64, 512, 1, 8, 16, 1, true, 1, false>" "4:conv_x3_kernel<1, 1, 64, 128, 2, 4, 4, 2, true, 1, false>"; do
  L=${spec%%:*}; PAT=${spec#*:}
  for C in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/pmc_${L}_$C
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_${L}_$C -o run --output-format csv -- python scripts_gpu/pmc_init_conv.py $B 10 $L > gpurun_out/pmc_${L}_$C.log 2>&1
    rc=$?; echo "layer $L $C rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_${L}_$C.log; exit $rc; }
  done
  python scripts_gpu/pmc_summary.py gpurun_out/pmc_${L}_FETCH_SIZE gpurun_out/pmc_${L}_WRITE_SIZE "$PAT" $B gpurun_out/pmc_layer$L.json
  find gpurun_out/pmc_${L}_* -name "*trace*.csv" -delete
done
