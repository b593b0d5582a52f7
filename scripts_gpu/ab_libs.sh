#!/bin/bash
# rocprofv3 kernel stats of one short generation per library: the in-tree one (arm "cur")
# and each _variants/<name>/libextdm_hip.so named in $LIBS (space-separated names)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
S=${S:-20}
for arm in cur $LIBS; do
  rm -rf gpurun_out/abp_$arm
  if [ $arm = cur ]; then unset EXTDM_LIB; else export EXTDM_LIB=_variants/$arm/libextdm_hip.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abp_$arm -o run --output-format csv -- python bench.py --sampling-steps $S --steps $S --warmup 2 --no-cpu-baseline > gpurun_out/abp_$arm.log 2>&1
  rc=$?; echo "$arm rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/abp_$arm.log; exit $rc; }
  find gpurun_out/abp_$arm -name "*kernel_trace.csv" -delete
done
