#!/bin/bash
# rocprofv3 kernel stats of one short generation under two settings (A: default, B: $AB)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
S=${S:-20}
for arm in A B; do
  if [ $arm = A ]; then envs=""; else envs="$AB"; fi
  rm -rf gpurun_out/abp_$arm
  for kv in $envs; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abp_$arm -o run --output-format csv -- python bench.py --sampling-steps $S --steps $S --warmup 2 --no-cpu-baseline > gpurun_out/abp_$arm.log 2>&1
  rc=$?; echo "$arm rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/abp_$arm.log; exit $rc; }
  for kv in $envs; do unset "${kv%%=*}"; done
  find gpurun_out/abp_$arm -name "*kernel_trace.csv" -delete
done
