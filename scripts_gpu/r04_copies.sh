# rocclr blit copies per reverse step: kernel stats of DDIM-20 vs DDIM-40 bench generations
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for S in 20 40; do
  rm -rf gpurun_out/prof_cp$S
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cp$S -o run --output-format csv -- python bench.py --sampling-steps $S --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_cp$S.log 2>&1 || exit 1
  python scripts_gpu/copy_sizes.py gpurun_out/prof_cp$S || exit 1
  find gpurun_out/prof_cp$S -name "*kernel_trace.csv" -delete
done
