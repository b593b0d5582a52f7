# SQ instruction-mix / stall passes (scripts_gpu/pmc_sq.sh) over the bench layers in $LAYERS
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for L in ${LAYERS:-1 5 0 6 7 9 10 12 13}; do
  echo "=== layer $L"
  LAYER=$L TAG=${TAG:-r04sq} bash scripts_gpu/pmc_sq.sh || exit 1
done > gpurun_out/${TAG:-r04sq}_table.txt 2>&1
tail -5 gpurun_out/${TAG:-r04sq}_table.txt
