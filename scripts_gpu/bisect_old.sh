# The pre-215c30b attention kernel (key descriptors shuffled inside the unit loop) at -O1 / -O3,
# 5 launches each: does the -O3 run-to-run difference of round 1 come back?
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/bisect_old.jsonl
for v in old_O1 old_O3; do
  EXTDM_LIB=$PWD/_variants/$v/libextdm_hip.so timeout -k 10 180 python scripts_gpu/o3_bisect.py $v >> gpurun_out/bisect_old.jsonl 2>gpurun_out/bisect_$v.err || { echo "fail $v"; tail -5 gpurun_out/bisect_$v.err; exit 1; }
done
cat gpurun_out/bisect_old.jsonl
