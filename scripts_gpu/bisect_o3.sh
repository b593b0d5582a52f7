cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/bisect.jsonl
for v in o1 o3 o3noslp; do
  EXTDM_LIB=$PWD/_variants/$v/libextdm_hip.so timeout -k 10 180 python scripts_gpu/o3_bisect.py $v >> gpurun_out/bisect.jsonl 2>gpurun_out/bisect_$v.err || { echo "fail $v rc=$?"; tail -5 gpurun_out/bisect_$v.err; exit 1; }
done
EXTDM_X3_ATTN_NW=4 EXTDM_LIB=$PWD/_variants/o3/libextdm_hip.so timeout -k 10 180 python scripts_gpu/o3_bisect.py o3_nw4 >> gpurun_out/bisect.jsonl 2>gpurun_out/bisect_nw4.err || { echo "fail nw4"; exit 1; }
cat gpurun_out/bisect.jsonl
