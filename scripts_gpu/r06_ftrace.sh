#!/bin/bash
# One config's eager forward, dispatches in launch order (rocprofv3 kernel trace + trace_order.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
c=${CONFIG:-cityscapes}
rm -rf gpurun_out/ftrace_$c
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ftrace_$c -o run --output-format csv -- python scripts_gpu/forward_trace_cfg.py $c > gpurun_out/ftrace_$c.log 2>&1 || { tail -5 gpurun_out/ftrace_$c.log; exit 1; }
python scripts_gpu/trace_order.py "$(find gpurun_out/ftrace_$c -name '*kernel_trace.csv' | head -1)" 3 > gpurun_out/r06_forward_order_$c.txt
find gpurun_out/ftrace_$c -name "*kernel_trace.csv" -delete
