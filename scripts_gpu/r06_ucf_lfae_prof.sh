#!/bin/bash
# UCF per-generation fixed cost (LFAE encode + decode around the sampler): one kernel trace of a
# 2-step UCF generation at the bench batch, then every launch outside the Unet's own kernels in
# dispatch order (name, grid, us) -> gpurun_out/r06_ucf_lfae_launches.txt
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/prof_ucf_lfae
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_ucf_lfae -o run --output-format csv -- python bench.py --config ucf --sampling-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > gpurun_out/prof_ucf_lfae.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -n 2 gpurun_out/prof_ucf_lfae.log; [ $rc -ne 0 ] && exit $rc
python - > gpurun_out/r06_ucf_lfae_launches.txt <<'PY'
import csv, glob
rows = []
for f in glob.glob('gpurun_out/prof_ucf_lfae/**/*kernel_trace.csv', recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
tot = {}
for r in rows:
    n = r['Kernel_Name'].replace('extdm::(anonymous namespace)::', '')
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    k = n.split('(')[0][:90]
    tot[k] = tot.get(k, 0) + d
    print(f"{d:9.1f}  grid={r.get('Grid_Size', r.get('Grid_Size_X'))} wg={r.get('Workgroup_Size', r.get('Workgroup_Size_X'))}  {n[:140]}")
print('---- totals (us)')
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:40]:
    print(f'{v:10.1f}  {k}')
PY
find gpurun_out/prof_ucf_lfae -name "*kernel_trace.csv" -delete
