"""Kernel launches of a rocprofv3 --kernel-trace directory grouped by (kernel, grid, workgroup),
sorted by total time: share of GPU time, launches, mean duration and workgroups per launch (to spot
launches that leave CUs idle). Usage: launch_groups.py TRACE_DIR [N]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
groups = collections.defaultdict(list)
for f in sorted(glob.glob(f'{d}/**/*kernel_trace.csv', recursive=True)):
    for r in csv.DictReader(open(f)):
        grid = int(r.get('Grid_Size', r.get('Grid_Size_X', '0')) or 0)
        wg = int(r.get('Workgroup_Size', r.get('Workgroup_Size_X', '1')) or 1)
        groups[(r.get('Kernel_Name', ''), grid, wg)].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
tot = sum(sum(v) for v in groups.values())
for (name, grid, wg), v in sorted(groups.items(), key=lambda kv: -sum(kv[1]))[:top]:
    short = name.replace('extdm::(anonymous namespace)::', '').replace('void ', '')[:120]
    print(f'{100 * sum(v) / tot:5.2f}%  n={len(v):5d}  mean={sum(v) / len(v):8.1f}us  wgs={grid // max(wg, 1):7d}  {short}')
