"""Per-launch durations from a rocprofv3 --kernel-trace directory: for every kernel whose
name contains the pattern, the launches grouped by (name, grid size) in dispatch order,
with count / mean / min / max in microseconds (so launches of different shapes of one
template are not averaged together, unlike the --stats summary).
Usage: kernel_launches.py TRACE_DIR PATTERN"""
import collections
import csv
import glob
import sys

d, pat = sys.argv[1], sys.argv[2]
groups = collections.OrderedDict()
for f in sorted(glob.glob(f'{d}/**/*kernel_trace.csv', recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r.get('Kernel_Name', '')
        if pat not in name:
            continue
        grid = r.get('Grid_Size', r.get('Grid_Size_X', '?'))
        wg = r.get('Workgroup_Size', r.get('Workgroup_Size_X', '?'))
        dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        groups.setdefault((name, grid, wg), []).append(dur)
for (name, grid, wg), v in groups.items():
    short = name.replace('extdm::(anonymous namespace)::', '')[:110]
    print(f'{short}  grid={grid} wg={wg}  n={len(v)}  mean={sum(v) / len(v):.1f}us  '
          f'min={min(v):.1f}  max={max(v):.1f}')
