"""Dispatches of the last of N identical forwards in a rocprofv3 kernel_trace.csv, in
launch order: duration, grid, kernel. Usage: trace_order.py trace.csv N"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
rows = [r for r in rows if 'rocclr' not in r['Kernel_Name']]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
per = len(rows) // n
last = rows[-per:]
tot = 0.0
for i, r in enumerate(last):
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    tot += d
    k = r['Kernel_Name'].replace('void ', '').replace('extdm::(anonymous namespace)::', '').split('(')[0][:60]
    print(f"{i:4d} {d:9.1f}us grid=({r['Grid_Size_X']},{r['Grid_Size_Y']},{r['Grid_Size_Z']}) wg={r['Workgroup_Size_X']} {k}")
print(f'total {tot / 1e3:.3f} ms over {len(last)} dispatches')
