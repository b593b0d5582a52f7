"""Group a rocprofv3 kernel_trace.csv by (kernel, grid) -> count, avg us, total ms."""
import csv
import sys
from collections import defaultdict

agg = defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(sys.argv[1])):
    name = r['Kernel_Name']
    short = name.replace('void ', '').replace('extdm::(anonymous namespace)::', '').split('(')[0]
    key = (short, r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'], r['LDS_Block_Size'])
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    agg[key][0] += 1
    agg[key][1] += d
flt = sys.argv[2] if len(sys.argv) > 2 else ''
rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
for (k, gx, gy, gz, lds), (n, t) in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    if flt and flt not in k:
        continue
    print(f'{t / 1e3:9.2f}ms n={n:5d} avg={t / n:8.1f}us grid=({gx},{gy},{gz}) lds={lds} {k}')
