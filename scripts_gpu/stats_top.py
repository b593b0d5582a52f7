"""Top kernels of a rocprofv3 kernel_stats.csv: total ms, calls, avg us, share."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
for r in rows[:n]:
    name = r['Name'].replace('extdm::(anonymous namespace)::', '').replace('void ', '')[:72]
    print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} ms {int(r['Calls']):6d} x {float(r['AverageNs']) / 1e3:9.1f} us "
          f"{float(r['Percentage']):6.2f}%  {name}")
