"""Summarise a rocprofv3 kernel_stats.csv (top kernels by total time)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f'total kernel time {tot / 1e6:.1f} ms')
for r in rows[:n]:
    print(f"{float(r['Percentage']):6.2f}% {float(r['TotalDurationNs']) / 1e6:9.2f}ms calls={r['Calls']:>6} "
          f"avg={float(r['AverageNs']) / 1e3:9.1f}us  {r['Name'][:100]}")
