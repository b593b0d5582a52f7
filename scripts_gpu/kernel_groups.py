"""Group a rocprofv3 kernel trace by (kernel name, grid size): launches and average
duration, so a kernel template shared by several layers (e.g. the 7x7 halo conv of
init_conv and of the LFAE generator's first block) is reported per layer."""
import csv
import json
import sys
from collections import defaultdict

trace, pattern = sys.argv[1], sys.argv[2]
g = defaultdict(list)
for r in csv.DictReader(open(trace)):
    if pattern in r['Kernel_Name']:
        nm = r['Kernel_Name']
        nm = nm[:nm.find('>(') + 1] if '>(' in nm else nm
        key = (nm, r.get('Grid_Size_X', r.get('Grid_Size', '')), r.get('Workgroup_Size_X', ''))
        g[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
out = [{'kernel': k[0], 'grid_x': k[1], 'block_x': k[2], 'launches': len(v), 'avg_ms': round(sum(v) / len(v), 4),
        'min_ms': round(min(v), 4), 'max_ms': round(max(v), 4)} for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))]
print(json.dumps(out, indent=1))
