"""Per-(kernel, grid) duration summary of a rocprofv3 SQLite result: python db_stats.py run_results.db"""
import sqlite3
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
g = defaultdict(list)
for name, gx, gy, gz, wx, d in c.execute('select name, grid_x, grid_y, grid_z, workgroup_x, duration from kernels'):
    g[(name, gx, gy, gz, wx)].append(d)
rows = sorted(g.items(), key=lambda kv: -sum(kv[1]))
for (name, gx, gy, gz, wx), ds in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
    ds = sorted(ds)
    print(f'{sum(ds) / 1e6:9.3f} ms n={len(ds):5d} mean={sum(ds) / len(ds) / 1e3:8.1f} us med={ds[len(ds) // 2] / 1e3:8.1f}'
          f' grid=({gx},{gy},{gz}) wg={wx} {name[:110]}')
