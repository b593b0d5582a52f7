"""Compare two rocprofv3 kernel-stat CSVs (ab_prof.sh arms): per-kernel total ms, A vs B."""
import csv
import sys

a_dir, b_dir = (sys.argv[1:3] + ['gpurun_out/abp_A', 'gpurun_out/abp_B'])[:2] if len(sys.argv) > 2 else \
    ('gpurun_out/abp_A', 'gpurun_out/abp_B')


def load(d):
    return {r['Name']: (float(r['TotalDurationNs']) / 1e6, int(r['Calls']))
            for r in csv.DictReader(open(f'{d}/run_kernel_stats.csv'))}


A, B = load(a_dir), load(b_dir)
ta, tb = sum(v[0] for v in A.values()), sum(v[0] for v in B.values())
print(f'total A {ta:.2f} ms   B {tb:.2f} ms   A/B {ta / tb:.4f}')
rows = sorted(set(A) | set(B), key=lambda n: -abs(A.get(n, (0, 0))[0] - B.get(n, (0, 0))[0]))
for n in rows[:12]:
    a, b = A.get(n, (0, 0)), B.get(n, (0, 0))
    print(f'{a[0]:9.2f} ({a[1]:5d})  {b[0]:9.2f} ({b[1]:5d})  {a[0] - b[0]:+8.2f}  {n[:90]}')
