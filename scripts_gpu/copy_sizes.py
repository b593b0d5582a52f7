"""Histogram of rocclr blit kernels (count by grid size) in a rocprofv3 kernel trace directory."""
import collections
import csv
import glob
import sys

path = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
c = collections.Counter()
tot = collections.Counter()
n_phase = 0
for r in csv.DictReader(open(path)):
    n = r['Kernel_Name']
    if 'conv_x3_kernel<5' in n:
        n_phase += 1
    if 'rocclr' in n:
        k = (n.split('(')[0][-30:], r.get('Grid_Size_X', r.get('Grid_Size', '?')))
        c[k] += 1
        tot[k] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
print(sys.argv[1], 'phase-conv launches', n_phase)
for k, v in c.most_common(25):
    print(f'{v:6d} {tot[k] / 1e6:9.3f} ms  {k}')
