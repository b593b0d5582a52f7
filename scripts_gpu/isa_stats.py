"""Static ISA census of one kernel in a hipcc --save-temps .s file: instruction counts by
class for the whole kernel and for its hottest loop (the largest basic-block range between
a loop label and its backward branch). Usage: isa_stats.py FILE.s KERNEL_SUBSTRING"""
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
lines = open(path).read().split('\n')
start = next(i for i, l in enumerate(lines) if re.match(r'^_Z\S*' + re.escape(pat) + r'\S*:', l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
body = [l.strip() for l in lines[start:end + 1]]


def cls(ins):
    op = ins.split()[0]
    if op.startswith('v_mfma'):
        return 'mfma'
    if op.startswith(('v_', )):
        return 'valu'
    if op.startswith('s_waitcnt'):
        return 'waitcnt'
    if op.startswith(('s_barrier',)):
        return 'barrier'
    if op.startswith('s_nop'):
        return 'nop'
    if op.startswith('s_'):
        return 'salu'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('buffer_', 'global_', 'scratch_', 'flat_')):
        return 'vmem'
    return 'other'


def census(ls):
    c = {}
    for l in ls:
        if not l or l.startswith(('.', ';', '//')) or re.match(r'^\S+:', l):
            continue
        k = cls(l)
        c[k] = c.get(k, 0) + 1
    return c


print('kernel', census(body))
labels = {l.split(':')[0]: i for i, l in enumerate(body) if re.match(r'^\.LBB\S+:', l)}
best = None
for i, l in enumerate(body):
    m = re.match(r'^s_cbranch_\w+\s+(\.LBB\S+)', l) or re.match(r'^s_branch\s+(\.LBB\S+)', l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        n = i - labels[m.group(1)]
        if best is None or n > best[1] - best[0]:
            best = (labels[m.group(1)], i)
if best:
    print('loop', best, census(body[best[0]:best[1] + 1]))
