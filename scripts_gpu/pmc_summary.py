"""Per-launch HBM bytes of one kernel from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE; KB units). MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE counts half the
bytes of a wide coalesced streaming read (16 B per lane) and other read widths are uncalibrated,
so the x2 correction is applied only when the caller says the kernel's HBM reads are of that kind
(argument `wide` = 1, bench.py WIDE_READS); otherwise hbm_bytes_per_launch is raw FETCH + WRITE.
Both the raw FETCH and the rule used are recorded. Also records the launched kernel's full name
and the sha256 prefix of the library the passes ran on, which bench.py checks before it reports
the traffic. Usage: pmc_summary.py FETCH_DIR WRITE_DIR PATTERN BATCH OUT.json [wide]"""
import csv
import glob
import hashlib
import json
import os
import re
import sys

fetch_dir, write_dir, pattern, batch, out = sys.argv[1:6]
wide = len(sys.argv) > 6 and sys.argv[6] == '1'
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = '140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd'


def norm(name):
    """Kernel name without its parameter list; rocprofv3 leaves names it cannot demangle
    (the _Float16 parameters) mangled: rebuild their `ident<args>` from the mangling."""
    if name.startswith('_Z'):
        for i in range(len(name)):
            for k in (1, 2):
                if not name[i:i + k].isdigit():
                    continue
                n, e = int(name[i:i + k]), i + k
                ident = name[e:e + n]
                if not (ident.endswith('kernel') and (ident[0].isalpha() or ident[0] == '_')):
                    continue
                args = re.match(r'I((?:L[ib]\d+E)+)E', name[e + n:])
                if not args:
                    return ident
                vals = [('true' if v == '1' else 'false') if t == 'b' else v
                        for t, v in re.findall(r'L([ib])(\d+)E', args.group(1))]
                return f'{ident}<{", ".join(vals)}>'
        return name
    return re.sub(r'\((?!anonymous).*$', '', name)


def rows(d, counter):
    vals, names, seen = [], set(), set()
    for f in glob.glob(f'{d}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get('Kernel_Name', '')
            seen.add(norm(name)[-90:])
            if pattern in norm(name) and r.get('Counter_Name') == counter:
                vals.append(float(r['Counter_Value']))
                names.add(norm(name))
    if not vals:
        sys.exit(f'no {counter} rows for {pattern!r}; kernels seen: {sorted(seen)}')
    return vals, names


fe, n1 = rows(fetch_dir, 'FETCH_SIZE')
wr, n2 = rows(write_dir, 'WRITE_SIZE')
names = n1 | n2
if len(names) != 1:
    sys.exit(f'pattern {pattern!r} matches several kernels: {sorted(names)}')
lib = os.environ.get('EXTDM_LIB') or os.path.join(REPO, PKG, 'libextdm_hip.so')
res = {'kernel': pattern, 'kernel_name': names.pop(), 'batch': int(batch),
       'precision': os.environ.get('PREC', 'f16x3'), 'lib_sha16': hashlib.sha256(open(lib, 'rb').read()).hexdigest()[:16],
       'launches': [len(fe), len(wr)],
       'fetch_kb_raw_per_launch': sum(fe) / len(fe), 'write_kb_per_launch': sum(wr) / len(wr)}
res['fetch_bytes_raw_per_launch'] = int(res['fetch_kb_raw_per_launch'] * 1024)
res['write_bytes_per_launch'] = int(res['write_kb_per_launch'] * 1024)
res['fetch_rule'] = ('x2 (whole-line streaming reads, gfx950 correction; calibrated on pw_x3: 0.506x)' if wide
                     else 'raw (uncalibrated read pattern: no correction)')
res['hbm_bytes_per_launch'] = int((2 if wide else 1) * res['fetch_bytes_raw_per_launch'] + res['write_bytes_per_launch'])
res['note'] = 'KB = 1024 B; hbm = FETCH (rule above) + WRITE'
json.dump(res, open(out, 'w'), indent=1)
print(json.dumps(res))
