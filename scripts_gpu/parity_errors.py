"""Fold a GPU suite run's parity log (EXTDM_PARITY_LOG lines, tests/parity_log.py) into one JSON:
per test and check, the achieved max-abs error, its bar and the bar's margin (bar / err).
Usage: parity_errors.py LOG.jsonl OUT.json [lib_sha16]"""
import json
import sys

rows = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
out = {'lib_sha16': sys.argv[3] if len(sys.argv) > 3 else None, 'checks': []}
for r in rows:
    r['margin'] = (r['bar'] / r['err']) if r['err'] > 0 else None
    out['checks'].append(r)
out['n_checks'] = len(rows)
out['min_margin'] = min((r['margin'] for r in rows if r['margin']), default=None)
json.dump(out, open(sys.argv[2], 'w'), indent=1)
print(f"{len(rows)} checks; smallest margin {out['min_margin']}")
for r in sorted(rows, key=lambda r: r['margin'] or 1e30)[:15]:
    print(f"  {r['margin'] or 0:9.1f}x  err {r['err']:.3e} bar {r['bar']:.1e}  {r['test']} {r['what']}")
