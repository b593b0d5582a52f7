"""Parity bars with their measured errors on record. Every tolerance check of the GPU parity tests
goes through check(err, bar, what): it asserts err <= bar and, with EXTDM_PARITY_LOG=<path>, appends
one JSON line {test, what, err, bar} — scripts_gpu/parity_errors.py folds a suite run's lines into
profiles/r0N_parity_errors.json, the measured errors the bars in tests/ are set from (about 3x the
largest measured error, within the SURVEY §8(c) contract)."""
import json
import os


def check(err, bar, what=''):
    err, bar = float(err), float(bar)
    test = os.environ.get('PYTEST_CURRENT_TEST', '?').split(' (')[0]
    path = os.environ.get('EXTDM_PARITY_LOG')
    if path:
        with open(path, 'a') as f:
            f.write(json.dumps({'test': test, 'what': what, 'err': err, 'bar': bar}) + '\n')
    print(f'parity {test} {what}: max|err| {err:.3e} (bar {bar:.1e})')
    assert err <= bar, (test, what, err, bar)
