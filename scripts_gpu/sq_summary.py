"""Per-wave instruction mix and stall fractions of each bench layer's kernel from the SQ passes
of scripts_gpu/r04_sq.sh (pmc_table.py text). Usage: sq_summary.py TABLE.txt"""
import sys

KERN = {'0': 'conv_x3_kernel<5', '1': 'conv_x3_kernel<3', '5': 'conv_x3_kernel<3', '6': 'attn_x3_kernel',
        '7': 'attn_x3_kernel', '8': 'cross_attn', '9': 'xpath_x3', '10': 'noise_pool', '11': 'fea_side',
        '12': 'conv_x3_kernel<1', '13': 'conv_x3_kernel<1', '4': 'conv_x3_kernel<1'}
txt = open(sys.argv[1]).read()
rows = {}
for b in txt.split('=== layer ')[1:]:
    L = b.split('\n')[0].strip()
    cur, ks = None, {}
    for line in b.split('\n')[1:]:
        if line.startswith('   '):
            p = line.split()
            if cur:
                ks[cur][p[0]] = float(p[1])
        elif line.strip() and not line.startswith(('pass', '===')):
            cur = line.strip()
            ks.setdefault(cur, {})
    cand = [k for k in ks if KERN.get(L, '@') in k]
    if not cand:
        continue
    k = max(cand, key=lambda k: ks[k].get('SQ_WAVES', 0))
    c = ks[k]
    w = c.get('SQ_WAVES', 1)
    mf = max(1.0, c.get('SQ_INSTS_MFMA', 0) / w)
    wc = c.get('SQ_WAVE_CYCLES', 1)
    rows[L] = (k, c)
    print(f'layer {L}: {k[:100]}')
    print('  per wave  VALU %6.0f  SALU %6.0f  LDS %5.0f  VMEM %5.0f  MFMA %5.0f   waves %d' %
          tuple([c.get(x, 0) / w for x in ['SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_LDS', 'SQ_INSTS_VMEM',
                                           'SQ_INSTS_MFMA']] + [w]))
    print('  per MFMA  VALU %5.2f  SALU %5.2f  LDS %5.2f  VMEM %5.2f' %
          tuple(c.get(x, 0) / w / mf for x in ['SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_LDS', 'SQ_INSTS_VMEM']))
    print('  of wave cycles: WAIT_INST_ANY %.2f  WAIT_ANY %.2f  ACTIVE_INST_ANY %.2f  WAIT_INST_LDS %.3f;'
          '  LDS bank conflict / LDS active %.2f' %
          (c.get('SQ_WAIT_INST_ANY', 0) / wc, c.get('SQ_WAIT_ANY', 0) / wc, c.get('SQ_ACTIVE_INST_ANY', 0) / wc,
           c.get('SQ_WAIT_INST_LDS', 0) / wc, c.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, c.get('SQ_LDS_IDX_ACTIVE', 1))))
