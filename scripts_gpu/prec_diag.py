"""Which f16x3 layer family loses precision at a small activation scale: the BAIR Unet3D at
B = 1 with tests/test_gpu_precision.scaled_sd(s), eps against the fp64 oracle, once per env
toggle that routes a family to its fp32 kernels (each toggle in a fresh process).
Usage: prec_diag.py S"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
s = float(sys.argv[1]) if len(sys.argv) > 1 else 1e-3
ref_path = f'/tmp/prec_ref_{s:g}.pt'
if len(sys.argv) > 2 and sys.argv[2] == 'child':
    import torch
    from tests.golden_inputs import CONFIGS, unet_inputs
    from tests import test_gpu_precision as T
    cfg = CONFIGS['bair']
    x, t, cond, fea = unet_inputs(cfg, B=1)
    x, cond, fea = x * s, cond * s, fea * s
    sd = T.scaled_sd(cfg, s)
    ref = torch.load(ref_path, weights_only=True)
    h = T.pkg._lib.Handle(cfg, 1000, 1, 0, precision=os.environ.get('PREC', 'f16x3'))
    full = dict(sd)
    full.update(T.pkg.schedule_buffers(1000))
    h.load_state(full)
    h.finalize()
    h.range_flag(reset=True)
    g = T.gpu_eps(h, x, t, cond, fea).double()
    d = g - ref['ref']
    print(json.dumps({'max': d.abs().max().item(), 'rms': d.pow(2).mean().sqrt().item(), 'flag': h.range_flag(),
                      'cpu_max': ref['cpu_max'], 'cpu_rms': ref['cpu_rms']}))
    sys.exit(0)
import torch
from tests.golden_inputs import CONFIGS, unet_inputs
from tests import test_gpu_precision as T
from oracle import extdm_oracle as O
cfg = CONFIGS['bair']
x, t, cond, fea = unet_inputs(cfg, B=1)
x, cond, fea = x * s, cond * s, fea * s
sd = T.scaled_sd(cfg, s)
ref = T._fp64_eps(cfg, x, t, cond, fea, sd=sd)
with torch.no_grad():
    c32 = O.unet_forward(sd, cfg.as_dict(), x, t, cond, fea).double()
d = c32 - ref
torch.save({'ref': ref, 'cpu_max': d.abs().max().item(), 'cpu_rms': d.pow(2).mean().sqrt().item()}, ref_path)
for name, env in [('f16x3', {}), ('fp32', {'PREC': 'fp32'}), ('no_x3_attn', {'EXTDM_NO_X3_ATTN': '1'}),
                  ('no_x3_core', {'EXTDM_NO_X3_CORE': '1'}), ('no_x3op', {'EXTDM_NO_X3OP': '1'}),
                  ('no_x3_stw', {'EXTDM_NO_X3_STW': '1'}), ('no_x3_temporal', {'EXTDM_NO_X3_TEMPORAL': '1'})]:
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, __file__, str(s), 'child'], env=e, capture_output=True, text=True, timeout=300)
    line = r.stdout.strip().split('\n')[-1] if r.stdout.strip() else r.stderr[-300:]
    print(f's={s:g} {name:12s} {line}', flush=True)
