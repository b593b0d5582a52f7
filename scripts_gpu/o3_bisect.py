"""A/B of the f16x3 attention builds (EXTDM_LIB selects the library): per layer,
the max error against the oracle and the max difference between 5 launches of the
same input; then the BAIR Unet3D forward against the reference golden, 3 launches.
Usage: EXTDM_LIB=... python scripts_gpu/o3_bisect.py TAG"""
import importlib
import json
import os
import sys

import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from tests.golden_inputs import CONFIGS, PKG, make_sd, unet_inputs  # noqa: E402
from tests.test_oracle_golden import load  # noqa: E402
from oracle import extdm_oracle as O  # noqa: E402

tag = sys.argv[1]
pkg = importlib.import_module(PKG)
dev = torch.device('cuda:0')
cfg = CONFIGS['bair']
B = 4
h = pkg._lib.Handle(cfg, 1000, B, 0, precision='f16x3')
sd = make_sd(cfg)
sd.update(pkg.schedule_buffers(1000))
h.load_state(sd)
h.finalize()
res = {'tag': tag, 'lib': pkg._lib.LIB_PATH, 'nw': os.environ.get('EXTDM_X3_ATTN_NW', '')}
for prefix, level, shifted in [('downs.0.1', 0, True), ('downs.0.3', 0, False), ('downs.1.1', 1, True),
                               ('init_temporal_attn', 0, None)]:
    C = cfg.dim * (1 if level == 0 else cfg.dim_mults[level])
    L = cfg.latent >> level
    gen = torch.Generator().manual_seed(5 + level)
    x = torch.randn(B, C, cfg.frames, L, L, generator=gen) * 1.5 + 0.3
    with torch.no_grad():
        if shifted is None:
            ref = O.temporal_attention(sd, prefix, x, O.time_pos_bias(sd, cfg.frames), cfg.heads, cfg.dim_head)
        else:
            win = tuple(cfg.window)
            ref = O.stw_attention(sd, prefix, x, win, tuple(w // 2 for w in win) if shifted else (0, 0, 0),
                                  cfg.heads, cfg.dim_head)
    outs = []
    xd = x.to(dev)
    for _ in range(5):
        out = torch.empty(x.shape, device=dev)
        h.attn_layer(prefix, xd, out, shifted=bool(shifted))
        torch.cuda.synchronize()
        outs.append(out.cpu())
    res[prefix] = {'err': float((outs[0] - ref).abs().max()),
                   'rep_diff': max(float((o - outs[0]).abs().max()) for o in outs[1:])}
x, t, cond, fea = unet_inputs(cfg)
g = load('unet_bair.npz')['eps']
eps = []
for _ in range(3):
    out = torch.empty(x.shape, device=dev)
    h.unet_forward(x.to(dev), t.to(dev), cond.to(dev), fea.to(dev), out)
    torch.cuda.synchronize()
    eps.append(out.cpu().numpy())
res['unet_bair'] = {'err': float(np.abs(eps[0] - g).max()),
                    'rep_diff': max(float(np.abs(e - eps[0]).max()) for e in eps[1:])}
print(json.dumps(res), flush=True)
