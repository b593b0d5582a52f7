"""Where does the f16x3 window attention (C = 64) differ from the oracle? Error per window,
with the window's wave slot in its block (gidx % NW), repeated runs for determinism."""
import importlib
import os
import sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from tests.golden_inputs import CONFIGS, PKG, make_sd  # noqa: E402
from oracle import extdm_oracle as O  # noqa: E402

pkg = importlib.import_module(PKG)
cfg = CONFIGS['bair']
prec = sys.argv[1] if len(sys.argv) > 1 else 'f16x3'
NB = int(os.environ.get('DIAG_B', '2'))
h = pkg._lib.Handle(cfg, 1000, max(NB, 2), 0, precision=prec)
sd = make_sd(cfg)
sd.update(pkg.schedule_buffers(1000))
h.load_state(sd)
h.finalize()
dev = torch.device('cuda:0')
nw = int(os.environ.get('EXTDM_X3_ATTN_NW', '8'))
for prefix, level in [('init_temporal_attn', 0), ('downs.0.3', 0)]:
    C = cfg.dim * (1 if level == 0 else cfg.dim_mults[level])
    L = cfg.latent >> level
    gen = torch.Generator().manual_seed(5 + level)
    x = torch.randn(NB, C, cfg.frames, L, L, generator=gen) * 1.5 + 0.3
    win = tuple(cfg.window)
    if prefix == 'init_temporal_attn':
        ref = O.temporal_attention(sd, prefix, x, O.time_pos_bias(sd, cfg.frames), cfg.heads, cfg.dim_head)
    else:
        ref = O.stw_attention(sd, prefix, x, win, (0, 0, 0), cfg.heads, cfg.dim_head)
    outs = []
    for rep in range(3):
        out = torch.empty(x.shape, device=dev)
        h.attn_layer(prefix, x.to(dev), out, shifted=False)
        torch.cuda.synchronize()
        outs.append(out.cpu())
    print(prefix, 'B', NB, 'C', C, 'L', L, 'T', cfg.frames, 'win', win, 'nw', nw)
    e0 = (outs[0] - ref).abs()
    print(' err by frame', np.round(e0.amax(dim=(0, 1, 3, 4)).numpy(), 6).tolist())
    print(' err by row', np.round(e0.amax(dim=(0, 1, 2, 4)).numpy(), 6).tolist())
    print(' err by channel', np.round(e0.amax(dim=(0, 2, 3, 4)).numpy(), 6).tolist())
    print(' rep errs', [float((o - ref).abs().max()) for o in outs],
          'rep-to-rep', float((outs[0] - outs[1]).abs().max()), float((outs[0] - outs[2]).abs().max()))
    e = (outs[0] - ref).abs()  # [B, C, T, L, L]
    B, _, T, H, W = e.shape
    nd, nh, nwn = -(-T // win[0]), -(-H // win[1]), -(-W // win[2])
    per = np.zeros((B, nd, nh, nwn))
    for b in range(B):
        for d in range(nd):
            for i in range(nh):
                for j in range(nwn):
                    blk = e[b, :, d * win[0]:(d + 1) * win[0], i * win[1]:(i + 1) * win[1], j * win[2]:(j + 1) * win[2]]
                    per[b, d, i, j] = float(blk.max())
    flat = per.reshape(-1)
    gpb = nd * nh * nwn
    idx = np.argsort(-flat)[:12]
    print(' worst windows (gidx, gidx%nw, err):', [(int(k), int(k % nw), round(float(flat[k]), 6)) for k in idx])
    slots = np.zeros(nw)
    for k in range(flat.size):
        slots[k % nw] = max(slots[k % nw], flat[k])
    print(' max err per wave slot:', np.round(slots, 6).tolist())
    print(' windows with err > 2e-5:', int((flat > 2e-5).sum()), 'of', flat.size, 'groups/sample', gpb)
    ch = e.amax(dim=(0, 2, 3, 4))
    continue
    print(' err per channel (max over tokens):', np.round(ch.numpy(), 6).tolist()[:64])
