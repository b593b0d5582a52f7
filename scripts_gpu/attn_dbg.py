"""Per-launch time of the fused f16x3 attention layers at B = 64 (HIP events over 20
launches of extdm_attn_layer, incl. the layer's x -> out copy): STW C = 64 unshifted /
shifted (level 0), STW C = 128 shifted (level 1, downs.1.1) and init_temporal_attn. EXTDM_LIB picks
the library (A/B runs); EXTDM_X3_DBG=8 drops the epilogue loads / stores (timing only)."""
import importlib
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from tests.golden_inputs import CONFIGS, PKG, make_sd  # noqa: E402

pkg = importlib.import_module(PKG)
cfg = CONFIGS['bair']
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
h = pkg._lib.Handle(cfg, 1000, B, 0, precision='f16x3')
sd = make_sd(cfg)
sd.update(pkg.schedule_buffers(1000))
h.load_state(sd)
h.finalize()
dev = torch.device('cuda:0')
out_s = []
for prefix, level, shifted in [('downs.0.1', 0, False), ('downs.0.3', 0, True), ('downs.1.1', 1, True),
                               ('init_temporal_attn', 0, None)]:
    C = cfg.dim * (1 if level == 0 else cfg.dim_mults[level])
    L = cfg.latent >> level
    x = torch.randn(B, C, 16, L, L, device=dev)
    out = torch.empty_like(x)
    h.attn_layer(prefix, x, out, shifted=bool(shifted))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        h.attn_layer(prefix, x, out, shifted=bool(shifted))
    e1.record()
    torch.cuda.synchronize()
    out_s.append(f'{prefix}: {e0.elapsed_time(e1) / reps:.3f} ms')
lib = os.environ.get('EXTDM_LIB', 'in-tree')
print(f"lib={lib} dbg={os.environ.get('EXTDM_X3_DBG', '0')} B={B}: " + '  '.join(out_s), flush=True)
