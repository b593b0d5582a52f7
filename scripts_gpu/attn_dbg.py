"""Per-launch time of the f16x3 STW C = 64 and temporal attention layers at B = 64 (HIP
events over 20 launches). Run once per EXTDM_X3_DBG value: 4 = no x loads, 8 = no
epilogue loads / stores (timing-only switches of stw_x3.hip)."""
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
h = pkg._lib.Handle(cfg, 1000, B, 0, precision='f16x3')
sd = make_sd(cfg)
sd.update(pkg.schedule_buffers(1000))
h.load_state(sd)
h.finalize()
dev = torch.device('cuda:0')
out_s = []
for prefix, level, shifted in [('downs.0.1', 0, False), ('downs.0.3', 0, True), ('init_temporal_attn', 0, None)]:
    C = cfg.dim
    L = cfg.latent >> level
    x = torch.randn(B, C, 16, L, L, device=dev)
    out = torch.empty_like(x)
    h.attn_layer(prefix, x, out, shifted=bool(shifted))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        h.attn_layer(prefix, x, out, shifted=bool(shifted))
    e1.record()
    torch.cuda.synchronize()
    out_s.append(f'{prefix}: {e0.elapsed_time(e1) / 20:.3f} ms')
print(f"dbg={os.environ.get('EXTDM_X3_DBG', '0')} B={B}: " + '  '.join(out_s), flush=True)
