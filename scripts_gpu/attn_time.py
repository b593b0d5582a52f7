"""Per-launch time of the attention layers at the bench batch: fp32 fused kernels vs the
f16x3 kernels (EXTDM_NO_X3_ATTN read per call), HIP events around 10 launches."""
import importlib
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from tests.golden_inputs import CONFIGS, PKG, make_sd  # noqa: E402

pkg = importlib.import_module(PKG)
cfg = CONFIGS['bair']
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
h = pkg._lib.Handle(cfg, 1000, B, 0, precision='f16x3')
sd = make_sd(cfg)
sd.update(pkg.schedule_buffers(1000))
h.load_state(sd)
h.finalize()
dev = torch.device('cuda:0')
for prefix, level, shifted in [('downs.0.1', 0, True), ('init_temporal_attn', 0, None), ('downs.1.1', 1, True)]:
    C = cfg.dim * (1 if level == 0 else cfg.dim_mults[level])
    L = cfg.latent >> level
    x = torch.randn(B, C, 16, L, L, device=dev)
    out = torch.empty_like(x)
    res = {}
    for mode in ('0', '1'):
        os.environ["EXTDM_NO_X3_ATTN"] = "0" if mode == "1" else "1"
        h.attn_layer(prefix, x, out, shifted=bool(shifted))
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            h.attn_layer(prefix, x, out, shifted=bool(shifted))
        e1.record()
        torch.cuda.synchronize()
        res['x3' if mode == '1' else 'fp32'] = e0.elapsed_time(e1) / 10
    print(f'{prefix} B={B} C={C} L={L}: fp32 {res["fp32"]:.3f} ms  f16x3 {res["x3"]:.3f} ms  (incl. the x->out copy)')
