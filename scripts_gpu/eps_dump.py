"""One BAIR Unet forward (full u12, B = 8, seeded inputs and weights) on the library EXTDM_LIB
selects, eps saved to the given path: two runs on two libraries compare bitwise (an A/B that must
not change results). Usage: eps_dump.py OUT.pt"""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from tests.golden_inputs import CONFIGS, PKG, make_sd, unet_inputs  # noqa: E402

pkg = importlib.import_module(PKG)
cfg = CONFIGS['bair']
B = 8
h = pkg._lib.Handle(cfg, 1000, B, 0)
sd = make_sd(cfg)
sd.update(pkg.schedule_buffers(1000))
h.load_state(sd)
h.finalize()
x, t, cond, fea = unet_inputs(cfg, B=B, seed=29)
dev = torch.device('cuda:0')
eps = torch.empty(x.shape, device=dev)
h.unet_forward(x.to(dev), torch.full((B,), 611, dtype=torch.long).to(dev), cond.to(dev), fea.to(dev), eps)
torch.cuda.synchronize()
torch.save(eps.cpu(), sys.argv[1])
print('saved', sys.argv[1], pkg._lib.LIB_PATH)
