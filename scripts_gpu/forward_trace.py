"""Three eager Unet3D forwards (BAIR u12, B = 64, f16x3) for a rocprofv3 kernel trace;
scripts_gpu/trace_order.py then lists the last forward's dispatches in launch order."""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from tests.golden_inputs import CONFIGS, make_sd, unet_inputs  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
pkg = importlib.import_module('140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd')
cfg = CONFIGS['bair']
h = pkg._lib.Handle(cfg, 1000, B, 0)
sd = make_sd(cfg)
sd.update(pkg.schedule_buffers(1000))
h.load_state(sd)
h.finalize()
x, t, cond, fea = unet_inputs(cfg, B=B)
dev = torch.device('cuda:0')
x, t, cond, fea = x.to(dev), t.to(dev), cond.to(dev), fea.to(dev)
out = torch.empty_like(x)
for _ in range(3):
    h.unet_forward(x, t, cond, fea, out)
    torch.cuda.synchronize()
print('ok', float(out.abs().mean()))
