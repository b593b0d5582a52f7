"""Isolate the f16x3 attention kernels: BAIR eps with x3 attention variants against the
golden, per env toggle (run once per setting in a fresh process)."""
import importlib
import os
import sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from tests.golden_inputs import CONFIGS, make_sd, unet_inputs  # noqa: E402
pkg = importlib.import_module('140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd')
name = sys.argv[1] if len(sys.argv) > 1 else 'bair'
cfg = CONFIGS[name]
h = pkg._lib.Handle(cfg, 1000, 2, 0, precision='f16x3')
sd = make_sd(cfg)
sd.update(pkg.schedule_buffers(1000))
h.load_state(sd)
h.finalize()
x, t, cond, fea = unet_inputs(cfg)
dev = torch.device('cuda:0')
out = torch.empty(x.shape, device=dev)
h.unet_forward(x.to(dev), t.to(dev), cond.to(dev), fea.to(dev), out)
torch.cuda.synchronize()
g = np.load(os.path.join(REPO, 'tests', 'golden', f'unet_{name}.npz'))['eps']
d = np.abs(out.cpu().numpy() - g)
env = {k: v for k, v in os.environ.items() if k.startswith('EXTDM_')}
print(name, env, 'max', d.max(), 'mean', d.mean(), 'range', h.range_flag())
