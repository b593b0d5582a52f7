"""Three eager Unet3D forwards of a BASELINE workload's denoiser (cfg_handle.py: its UnetConfig,
bench batch and precision) for a rocprofv3 kernel trace; trace_order.py then lists the last forward's
dispatches in launch order. Usage: forward_trace_cfg.py CONFIG"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import cfg_handle  # noqa: E402
import torch  # noqa: E402
from tests.golden_inputs import unet_inputs  # noqa: E402

c = sys.argv[1]
ucfg = cfg_handle.unet_config(c)
h, B, prec = cfg_handle.make(c)
x, t, cond, fea = unet_inputs(ucfg, B=B)
dev = torch.device('cuda:0')
x, t, cond, fea = x.to(dev), t.to(dev), cond.to(dev), fea.to(dev)
out = torch.empty_like(x)
for _ in range(3):
    h.unet_forward(x, t, cond, fea, out)
torch.cuda.synchronize()
print('done', c, B, prec)
