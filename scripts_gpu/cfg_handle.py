"""The denoiser handle of a BASELINE workload for the GPU measurement scripts: bench.py WORKLOADS'
UnetConfig (latent / fea_size of the wrapper), per-GPU batch (B env overrides) and precision (PREC
env overrides), synthetic weights (seed 1234)."""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402

pkg = importlib.import_module(bench.PKG)
LATENT = {'bair': (32, 16), 'kth': (32, 16), 'smmnist': (64, 64), 'cityscapes': (32, 32), 'ucf': (128, 64)}


def make(cfg_name):
    w = bench.WORKLOADS[cfg_name]
    _, arch = pkg.configs.dm_arch(cfg_name)
    lat, fs = LATENT[cfg_name]
    ucfg = pkg.spec.UnetConfig.for_arch(arch, tc=w['tc'], tp=w['tp'], latent=lat, fea_size=fs)
    prec = os.environ.get('PREC') or w['precision'] or pkg._lib.DEFAULT_PRECISION
    B = int(os.environ.get('B', w['batch']))
    torch.cuda.set_device(0)
    sd = pkg.weights.synth_state_dict(pkg.spec.unet_spec(ucfg), seed=1234, window=tuple(ucfg.window))
    sd.update(pkg.schedule_buffers(1000))
    h = pkg._lib.Handle(ucfg, 1000, B, 0, precision=prec)
    h.load_state(sd)
    h.finalize()
    return h, B, prec
