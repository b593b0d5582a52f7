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


def unet_config(cfg_name):
    """The UnetConfig bench.py's FlowDiffusion builds for the workload (round 6: read from the
    model itself — the hard-coded latent / fea_size table had SMMNIST at 64 / 64 and Cityscapes'
    fea_size at 32, not the bench's 32 / 32 and 16)."""
    a = bench.parse(['--config', cfg_name])
    w = bench.WORKLOADS[cfg_name]
    wrapper, arch = pkg.configs.dm_arch(cfg_name)
    cfg = pkg.configs.dm_config(cfg_name, pred_frames=a.tp, sampling_timesteps=a.sampling_steps,
                                estimate_occlusion_map=w['occ'])
    cfg['dataset_params']['frame_shape'] = w['image']
    fd = pkg.FlowDiffusion(config=cfg, is_train=False, Unet3D_architecture=arch, wrapper=wrapper,
                           timesteps=w['timesteps'])
    return fd.unet.ucfg


def make(cfg_name):
    w = bench.WORKLOADS[cfg_name]
    ucfg = unet_config(cfg_name)
    prec = os.environ.get('PREC') or w['precision'] or pkg._lib.DEFAULT_PRECISION
    B = int(os.environ.get('B', w['batch']))
    torch.cuda.set_device(0)
    sd = pkg.weights.synth_state_dict(pkg.spec.unet_spec(ucfg), seed=1234, window=tuple(ucfg.window))
    sd.update(pkg.schedule_buffers(1000))
    h = pkg._lib.Handle(ucfg, 1000, B, 0, precision=prec)
    h.load_state(sd)
    h.finalize()
    return h, B, prec
