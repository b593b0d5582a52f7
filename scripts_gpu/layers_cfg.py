"""Time extdm_bench_layer ids on the denoiser of a BASELINE workload (bench.py WORKLOADS: its
UnetConfig, per-GPU batch and precision). Usage: layers_cfg.py CONFIG IDS [ITERS]
(e.g. `layers_cfg.py kth 6,7`); A/B through the environment (EXTDM_NO_STW64=1 ...)."""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402

cfg_name = sys.argv[1]
ids = [int(v) for v in sys.argv[2].split(',')]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
pkg = importlib.import_module(bench.PKG)
w = bench.WORKLOADS[cfg_name]
_, arch = pkg.configs.dm_arch(cfg_name)
lat = {'bair': 32, 'kth': 32, 'smmnist': 64, 'cityscapes': 32, 'ucf': 128}[cfg_name]
fs = {'bair': 16, 'kth': 16, 'smmnist': 64, 'cityscapes': 32, 'ucf': 64}[cfg_name]
ucfg = pkg.spec.UnetConfig.for_arch(arch, tc=w['tc'], tp=w['tp'], latent=lat, fea_size=fs)
prec = os.environ.get('PREC') or w['precision'] or pkg._lib.DEFAULT_PRECISION
B = int(os.environ.get('B', w['batch']))
torch.cuda.set_device(0)
sd = pkg.weights.synth_state_dict(pkg.spec.unet_spec(ucfg), seed=1234, window=tuple(ucfg.window))
sd.update(pkg.schedule_buffers(1000))
h = pkg._lib.Handle(ucfg, 1000, B, 0, precision=prec)
h.load_state(sd)
h.finalize()
h.bench_layer(B, ids[0], 5)
for layer in ids:
    ms, flops = h.bench_layer(B, layer, iters)
    print(f'{cfg_name} {prec} B={B} layer {layer}: {ms * 1e3:9.1f} us/launch, {flops / ms / 1e9:7.1f} TFLOP/s '
          f'env={ {k: v for k, v in os.environ.items() if k.startswith("EXTDM_")} }', flush=True)
