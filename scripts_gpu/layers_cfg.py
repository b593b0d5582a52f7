"""Time extdm_bench_layer ids on the denoiser of a BASELINE workload (cfg_handle.py: its
UnetConfig, per-GPU batch and precision). Usage: layers_cfg.py CONFIG IDS [ITERS]
(e.g. `layers_cfg.py kth 6,7`); A/B through the environment (EXTDM_NO_STW64=1 ...)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import cfg_handle  # noqa: E402

cfg_name = sys.argv[1]
ids = [int(v) for v in sys.argv[2].split(',')]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
h, B, prec = cfg_handle.make(cfg_name)
h.bench_layer(B, ids[0], 5)
for layer in ids:
    ms, flops = h.bench_layer(B, layer, iters)
    print(f'{cfg_name} {prec} B={B} layer {layer}: {ms * 1e3:9.1f} us/launch, {flops / ms / 1e9:7.1f} TFLOP/s '
          f'{h.bench_layer_kernel(layer)} env={ {k: v for k, v in os.environ.items() if k.startswith("EXTDM_")} }',
          flush=True)
