"""Time the bench_layer convs (extdm_bench_layer ids 0-4) in both precisions at batch B."""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
precs = sys.argv[3].split(',') if len(sys.argv) > 3 else ['fp32', 'f16x3']
layers = [int(v) for v in sys.argv[4].split(',')] if len(sys.argv) > 4 else [0, 1, 2, 3, 4]
pkg = importlib.import_module('140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd')
torch.cuda.set_device(0)
ucfg = pkg.spec.UnetConfig()
sd = pkg.weights.synth_state_dict(pkg.spec.unet_spec(ucfg), seed=1234)
sd.update(pkg.schedule_buffers(1000))
for prec in precs:
    h = pkg._lib.Handle(ucfg, 1000, B, 0, precision=prec)
    h.load_state(sd)
    h.finalize()
    h.bench_layer(B, layers[0], iters)  # clock ramp
    for layer in layers:
        ms, flops = h.bench_layer(B, layer, iters)
        tag = os.environ.get('EXTDM_X3_NO_BX', '')
        print(f'{prec:6s} layer {layer} B={B}: {ms * 1e3:9.1f} us/launch, {flops / ms / 1e9:7.1f} TFLOP/s '
              f'{h.bench_layer_kernel(layer)} NO_BX={tag}', flush=True)
    del h
