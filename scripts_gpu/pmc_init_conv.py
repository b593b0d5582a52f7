"""init_conv in isolation for the PMC passes (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE):
the BAIR u12 handle at the bench batch, `iters` launches of the (1,7,7) 512->64 conv
exactly as the forward issues it (extdm_bench_layer layer 0)."""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
layer = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # extdm_bench_layer id (0 = init_conv)
pkg = importlib.import_module('140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd')
torch.cuda.set_device(0)
ucfg = pkg.spec.UnetConfig()
h = pkg._lib.Handle(ucfg, 1000, B, 0)
sd = pkg.weights.synth_state_dict(pkg.spec.unet_spec(ucfg), seed=1234)
sd.update(pkg.schedule_buffers(1000))
h.load_state(sd)
h.finalize()
ms, flops = h.bench_layer(B, layer, iters)
print(f'layer {layer} B={B}: {ms:.3f} ms/launch, {flops / ms / 1e9:.1f} TFLOP/s')
