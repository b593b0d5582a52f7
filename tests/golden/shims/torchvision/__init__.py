"""Import-only stand-in for torchvision (absent here): VideoFlowDiffusion_multi_w_ref_u22.py
imports `models` for a Vgg19 perceptual loss that only training constructs (its
construction is commented out, :236-238); sampling never touches it."""
import types


def _vgg19(*a, **k):
    raise NotImplementedError('torchvision is not available in the golden harness (training-only Vgg19)')


models = types.SimpleNamespace(vgg19=_vgg19)
