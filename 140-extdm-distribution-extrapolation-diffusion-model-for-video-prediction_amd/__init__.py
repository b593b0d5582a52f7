"""MI355X-native ExtDM sampling path (gfx950 HIP kernels behind a C ABI).

Import with importlib (the directory name is not a Python identifier):
    pkg = importlib.import_module('140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd')
"""
from . import spec, weights, configs, dist, metrics, _lib  # noqa: F401
from .models import (Unet3D, Unet3DAda, Unet3DAdaU22, Unet3DWoRef, UNET3D_BY_MODULE, GaussianDiffusion,  # noqa: F401
                     schedule_buffers, ddim_time_pairs)
from .lfae import (Generator, RegionPredictor, BGMotionPredictor, FlowDiffusion,  # noqa: F401
                   FlowDiffusionMultiWRef, FlowDiffusionMultiWRefU22, FlowDiffusionMulti1248,
                   FLOW_DIFFUSION_BY_MODULE, autoregressive_sample)
