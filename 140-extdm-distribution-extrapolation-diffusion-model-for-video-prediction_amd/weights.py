"""Deterministic synthetic weights for the sampling path (no checkpoints are
available offline). NumPy PCG64, consumed in state_dict order, fan-in scaled.

Rules: conv/linear weights ~ N(0,1)/sqrt(fan_in); biases 0.1*N;
norm gains 1 + 0.1*N; bias tables 0.5*N; BN running stats positive-variance.
The reference zero-inits the MotionAdaptor extrapolators (u12:650-668); here
they are non-zero so the adaptor path is live. Deterministic buffers
(`relative_position_index`, rotary `freqs`, `num_batches_tracked`) keep their
reference values.
"""
import math

import numpy as np
import torch


def rel_pos_index(ws):
    """WindowAttention3D.relative_position_index (u12:436-451)."""
    c = np.stack(np.meshgrid(np.arange(ws[0]), np.arange(ws[1]), np.arange(ws[2]), indexing='ij')).reshape(3, -1)
    r = (c[:, :, None] - c[:, None, :]).transpose(1, 2, 0).copy()
    r[:, :, 0] += ws[0] - 1
    r[:, :, 1] += ws[1] - 1
    r[:, :, 2] += ws[2] - 1
    r[:, :, 0] *= (2 * ws[1] - 1) * (2 * ws[2] - 1)
    r[:, :, 1] *= (2 * ws[2] - 1)
    return r.sum(-1).astype(np.int64)


def rope_freqs(dim, theta=10000):
    """rotary-embedding-torch 0.8.3 `freqs` (computed with torch fp32 ops so the
    bits match the reference's parameter)."""
    return 1. / (theta ** (torch.arange(0, dim, 2)[:(dim // 2)].float() / dim))


def antialias_kernel(channels, k):
    """AntiAliasInterpolation2d.weight (util.py:224-254) for kernel size k; the
    sigma that yields k is (k - 1) / 8 for the configs' scales 1/2 and 1/4."""
    sigma = (k - 1) / 8
    grids = torch.meshgrid([torch.arange(k, dtype=torch.float32)] * 2, indexing='ij')
    kern = 1
    for g in grids:
        mean = (k - 1) / 2
        kern = kern * torch.exp(-(g - mean) ** 2 / (2 * sigma ** 2))
    kern = kern / torch.sum(kern)
    return kern.view(1, 1, k, k).repeat(channels, 1, 1, 1)


_BG_IDENTITY = {2: [0, 0], 6: [1, 0, 0, 0, 1, 0], 8: [1, 0, 0, 0, 1, 0, 0, 0]}


def synth_state_dict(spec, seed=1234, window=(2, 4, 4)):
    """Return an ordered dict name -> CPU torch tensor for `spec`."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = {}
    for name, shape, dtype in spec:
        leaf = name.rsplit('.', 1)[-1]
        if leaf == 'relative_position_index':
            sd[name] = torch.from_numpy(rel_pos_index(window)[:shape[0], :shape[1]].copy())
            continue
        if leaf == 'freqs':
            sd[name] = rope_freqs(shape[0] * 2)
            continue
        if leaf == 'num_batches_tracked':
            sd[name] = torch.tensor(0, dtype=torch.int64)
            continue
        if name.endswith('down.weight') and len(shape) == 4 and shape[1] == 1:
            sd[name] = antialias_kernel(shape[0], shape[2])
            continue
        n = int(np.prod(shape)) if len(shape) else 1
        z = rng.standard_normal(n, dtype=np.float32)
        if name.endswith('fc.bias') and n in _BG_IDENTITY:
            # BGMotionPredictor.fc starts at the identity transform (bg_motion_predictor.py:27-41);
            # keep it near there so the background grid stays in frame
            v = np.array(_BG_IDENTITY[n], np.float32) + 0.05 * z
            sd[name] = torch.from_numpy(v.astype(np.float32).reshape(shape))
            continue
        if name.endswith('regions.weight'):
            # RegionPredictor logits are divided by temperature 0.1: keep them O(1) so the
            # region heatmaps stay smooth (well-conditioned covariances)
            sd[name] = torch.from_numpy((0.2 * z / math.sqrt(int(np.prod(shape[1:])))).astype(np.float32)
                                        .reshape(shape))
            continue
        if name.endswith('fc.weight') and shape[0] in _BG_IDENTITY:
            sd[name] = torch.from_numpy((0.05 * z / math.sqrt(shape[1])).astype(np.float32).reshape(shape))
            continue
        if leaf == 'running_var':
            v = 0.5 + np.abs(z)
        elif leaf == 'running_mean':
            v = 0.1 * z
        elif leaf in ('relative_position_bias_table',) or name.startswith('time_rel_pos_bias'):
            v = 0.5 * z
        elif leaf == 'gamma' or (len(shape) == 1 and leaf == 'weight'):
            v = 1.0 + 0.1 * z
        elif len(shape) == 1:
            v = 0.1 * z
        else:
            fan_in = int(np.prod(shape[1:]))
            if name.startswith('ups.') and len(shape) == 5 and tuple(shape[2:]) == (1, 4, 4):
                # ConvTranspose3d weight is (Cin, Cout, kt, kh, kw): fan-in = Cin*k*k/4
                fan_in = shape[0] * shape[2] * shape[3] * shape[4] // 4
            v = z / math.sqrt(fan_in)
        sd[name] = torch.from_numpy(v.astype(np.float32).reshape(shape))
    return sd
