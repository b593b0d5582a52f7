"""Pin the LFAE encoder / sample_one_video oracle (oracle/lfae_oracle.py) against
the reference's own outputs (tests/golden/lfae.npz, make_golden.py --lfae) and
the 2x2 SVD restatement against torch.svd."""
import dataclasses
import json
import os

import numpy as np
import pytest
import torch

from oracle import extdm_oracle as O
from oracle import lfae_oracle as LO
from tests.golden_inputs import LFAE_CFG, FD_UNET, PKG, make_lfae_sd, make_sd, video_inputs

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def gold():
    return np.load(os.path.join(GOLD, 'lfae.npz'))


def flat_sd(lc):
    sds = make_lfae_sd(lc)
    return {f'{k}.{n}': v for k, sd in sds.items() for n, v in sd.items()}


def lcfg(occ):
    return dataclasses.replace(LFAE_CFG, pf_estimate_occlusion_map=occ)


def test_svd2_matches_torch_svd_signs():
    g = torch.Generator().manual_seed(5)
    a = torch.randn(3000, 2, 2, generator=g)
    c = a @ a.transpose(1, 2) * torch.rand(3000, 1, 1, generator=g)
    # plus exact-diagonal, equal-diagonal and rank-one cases
    extra = torch.tensor([[[2., 0.], [0., 1.]], [[1., 0.], [0., 2.]], [[1., .5], [.5, 1.]], [[1., -.5], [-.5, 1.]],
                          [[4., 2.], [2., 1.]], [[1e-4, 0.], [0., 1e-4]]])
    c = torch.cat([c, extra])
    u, s, _ = torch.svd(c)
    for i in range(c.shape[0]):
        uu, ss = LO.svd2(c[i].numpy())
        np.testing.assert_allclose(uu, u[i].numpy(), atol=2e-5)
        # singular values to rounding relative to the matrix norm
        np.testing.assert_allclose(ss, s[i].numpy(), rtol=2e-5, atol=2e-6 * float(s[i, 0]))


def test_lfae_keys_match_reference():
    spec = __import__('importlib').import_module(PKG + '.spec')
    keys = json.load(open(os.path.join(GOLD, 'lfae_keys.json')))
    for occ, tag in ((True, 'occ'), (False, 'noocc')):
        lc = lcfg(occ)
        mine = {'generator': spec.generator_spec(lc.generator(), lfae=lc),
                'region_predictor': spec.region_predictor_spec(lc), 'bg_predictor': spec.bg_predictor_spec(lc)}
        for name, sp in mine.items():
            assert [[n, list(s)] for n, s, _ in sp] == keys[f'{name}_{tag}'], (name, tag)


def test_region_and_bg_predictors():
    g = gold()
    lc = lcfg(True)
    sd = flat_sd(lc)
    vid = video_inputs()
    with torch.no_grad():
        src = LO.region_predictor(sd, lc, vid[:, :, 1])
        drv = LO.region_predictor(sd, lc, vid[:, :, 0])
        bg = LO.bg_predictor(sd, lc, vid[:, :, 1], vid[:, :, 0])
        bott = LO.bottleneck(sd, lc, vid[:, :, 0])
    for tag, p in (('src', src), ('drv', drv)):
        np.testing.assert_allclose(p['heatmap'].numpy(), g[f'rp_{tag}_heatmap'], rtol=1e-4, atol=1e-8)
        np.testing.assert_allclose(p['shift'].numpy(), g[f'rp_{tag}_shift'], atol=2e-6)
        np.testing.assert_allclose(p['covar'].numpy(), g[f'rp_{tag}_covar'], atol=2e-6)
        np.testing.assert_allclose(p['affine'].numpy(), g[f'rp_{tag}_affine'], atol=2e-5)
    np.testing.assert_allclose(bg.numpy(), g['bg'], atol=1e-5)
    np.testing.assert_allclose(bott.numpy(), g['bottle'], atol=1e-5)


@pytest.mark.parametrize('occ', [True, False])
def test_generator_forward(occ):
    g = gold()
    lc = lcfg(occ)
    sd = flat_sd(lc)
    vid = video_inputs()
    tag = 'occ' if occ else 'noocc'
    with torch.no_grad():
        src = LO.region_predictor(sd, lc, vid[:, :, 1])
        drv = LO.region_predictor(sd, lc, vid[:, :, 0])
        bg = LO.bg_predictor(sd, lc, vid[:, :, 1], vid[:, :, 0])
        out = LO.generator_forward(sd, lc, vid[:, :, 1], drv, src, bg)
    for k, v in out.items():
        np.testing.assert_allclose(v.numpy(), g[f'gen_{tag}_{k}'], atol=5e-5, err_msg=k)


@pytest.mark.parametrize('occ', [True, False])
def test_sample_one_video(occ):
    """Encoder round + DDIM-10 (reference RNG order) + decode == the reference's
    FlowDiffusion.sample_one_video."""
    g = gold()
    lc = lcfg(occ)
    sd = flat_sd(lc)
    usd = make_sd(FD_UNET)
    vid = video_inputs()
    tag = 'occ' if occ else 'noocc'
    with torch.no_grad():
        ret, x_cond, fea, ref = LO.encode_round(sd, lc, FD_UNET, vid)
        torch.manual_seed(31)
        shape = (vid.shape[0], 3, FD_UNET.tp, FD_UNET.latent, FD_UNET.latent)
        xT = torch.randn(shape)
        noises = [torch.randn(shape) for _ in range(10)]
        den = lambda xx, tt: O.unet_forward(usd, FD_UNET.as_dict(), xx, tt, x_cond, fea)
        pred = O.ddim_sample(O.schedule(1000), den, xT, noises, 10)
        ret = LO.decode_round(sd, lc, FD_UNET, ret, pred, ref)
    keys = [k[len(f'sov_{tag}_'):] for k in g.files if k.startswith(f'sov_{tag}_')]
    assert sorted(keys) == sorted(ret)
    for k in keys:
        np.testing.assert_allclose(ret[k].numpy(), g[f'sov_{tag}_{k}'], atol=1e-4, err_msg=k)
