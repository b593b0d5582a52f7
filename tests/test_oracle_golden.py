"""Pin the CPU oracle (oracle/extdm_oracle.py) against golden vectors produced
by running the reference itself (tests/golden/make_golden.py)."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import extdm_oracle as O
from tests.golden_inputs import (CONFIGS, GEN_CFG, GOLDEN_BATCH, unet_inputs, decoder_inputs, make_sd, make_gen_sd,
                                 PKG)

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def load(name):
    return np.load(os.path.join(GOLD, name))


def test_schedule_matches_reference_buffers():
    g = load('schedule_1000.npz')
    s = O.schedule(1000)
    for k, v in s.items():
        np.testing.assert_array_equal(v.numpy(), g[k], err_msg=k)


def test_ddim_pairs():
    g = json.load(open(os.path.join(GOLD, 'ddim_pairs.json')))
    for S, pairs in g.items():
        assert [list(p) for p in O.ddim_pairs(1000, int(S))] == pairs


def test_quantile_cases():
    g = load('quantile.npz')
    for k in ('ties', 'random', 'spike', 'tiny', 'lowval'):
        out = torch.quantile(torch.from_numpy(g[k + '_in']), 0.9, dim=-1).numpy()
        np.testing.assert_array_equal(out, g[k + '_out'])


@pytest.mark.parametrize('name', list(CONFIGS))
def test_unet_forward(name):
    """All four denoisers (u12, ada, ada_u22, wo_ref) at reduced and dataset sizes."""
    cfg = CONFIGS[name]
    sd = make_sd(cfg)
    x, t, cond, fea = unet_inputs(cfg, B=GOLDEN_BATCH.get(name, 2))
    with torch.no_grad():
        eps = O.unet_forward(sd, cfg.as_dict(), x, t, cond, fea)
    g = load(f'unet_{name}.npz')
    np.testing.assert_allclose(eps.numpy(), g['eps'], atol=2e-5, rtol=1e-5)


def test_sampler_steps_small():
    cfg = CONFIGS['small']
    sd = make_sd(cfg)
    x, t, cond, fea = unet_inputs(cfg)
    sch = O.schedule(1000)
    g = load('sampler_small.npz')
    den = lambda xx, tt: O.unet_forward(sd, cfg.as_dict(), xx, tt, cond, fea)
    with torch.no_grad():
        for ti in (999, 500, 1, 0):
            tt = torch.full((2,), ti, dtype=torch.long)
            torch.manual_seed(100 + ti)
            noise = torch.randn(x.shape)
            out = O.ddpm_step(sch, x, den(x, tt), tt, noise)
            np.testing.assert_allclose(out.numpy(), g[f'p_sample_{ti}'], atol=2e-5, rtol=1e-5)
        # DDPM chain over a 10-step schedule, noise in the reference's RNG order
        assert int(g['p_sample_loop_raises']) == 1
        s10 = O.schedule(10)
        torch.manual_seed(7)
        xT = torch.randn(x.shape)
        noises = [torch.randn(x.shape) for _ in range(10)]
        out = O.p_sample_loop(s10, den, xT, noises)
        np.testing.assert_allclose(out.numpy(), g['ddpm10'], atol=5e-5, rtol=1e-5)
        torch.manual_seed(11)
        xT = torch.randn(x.shape)
        noises = [torch.randn(x.shape) for _ in range(10)]
        out = O.ddim_sample(sch, den, xT, noises, 10)
        np.testing.assert_allclose(out.numpy(), g['ddim10'], atol=5e-5, rtol=1e-5)


def test_decoder():
    sd = make_gen_sd()
    src, flow, occ = decoder_inputs()
    g = load('decoder.npz')
    with torch.no_grad():
        p1, d1 = O.decoder_forward(sd, GEN_CFG.as_dict(), src, flow, occ)
        p0, d0 = O.decoder_forward(sd, GEN_CFG.as_dict(), src, flow, None)
    np.testing.assert_allclose(p1.numpy(), g['pred_occ'], atol=1e-5)
    np.testing.assert_allclose(d1.numpy(), g['deformed'], atol=1e-6)
    np.testing.assert_array_equal(p0.numpy(), g['pred_noocc'])
    # quirk: without occlusion the prediction IS the warped source
    np.testing.assert_array_equal(p0.numpy(), d0.numpy())
