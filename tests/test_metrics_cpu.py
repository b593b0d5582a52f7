"""Metric oracle and host-side metric API against the reference's own metric code
(tests/golden/metrics.npz; make_golden.py --metrics). No GPU."""
import importlib
import os

import numpy as np
import pytest

from tests.golden_inputs import PKG, METRIC_CASES, metric_videos, metric_feats
from oracle import metrics_oracle as mo

M = importlib.import_module(PKG + '.metrics')
G = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'metrics.npz'))


@pytest.mark.parametrize('name', list(METRIC_CASES))
def test_oracle_frame_metrics_vs_reference(name):
    a, b = metric_videos(name)
    p, s = mo.frame_metrics(a.numpy(), b.numpy())
    # the reference's mse is a float32 numpy mean: ~1e-7 relative -> < 1e-5 dB
    np.testing.assert_allclose(p, G[f'{name}_psnr'], rtol=0, atol=1e-5)
    np.testing.assert_allclose(s, G[f'{name}_ssim'], rtol=0, atol=1e-12)
    assert np.max(np.mean(p, -1)) == pytest.approx(float(G[f'{name}_psnr2']), abs=1e-5)
    assert np.max(np.mean(s, -1)) == pytest.approx(float(G[f'{name}_ssim2']), abs=1e-12)
    np.testing.assert_allclose(np.mean(p, 0), G[f'{name}_psnr_avg'], atol=1e-5)
    np.testing.assert_allclose(np.std(s, 0), G[f'{name}_ssim_std'], atol=1e-12)


def test_frechet_distance_vs_reference():
    fake, real = metric_feats()
    assert M.frechet_distance(fake, real) == pytest.approx(float(G['fd']), rel=1e-10)
    assert M.frechet_distance(fake[:1], real) == pytest.approx(float(G['fd_single']), rel=1e-6)
    assert abs(M.frechet_distance(real, real) - float(G['fd_self'])) < 1e-6


def test_select_best_is_l1_argmin():
    g = np.random.Generator(np.random.PCG64(3))
    o = g.standard_normal((4, 400))
    r = g.standard_normal((4 * 3, 400))
    r[1 * 3 + 2] = o[1] + 1e-3  # clip 1's third sample is nearest
    idx = M.select_best(o, r, 3)
    ref = [int(np.argmin([np.abs(o[i] - r[i * 3 + k]).sum() for k in range(3)])) for i in range(4)]
    assert list(idx) == ref and idx[1] == 2


def test_metric_stuff_interval():
    import scipy.stats as st
    x = np.array([0.91, 0.88, 0.95, 0.9, 0.87])
    avg, std, c95 = M.metric_stuff(x)
    assert avg == pytest.approx(x.mean()) and std == pytest.approx(x.std())
    assert c95 == pytest.approx(1.959963984540054 * st.sem(x), rel=1e-9)
