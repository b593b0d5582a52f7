"""metrics.hip (extdm_frame_metrics) against the reference's metric code
(tests/golden/metrics.npz) and the numpy oracle.

The SSIM goldens come from the reference's ssim() running on tests/golden/shims/cv2, a
scipy restatement of cv2.getGaussianKernel / cv2.filter2D (OpenCV is absent here): the
1e-12 SSIM match pins the device kernel to the reference's formula and crop through that
shim's arithmetic — parity with OpenCV's own filter arithmetic is unpinned."""
import importlib
import os

import numpy as np
import pytest
import torch

from tests.golden_inputs import PKG, METRIC_CASES, metric_videos
from oracle import metrics_oracle as mo

pytestmark = pytest.mark.gpu
M = importlib.import_module(PKG + '.metrics')
G = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'metrics.npz'))


@pytest.mark.parametrize('name', list(METRIC_CASES))
def test_frame_metrics_vs_reference(name):
    a, b = metric_videos(name)
    p, s = M.frame_metrics(a.cuda(), b.cuda())
    p, s = p.cpu().numpy(), s.cpu().numpy()
    np.testing.assert_allclose(p, G[f'{name}_psnr'], rtol=0, atol=1e-5)  # fp64 vs the reference's fp32 mse
    np.testing.assert_allclose(s, G[f'{name}_ssim'], rtol=0, atol=1e-12)
    assert M.calculate_psnr2(a.cuda(), b.cuda()) == pytest.approx(float(G[f'{name}_psnr2']), abs=1e-5)
    assert M.calculate_ssim2(a.cuda(), b.cuda()) == pytest.approx(float(G[f'{name}_ssim2']), abs=1e-12)
    np.testing.assert_allclose(list(M.calculate_psnr(a.cuda(), b.cuda())['psnr'].values()), G[f'{name}_psnr_avg'],
                               atol=1e-5)
    np.testing.assert_allclose(list(M.calculate_ssim(a.cuda(), b.cuda())['ssim_std'].values()),
                               G[f'{name}_ssim_std'], atol=1e-12)


def test_frame_metrics_channel_first_and_large():
    """The sampler's [n, c, t, h, w] layout without a transpose, at the 256 x 256 UCF size."""
    g = torch.Generator().manual_seed(7)
    a = torch.rand(2, 3, 3, 256, 256, generator=g)
    b = (a + 0.03 * torch.randn(a.shape, generator=g)).clamp(0, 1)
    p, s = M.frame_metrics(a.cuda(), b.cuda(), layout='ncthw')
    op, os_ = mo.frame_metrics(a.permute(0, 2, 1, 3, 4).numpy(), b.permute(0, 2, 1, 3, 4).numpy())
    np.testing.assert_allclose(p.cpu().numpy(), op, atol=1e-9)
    np.testing.assert_allclose(s.cpu().numpy(), os_, atol=1e-12)


def test_best_of_n_matches_per_clip_reference_reduction():
    a, b = metric_videos('rgb')  # [n, t, c, h, w]; two clips of n samples
    orig = torch.stack([a, a.flip(0)])
    res = torch.stack([b, b.flip(0)])
    ps, ss = M.best_of_n(orig.cuda(), res.cuda(), cond_frames=1)
    for i in range(2):
        p, s = mo.frame_metrics(orig[i, :, 1:].numpy(), res[i, :, 1:].numpy())
        assert ps[i] == pytest.approx(np.max(p.mean(-1)), abs=1e-9)
        assert ss[i] == pytest.approx(np.max(s.mean(-1)), abs=1e-12)


def test_frame_metrics_rejects_two_channels():
    a = torch.rand(1, 1, 2, 16, 16).cuda()
    with pytest.raises(ValueError):
        M.frame_metrics(a, a)


def test_eval_metrics_summary():
    """valid.py:226-257's reductions: best-of-n per clip, then metric_stuff; fvd_best from
    the feature-L1 selection."""
    from tests.golden_inputs import metric_feats
    a, b = metric_videos('rgb')
    orig = torch.stack([a, a.flip(0), a])
    res = torch.stack([b, b.flip(0), b.flip(1)])
    fake, real = metric_feats()
    ofeat, rfeat = real[:3].astype(np.float64), np.concatenate([fake[:9]]).astype(np.float64)
    out = M.eval_metrics(orig.cuda(), res.cuda(), 1, ofeat, rfeat)
    ps = []
    for i in range(3):
        p, _ = mo.frame_metrics(orig[i, :, 1:].numpy(), res[i, :, 1:].numpy())
        ps.append(np.max(p.mean(-1)))
    assert out['psnr'] == pytest.approx(np.mean(ps), abs=1e-9)
    assert out['psnr_std'] == pytest.approx(np.std(ps), abs=1e-9)
    idx = M.select_best(ofeat, rfeat, 3)
    best = rfeat.reshape(3, 3, -1)[np.arange(3), idx]
    assert out['fvd_best'] == pytest.approx(M.frechet_distance(ofeat, best), rel=1e-12)
    # valid.py:207-213: one frechet_distance per trajectory, then metric_stuff
    fl = np.array([M.frechet_distance(ofeat, rfeat.reshape(3, 3, -1)[:, t]) for t in range(3)])
    assert out['fvd_traj_mean'] == pytest.approx(fl.mean(), rel=1e-12)
    assert out['fvd_traj_std'] == pytest.approx(fl.std(), rel=1e-12)


def test_single_images_2d_and_3d():
    """img_psnr / calculate_ssim_function take [c, h, w] and, like the reference
    (calculate_ssim.py:31-32), a 2-D [h, w] image."""
    a, b = metric_videos('gray')
    i1, i2 = a[0, 0, 0], b[0, 0, 0]  # [h, w]
    p, s = mo.frame_metrics(a[:1, :1].numpy(), b[:1, :1].numpy())
    assert M.img_psnr(i1.cuda(), i2.cuda()) == pytest.approx(float(p[0, 0]), abs=1e-9)
    assert M.calculate_ssim_function(i1.cuda(), i2.cuda()) == pytest.approx(float(s[0, 0]), abs=1e-12)
    assert M.calculate_ssim_function(i1[None].cuda(), i2[None].cuda()) == pytest.approx(float(s[0, 0]), abs=1e-12)
