"""Evaluation-metric ORACLE — test infrastructure only (tests/ import it as the
checker; the product path, metrics.hip behind extdm_frame_metrics, never does).

A numpy fp64 restatement of the per-frame metrics the eval driver computes
(scripts/DM/valid.py:226-233), written from the reference's behaviour:
  psnr_frame  metrics/calculate_psnr.py:6-15  20 log10(1 / sqrt(mse)); 100 when mse < 1e-10
  ssim_frame  metrics/calculate_ssim.py:6-41  11x11 Gaussian window (sigma 1.5) over the
              'valid' region, C1 = 0.01^2, C2 = 0.03^2, map mean, then the channel mean
Parity pinning: checked against tests/golden/metrics.npz, written by the reference's own
metric functions (tests/golden/make_golden.py --metrics). cv2 is absent offline; the
fixture's SSIM ran through tests/golden/shims/cv2 (getGaussianKernel / filter2D
restated), so SSIM is pinned to the reference's formula and crop, not to OpenCV's
arithmetic.
"""
import numpy as np


def gaussian_window(k=11, sigma=1.5):
    x = np.arange(k, dtype=np.float64) - (k - 1) / 2
    g = np.exp(-x * x / (2 * sigma * sigma))
    g /= g.sum()
    return np.outer(g, g)


def _valid_filter(img, win):
    """2-D correlation of img with win over positions where the window fits."""
    k = win.shape[0]
    h, w = img.shape[0] - k + 1, img.shape[1] - k + 1
    out = np.zeros((h, w))
    for i in range(k):
        for j in range(k):
            out += win[i, j] * img[i:i + h, j:j + w]
    return out


def ssim_plane(a, b):
    a = a.astype(np.float64)
    b = b.astype(np.float64)
    win = gaussian_window()
    mu1, mu2 = _valid_filter(a, win), _valid_filter(b, win)
    s11 = _valid_filter(a * a, win) - mu1 * mu1
    s22 = _valid_filter(b * b, win) - mu2 * mu2
    s12 = _valid_filter(a * b, win) - mu1 * mu2
    c1, c2 = 0.01 ** 2, 0.03 ** 2
    m = ((2 * mu1 * mu2 + c1) * (2 * s12 + c2)) / ((mu1 * mu1 + mu2 * mu2 + c1) * (s11 + s22 + c2))
    return m.mean()


def ssim_frame(a, b):
    """a, b: [c, h, w] with c in {1, 3}."""
    return float(np.mean([ssim_plane(a[c], b[c]) for c in range(a.shape[0])]))


def psnr_frame(a, b):
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return 100.0 if mse < 1e-10 else 20 * np.log10(1 / np.sqrt(mse))


def frame_metrics(v1, v2):
    """[n, t, c, h, w] numpy -> (psnr [n, t], ssim [n, t])."""
    n, t = v1.shape[:2]
    p = np.array([[psnr_frame(v1[i, j], v2[i, j]) for j in range(t)] for i in range(n)])
    s = np.array([[ssim_frame(v1[i, j], v2[i, j]) for j in range(t)] for i in range(n)])
    return p, s
