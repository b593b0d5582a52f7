"""CPU check of the phase-composed cond_fea branch's algebra (fea_x3.hip header, runtime.cpp
Pfea_phase): conv7x7(pad 3) of the bilinear x2 upsample (align_corners=False, as
u12:1035-1037) equals the per-phase 5x5 over the zero-padded map plus the edge-line and corner
corrections. The composition below restates runtime.cpp's formulas in numpy (fp64) and is
compared with torch's F.interpolate + F.conv2d on random data."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F


def up_true(r, k, n):
    if r < 0 or r >= 2 * n:
        return 0.0
    src = max(0.0, (r + 0.5) * 0.5 - 0.5)
    k0 = int(src)
    k1 = k0 + 1 if k0 < n - 1 else k0
    lam = src - k0
    return (1.0 - lam if k == k0 else 0.0) + (lam if k == k1 else 0.0)


def up_inf(r, k):
    j = r // 2
    if k == j:
        return 0.75
    return 0.25 if (k == j - 1 if r - 2 * j == 0 else k == j + 1) else 0.0


def compose(w, n):
    """w [Co][Cf][7][7] -> (k5 [2][2][Co][Cf][5][5], side [pair][side][d][py][px][Co][Cf][5],
    corner [4][4][4][Co][Cf])"""
    A = np.array([[[up_inf(2 * 8 + p + d - 3, 8 - 2 + l) for d in range(7)] for l in range(5)] for p in range(2)])
    k5 = np.einsum('ayd,bxe,oide->aboiyx', A, A, w)
    delta = lambda r, ke: up_true(r, ke, n) - up_inf(r, ke)  # noqa: E731
    Co, Cf = w.shape[:2]
    side = np.zeros((2, 2, 2, 2, 2, Co, Cf, 5))
    for pair in range(2):
        for sd in range(2):
            ke, base = (n - 1, 2 * n - 4) if sd else (0, 0)
            for d in range(2):
                for py in range(2):
                    for px in range(2):
                        e = base + 2 * d + (px if pair else py)
                        dl = np.array([delta(e + k - 3, ke) for k in range(7)])
                        if pair == 0:  # rows: delta along y, interior phase px along x
                            side[pair, sd, d, py, px] = np.einsum('y,lx,oiyx->oil', dl, A[px], w)
                        else:
                            side[pair, sd, d, py, px] = np.einsum('x,ly,oiyx->oil', dl, A[py], w)
    corner = np.zeros((4, 4, 4, Co, Cf))
    for c in range(4):
        ky, kx = (n - 1 if c >> 1 else 0), (n - 1 if c & 1 else 0)
        yb, xb = (2 * n - 4 if c >> 1 else 0), (2 * n - 4 if c & 1 else 0)
        for yy in range(4):
            for xx in range(4):
                dy = np.array([delta(yb + yy + k - 3, ky) for k in range(7)])
                dx = np.array([delta(xb + xx + k - 3, kx) for k in range(7)])
                corner[c, yy, xx] = np.einsum('y,x,oiyx->oi', dy, dx, w)
    return k5, side, corner


def apply(f, k5, side, corner):
    """f [Cf][n][n] -> out [Co][2n][2n] through the decomposition (fp64)"""
    Cf, n, _ = f.shape
    Co = k5.shape[2]
    fp = np.zeros((Cf, n + 4, n + 4))
    fp[:, 2:n + 2, 2:n + 2] = f
    out = np.zeros((Co, 2 * n, 2 * n))
    for py in range(2):
        for px in range(2):
            acc = np.zeros((Co, n, n))
            for ly in range(5):
                for lx in range(5):
                    acc += np.einsum('oi,iyx->oyx', k5[py, px, :, :, ly, lx], fp[:, ly:ly + n, lx:lx + n])
            out[:, py::2, px::2] = acc
    for pair in range(2):
        for sd in range(2):
            ke = n - 1 if sd else 0
            line = np.zeros((Cf, n + 4))
            line[:, 2:n + 2] = f[:, ke, :] if pair == 0 else f[:, :, ke]
            base = 2 * n - 4 if sd else 0
            for d in range(2):
                for py in range(2):
                    for px in range(2):
                        v = sum(np.einsum('oi,ij->oj', side[pair, sd, d, py, px, :, :, l], line[:, l:l + n])
                                for l in range(5))
                        for j in range(n):
                            if pair == 0:
                                out[:, base + 2 * d + py, 2 * j + px] += v[:, j]
                            else:
                                out[:, 2 * j + py, base + 2 * d + px] += v[:, j]
    for c in range(4):
        ky, kx = (n - 1 if c >> 1 else 0), (n - 1 if c & 1 else 0)
        yb, xb = (2 * n - 4 if c >> 1 else 0), (2 * n - 4 if c & 1 else 0)
        for yy in range(4):
            for xx in range(4):
                out[:, yb + yy, xb + xx] += corner[c, yy, xx] @ f[:, ky, kx]
    return out


@pytest.mark.parametrize('n', [8, 16])
def test_phase_composition_equals_upsample_then_conv7(n):
    rng = np.random.default_rng(n)
    Co, Cf = 3, 4
    w = rng.standard_normal((Co, Cf, 7, 7))
    f = rng.standard_normal((Cf, n, n))
    ft = torch.from_numpy(f)[None]
    up = F.interpolate(ft, size=(2 * n, 2 * n), mode='bilinear')  # u12:1036
    ref = F.conv2d(up, torch.from_numpy(w), padding=3)[0].numpy()
    got = apply(f, *compose(w, n))
    assert np.abs(got - ref).max() < 1e-10 * np.abs(ref).max()


def test_edge_deltas_only_touch_the_border():
    n = 16
    for r in range(-3, 2 * n + 3):
        for k in range(n):
            dlt = up_true(r, k, n) - up_inf(r, k)
            if dlt != 0.0:
                assert (k == 0 and r in (-1, 0)) or (k == n - 1 and r in (2 * n - 1, 2 * n)), (r, k, dlt)
