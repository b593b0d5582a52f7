"""Evaluation metrics of the reference's eval driver (scripts/DM/valid.py:199-243):
per-frame PSNR / SSIM on the device (metrics.hip through extdm_frame_metrics), the
reference's per-video reductions, best-of-n selection, frechet_distance and the
mean / std / 95 % interval summary.

Videos follow the reference's metric layout [n, t, c, h, w] (valid.py:194-195 rearranges
`(b n) c t h w -> b n t c h w`); `frame_metrics` also takes the sampler's channel-first
[n, c, t, h, w] through `layout='ncthw'`, so generated clips need no transpose. Values
are in [0, 1] as the reference's (calculate_psnr.py:6-7). LPIPS and the I3D features of
FVD need network weights the reference does not ship; frechet_distance
takes the features as given.
"""
import numpy as np

from . import _lib


def frame_metrics(videos1, videos2, layout='ntchw'):
    """Per-frame (PSNR, SSIM) of two fp32 ROCm tensors [n, t, c, h, w] (or [n, c, t, h, w]
    with layout='ncthw'), c in {1, 3}: two float64 tensors [n, t] on the same device.
    PSNR: metrics/calculate_psnr.py:6-15; SSIM: metrics/calculate_ssim.py:6-41."""
    import torch
    if videos1.shape != videos2.shape:
        raise AssertionError('videos must have the same shape')  # calculate_psnr.py:24
    if videos1.dim() != 5:
        raise ValueError('expected 5-D videos')
    _lib._require_device(videos1, videos2)
    if layout == 'ntchw':
        n, t, c, h, w = videos1.shape
        sn, st, sc = t * c * h * w, c * h * w, h * w
    elif layout == 'ncthw':
        n, c, t, h, w = videos1.shape
        sn, st, sc = c * t * h * w, h * w, t * h * w
    else:
        raise ValueError(f'unknown layout {layout!r}')
    if c not in (1, 3):
        raise ValueError('Wrong input image dimensions.')  # calculate_ssim.py:40-41
    L = _lib.load()
    psnr = torch.empty(n, t, dtype=torch.float64, device=videos1.device)
    ssim = torch.empty(n, t, dtype=torch.float64, device=videos1.device)
    work = torch.empty(max(1, L.extdm_frame_metrics_workspace(n, t, c, h, w)), dtype=torch.uint8,
                       device=videos1.device)
    with torch.cuda.device(videos1.device):
        _lib.check(L.extdm_frame_metrics(_lib._ptr(videos1), _lib._ptr(videos2), n, t, c, h, w, sn, st, sc,
                                         _lib._ptr(psnr), _lib._ptr(ssim), _lib._ptr(work), _lib._stream()))
    return psnr, ssim


def _as_chw(img):
    # the reference also takes a 2-D [h, w] image (calculate_ssim.py:31-32)
    return img[None] if img.dim() == 2 else img


def img_psnr(img1, img2):
    """metrics/calculate_psnr.py:6-15 for one [c, h, w] (or [h, w]) image."""
    return float(frame_metrics(_as_chw(img1)[None, None], _as_chw(img2)[None, None])[0][0, 0])


def calculate_ssim_function(img1, img2):
    """metrics/calculate_ssim.py:26-41 for one [c, h, w] (c in {1, 3}) or [h, w] image."""
    if img1.shape != img2.shape:
        raise ValueError('Input images must have the same dimensions.')
    if img1.dim() not in (2, 3):
        raise ValueError('Wrong input image dimensions.')
    return float(frame_metrics(_as_chw(img1)[None, None], _as_chw(img2)[None, None])[1][0, 0])


def _per_frame_summary(vals, name, shape):
    v = vals.cpu().numpy()
    return {name: {f'avg[{i}]': np.mean(v[:, i]) for i in range(v.shape[1])},
            f'{name}_std': {f'std[{i}]': np.std(v[:, i]) for i in range(v.shape[1])},
            f'{name}_video_setting': shape, f'{name}_video_setting_name': 'time, channel, heigth, width'}


def calculate_psnr(videos1, videos2):
    """metrics/calculate_psnr.py:19-69: mean / std over videos per frame index."""
    return _per_frame_summary(frame_metrics(videos1, videos2)[0], 'psnr', videos1.shape[1:])


def calculate_ssim(videos1, videos2):
    """metrics/calculate_ssim.py:46-101."""
    return _per_frame_summary(frame_metrics(videos1, videos2)[1], 'ssim', videos1.shape[1:])


def calculate_psnr1(videos1, videos2):
    """metrics/calculate_psnr.py:71-87: (mean, std) over every frame."""
    v = frame_metrics(videos1, videos2)[0].cpu().numpy()
    return np.mean(v), np.std(v)


def calculate_ssim1(videos1, videos2):
    """metrics/calculate_ssim.py:103-117."""
    v = frame_metrics(videos1, videos2)[1].cpu().numpy()
    return np.mean(v), np.std(v)


def calculate_psnr2(videos1, videos2):
    """metrics/calculate_psnr.py:89-106: the best of the n samples, max over n of the
    per-sample mean over frames (valid.py:232 passes one clip's n samples)."""
    v = frame_metrics(videos1, videos2)[0].cpu().numpy()
    return np.max(np.mean(v, axis=-1))


def calculate_ssim2(videos1, videos2):
    """metrics/calculate_ssim.py:119-134."""
    v = frame_metrics(videos1, videos2)[1].cpu().numpy()
    return np.max(np.mean(v, axis=-1))


def best_of_n(origin_videos, result_videos, cond_frames):
    """valid.py:226-233: PSNR / SSIM of each clip's best sample over the predicted frames.
    origin_videos, result_videos: [b, n, t, c, h, w]. Returns (psnr_list, ssim_list), one
    value per clip; all b*n*t frames go through one device launch."""
    b, n = result_videos.shape[:2]
    a = origin_videos[:, :, cond_frames:].contiguous().flatten(0, 1)
    r = result_videos[:, :, cond_frames:].contiguous().flatten(0, 1)
    psnr, ssim = frame_metrics(a, r)
    pm = psnr.mean(dim=-1).view(b, n).max(dim=1).values.cpu().numpy()
    sm = ssim.mean(dim=-1).view(b, n).max(dim=1).values.cpu().numpy()
    return list(pm), list(sm)


def select_best(origin_feats, result_feats, num_sample_video):
    """valid.py:234-240: per clip, the sample whose features are nearest (L1) to the
    ground truth's: origin_feats [b, d], result_feats [b * n, d] -> indices [b]."""
    o = np.asarray(origin_feats)
    r = np.asarray(result_feats).reshape(o.shape[0], num_sample_video, -1)
    scores = np.abs(o[:, None, :] - r).sum(axis=-1)
    return np.argmin(scores, axis=-1)


def frechet_distance(feats_fake, feats_real):
    """metrics/fvd.py:276-293: squared distance of the feature means plus
    tr(S_fake) + tr(S_real) - 2 tr(sqrtm(S_fake S_real)) of the (unbiased) covariances;
    the mean term alone when there is a single fake feature. Host fp64 (scipy sqrtm),
    as the reference computes it."""
    from scipy.linalg import sqrtm
    fake, real = np.asarray(feats_fake), np.asarray(feats_real)
    dmu = fake.mean(axis=0) - real.mean(axis=0)
    mean_term = np.square(dmu).sum()
    if fake.shape[0] <= 1:
        return float(np.real(mean_term))
    cov_f, cov_r = np.cov(fake, rowvar=False), np.cov(real, rowvar=False)
    root = sqrtm(cov_f @ cov_r, disp=False)[0]
    return float(np.real(mean_term + np.trace(cov_f + cov_r - 2 * root)))


def metric_stuff(metric):
    """valid.py:24-27: mean, std and the half-width of the normal 95 % interval."""
    import scipy.stats as st
    avg_metric, std_metric = metric.mean().item(), metric.std().item()
    conf95_metric = avg_metric - float(st.norm.interval(confidence=0.95, loc=avg_metric, scale=st.sem(metric))[0])
    return avg_metric, std_metric, conf95_metric


def eval_metrics(origin_videos, result_videos, cond_frames, origin_feats=None, result_feats=None):
    """The metric half of valid.py:199-257 on [b, n, t, c, h, w] videos: per clip the best of
    its n samples for PSNR and SSIM over the predicted frames (calculate_psnr2 /
    calculate_ssim2), summarised by metric_stuff. With video features given (origin [b, d],
    result [b * n, d]; the reference's I3D features, not shipped with it), the best sample
    per clip by feature L1 (valid.py:234-240) and its frechet_distance to the originals
    ('fvd_best'), and one frechet_distance per sample trajectory summarised by metric_stuff
    ('fvd_traj_mean' / '_std' / '_conf95', valid.py:207-213). LPIPS needs network weights
    the reference does not ship: not computed."""
    psnr_list, ssim_list = best_of_n(origin_videos, result_videos, cond_frames)
    avg_psnr, std_psnr, conf95_psnr = metric_stuff(np.array(psnr_list))
    avg_ssim, std_ssim, conf95_ssim = metric_stuff(np.array(ssim_list))
    out = {'psnr': avg_psnr, 'psnr_std': std_psnr, 'psnr_conf95': conf95_psnr,
           'ssim': avg_ssim, 'ssim_std': std_ssim, 'ssim_conf95': conf95_ssim}
    if origin_feats is not None and result_feats is not None:
        n = result_videos.shape[1]
        idx = select_best(origin_feats, result_feats, n)
        rf = np.asarray(result_feats).reshape(len(idx), n, -1)
        best = rf[np.arange(len(idx)), idx]
        out['fvd_best'] = frechet_distance(np.asarray(origin_feats), best)
        out['selected_index'] = idx
        # per trajectory: the features of every clip's traj-th sample (valid.py:207-209)
        fvd_list = [frechet_distance(np.asarray(origin_feats), rf[:, traj]) for traj in range(n)]
        out['fvd_traj_mean'], out['fvd_traj_std'], out['fvd_traj_conf95'] = metric_stuff(np.array(fvd_list))
    return out
