"""LFAE encoder + FlowDiffusion.sample_one_video ORACLE — test infrastructure only.

PyTorch-CPU (fp32) restatement of the reference's region / background / flow
predictors and the sample_one_video round, written from the
behaviour of model/LFAE/*.py and model/BaseDM_adaptor/VideoFlowDiffusion_*.py
(cited per function). Same import rules as extdm_oracle: only tests/, smoke()
and bench.py's cpu_baseline may use it, as the checker.

The 2x2 SVD inside RegionPredictor (region_predictor.py:16-25, 140-146) is
torch.svd on CPU, i.e. LAPACK sgesdd; its singular-vector signs are part of the
result (they flow into the region affines), so `svd2` restates the sgesdd path
for a 2x2 matrix in float32: Householder bidiagonalisation (slarfg), the 2x2
bidiagonal SVD (slasv2), sign fix and ordering (sbdsqr), back-transformation
(sormbr). Checked against torch.svd in tests/test_lfae_oracle.py.

Pinned by tests/golden/lfae.npz (make_golden.py runs the reference modules).
"""
import numpy as np
import torch
import torch.nn.functional as F

from oracle import extdm_oracle as O

f32 = np.float32

# ----------------------------------------------------------------------------
# LAPACK sgesdd for one 2x2 matrix (float32)
# ----------------------------------------------------------------------------


def _fsign(a, b):
    """Fortran SIGN(a, b)."""
    return abs(a) if b >= 0 else -abs(a)


def _slarfg(alpha, x):
    if x == 0:
        return f32(0), f32(alpha), f32(0)
    beta = f32(-_fsign(f32(np.sqrt(f32(alpha) * f32(alpha) + f32(x) * f32(x))), alpha))
    tau = f32((beta - alpha) / beta)
    v = f32(x * f32(1 / f32(alpha - beta)))
    return tau, beta, v


def _slasv2(F_, G, H):
    ft, ht, gt = f32(F_), f32(H), f32(G)
    fa, ha, ga = abs(ft), abs(ht), abs(gt)
    pmax = 1
    swap = ha > fa
    if swap:
        pmax = 3
        ft, ht = ht, ft
        fa, ha = ha, fa
    eps = f32(np.finfo(np.float32).eps / 2)
    if ga == 0:
        ssmin, ssmax, clt, crt, slt, srt = ha, fa, f32(1), f32(1), f32(0), f32(0)
    else:
        gasmal = True
        if ga > fa:
            pmax = 2
            if fa / ga < eps:
                gasmal = False
                ssmax = ga
                ssmin = f32(fa / (ga / ha)) if ha > 1 else f32((fa / ga) * ha)
                clt, slt, srt, crt = f32(1), f32(ht / gt), f32(1), f32(ft / gt)
        if gasmal:
            d = f32(fa - ha)
            l = f32(1) if d == fa else f32(d / fa)
            m = f32(gt / ft)
            t = f32(2 - l)
            mm, tt = f32(m * m), f32(t * t)
            s = f32(np.sqrt(tt + mm))
            r = abs(m) if l == 0 else f32(np.sqrt(f32(l * l) + mm))
            a = f32(0.5 * (s + r))
            ssmin, ssmax = f32(ha / a), f32(fa * a)
            if mm == 0:
                t = f32(_fsign(2, ft) * _fsign(1, gt)) if l == 0 else f32(gt / _fsign(d, ft) + m / t)
            else:
                t = f32((m / (s + t) + m / (r + l)) * (1 + a))
            l = f32(np.sqrt(t * t + 4))
            crt, srt = f32(2 / l), f32(t / l)
            clt = f32((crt + srt * m) / a)
            slt = f32((ht / ft) * srt / a)
    if swap:
        csl, snl, csr, snr = srt, crt, slt, clt
    else:
        csl, snl, csr, snr = clt, slt, crt, srt
    if pmax == 1:
        tsign = _fsign(1, csr) * _fsign(1, csl) * _fsign(1, F_)
    elif pmax == 2:
        tsign = _fsign(1, snr) * _fsign(1, csl) * _fsign(1, G)
    else:
        tsign = _fsign(1, snr) * _fsign(1, snl) * _fsign(1, H)
    ssmax = _fsign(ssmax, tsign)
    ssmin = _fsign(ssmin, tsign * _fsign(1, F_) * _fsign(1, H))
    return ssmin, ssmax, snr, csr, snl, csl


def svd2(m):
    """(u, s) of torch.svd(m) for a 2x2 float32 matrix, via the sgesdd path."""
    a, b, c, d = f32(m[0][0]), f32(m[1][0]), f32(m[0][1]), f32(m[1][1])
    tau, beta, v = _slarfg(a, b)
    w = f32(c + v * d)
    c2, d2 = f32(c - tau * w), f32(d - tau * v * w)
    # sbdsqr: the superdiagonal is negligible below tol * (smallest-singular-value
    # estimate); the matrix then splits into two 1x1 blocks and no rotation is applied
    tol = f32(10 * np.finfo(np.float32).eps / 2)
    sminoa = abs(beta)
    if sminoa != 0:
        mu = f32(abs(d2) * f32(sminoa / f32(sminoa + abs(c2))))
        sminoa = min(sminoa, mu)
    sminoa = f32(sminoa / f32(np.sqrt(f32(2))))
    if abs(c2) <= f32(tol * sminoa):
        ub = np.eye(2, dtype=np.float32)
        s = np.array([abs(beta), abs(d2)], dtype=np.float32)
    else:
        ssmin, ssmax, _, _, snl, csl = _slasv2(beta, c2, d2)
        ub = np.array([[csl, -snl], [snl, csl]], dtype=np.float32)
        s = np.array([abs(ssmax), abs(ssmin)], dtype=np.float32)
    if s[1] > s[0]:
        ub, s = ub[:, ::-1].copy(), s[::-1].copy()
    h = np.eye(2, dtype=np.float32) - tau * np.outer([1, v], [1, v]).astype(np.float32)
    return h @ ub, s


# ----------------------------------------------------------------------------
# blocks (model/LFAE/util.py)
# ----------------------------------------------------------------------------


def _conv_bn_relu(sd, p, x, pad=1):
    x = F.conv2d(x, sd[p + '.conv.weight'], sd[p + '.conv.bias'], padding=pad)
    return F.relu(O._bn(sd, p + '.norm', x))


def down_block(sd, p, x):
    """DownBlock2d (util.py:117-132): conv, BN, ReLU, AvgPool2d(2)."""
    return F.avg_pool2d(_conv_bn_relu(sd, p, x), (2, 2))


def up_block(sd, p, x):
    """UpBlock2d (util.py:97-114): nearest x2, conv, BN, ReLU."""
    return _conv_bn_relu(sd, p, F.interpolate(x, scale_factor=2))


def hg_encoder(sd, p, x, nb):
    """Encoder (util.py:152-168): the input and every down block's output."""
    outs = [x]
    for i in range(nb):
        outs.append(down_block(sd, f'{p}.down_blocks.{i}', outs[-1]))
    return outs


def hourglass(sd, p, x, nb):
    """Hourglass (util.py:171-222); NaN -> 0 on every encoder output (util.py:194-196)."""
    outs = [torch.nan_to_num(o, nan=0.0, posinf=float('inf'), neginf=float('-inf'))
            for o in hg_encoder(sd, p + '.encoder', x, nb)]
    out = outs.pop()
    for j in range(nb):
        out = up_block(sd, f'{p}.decoder.up_blocks.{j}', out)
        out = torch.cat([out, outs.pop()], dim=1)
    return out


def antialias(weight, x, scale):
    """AntiAliasInterpolation2d.forward (util.py:256-264)."""
    if scale == 1:
        return x
    k = weight.shape[-1]
    ka = k // 2
    kb = ka - 1 if k % 2 == 0 else ka
    out = F.conv2d(F.pad(x, (ka, kb, ka, kb)), weight, groups=x.shape[1])
    step = int(1 / scale)
    return out[:, :, ::step, ::step]


def coordinate_grid(h, w):
    """make_coordinate_grid (util.py:50-66): [h, w, 2] of (x, y) in [-1, 1]."""
    x = 2 * (torch.arange(w, dtype=torch.float32) / (w - 1)) - 1
    y = 2 * (torch.arange(h, dtype=torch.float32) / (h - 1)) - 1
    return torch.stack([x.view(1, -1).repeat(h, 1), y.view(-1, 1).repeat(1, w)], dim=2)


# ----------------------------------------------------------------------------
# RegionPredictor / BGMotionPredictor
# ----------------------------------------------------------------------------


def region_predictor(sd, lc, x, prefix='region_predictor.'):
    """RegionPredictor.forward, PCA-based (region_predictor.py:62-150):
    heatmaps = softmax(conv7x7(hourglass) / T) over space; shift = E[grid];
    covar = E[(g - m)(g - m)^T]; affine = U diag(sqrt(S)) from the 2x2 SVD."""
    if lc.rp_scale_factor != 1:
        x = antialias(sd[prefix + 'down.weight'], x, lc.rp_scale_factor)
    fm = hourglass(sd, prefix + 'predictor', x, lc.rp_num_blocks)
    pred = F.conv2d(fm, sd[prefix + 'regions.weight'], sd[prefix + 'regions.bias'], padding=lc.rp_pad)
    N, R, h, w = pred.shape
    heat = F.softmax(pred.view(N, R, -1) / lc.rp_temperature, dim=2).view(N, R, h, w)
    grid = coordinate_grid(h, w)[None, None]
    hm = heat.unsqueeze(-1)
    shift = (hm * grid).sum(dim=(2, 3))
    out = {'shift': shift, 'heatmap': heat}
    if lc.rp_pca_based:
        ms = grid - shift.unsqueeze(-2).unsqueeze(-2)
        covar = (torch.matmul(ms.unsqueeze(-1), ms.unsqueeze(-2)) * hm.unsqueeze(-1)).sum(dim=(2, 3))
        out['covar'] = covar
        us, ss = [], []
        for m in covar.view(-1, 2, 2).numpy():
            u, s = svd2(m)
            us.append(u)
            ss.append(s)
        u = torch.from_numpy(np.stack(us))
        d = torch.diag_embed(torch.from_numpy(np.stack(ss)) ** 0.5)
        out['affine'] = torch.matmul(u, d).view(N, R, 2, 2)
    else:
        raise NotImplementedError('only the PCA-based region predictor is configured (config/DM/*.yaml)')
    return out


def bg_predictor(sd, lc, src, drv, prefix='bg_predictor.'):
    """BGMotionPredictor.forward (bg_motion_predictor.py:47-64) -> [N, 3, 3]."""
    N = src.shape[0]
    out = torch.eye(3).unsqueeze(0).repeat(N, 1, 1)
    if lc.bg_type == 'zero':
        return out
    feat = hg_encoder(sd, prefix + 'encoder', torch.cat([src, drv], dim=1), lc.bg_num_blocks)[-1]
    p = F.linear(feat.mean(dim=(2, 3)), sd[prefix + 'fc.weight'], sd[prefix + 'fc.bias'])
    if lc.bg_type == 'shift':
        out[:, :2, 2] = p
    elif lc.bg_type == 'affine':
        out[:, :2, :] = p.view(N, 2, 3)
    else:
        out[:, :2, :] = p[:, :6].view(N, 2, 3)
        out[:, 2, :2] = p[:, 6:].view(N, 2)
    return out


# ----------------------------------------------------------------------------
# PixelwiseFlowPredictor (pixelwise_flow_predictor.py)
# ----------------------------------------------------------------------------


def region2gaussian(center, covar, h, w):
    """util.region2gaussian (util.py:22-47) with a matrix covariance."""
    grid = coordinate_grid(h, w)
    lead = center.shape[:-1]
    ms = grid.view((1,) * len(lead) + (h, w, 2)) - center.view(lead + (1, 1, 2))
    if isinstance(covar, float):
        return torch.exp(-0.5 * (ms ** 2).sum(-1) / covar)
    inv = torch.inverse(covar).view(lead + (1, 1, 2, 2))
    q = torch.matmul(torch.matmul(ms.unsqueeze(-2), inv), ms.unsqueeze(-1))
    return torch.exp(-0.5 * q.sum(dim=(-1, -2)))


def pixelwise_flow(sd, lc, src, drv_p, src_p, bg, prefix='generator.pixelwise_flow_predictor.'):
    """PixelwiseFlowPredictor.forward (pixelwise_flow_predictor.py:106-153) ->
    (optical_flow [N, h, w, 2], occlusion_map [N, 1, h, w] or None)."""
    if lc.pf_scale_factor != 1:
        src = antialias(sd[prefix + 'down.weight'], src, lc.pf_scale_factor)
    N, C, h, w = src.shape
    R = lc.num_regions
    cd = drv_p['covar'] if lc.pf_use_covar_heatmap else lc.pf_region_var
    cs = src_p['covar'] if lc.pf_use_covar_heatmap else lc.pf_region_var
    heat = region2gaussian(drv_p['shift'], cd, h, w) - region2gaussian(src_p['shift'], cs, h, w)
    heat = torch.cat([torch.zeros(N, 1, h, w), heat], dim=1).unsqueeze(2)
    # sparse motions (create_sparse_motions, :70-97)
    ident = coordinate_grid(h, w).view(1, 1, h, w, 2)
    cg = ident - drv_p['shift'].view(N, R, 1, 1, 2)
    if 'affine' in drv_p:
        aff = torch.matmul(src_p['affine'], torch.inverse(drv_p['affine']))
        if lc.revert_axis_swap:
            aff = aff * torch.sign(aff[:, :, 0:1, 0:1])
        aff = aff.unsqueeze(-3).unsqueeze(-3).repeat(1, 1, h, w, 1, 1)
        cg = torch.matmul(aff, cg.unsqueeze(-1)).squeeze(-1)
    d2s = cg + src_p['shift'].view(N, R, 1, 1, 2)
    bgg = ident.repeat(N, 1, 1, 1, 1)
    if bg is not None:
        hom = torch.cat([bgg, torch.ones(N, 1, h, w, 1)], dim=-1)
        bgg = torch.matmul(bg.view(N, 1, 1, 1, 3, 3), hom.unsqueeze(-1)).squeeze(-1)
        bgg = bgg[..., :2] / (bgg[..., 2:3] + 1e-10)
    sparse = torch.cat([bgg, d2s], dim=1)  # [N, R+1, h, w, 2]
    # deformed sources (create_deformed_source_image, :99-104)
    rep = src.unsqueeze(1).repeat(1, R + 1, 1, 1, 1).view(N * (R + 1), C, h, w)
    deformed = F.grid_sample(rep, sparse.view(N * (R + 1), h, w, 2), align_corners=True).view(N, R + 1, C, h, w)
    inp = torch.cat([heat, deformed], dim=2) if lc.pf_use_deformed_source else heat
    pred = hourglass(sd, prefix + 'hourglass', inp.view(N, -1, h, w), lc.pf_num_blocks)
    mask = F.softmax(F.conv2d(pred, sd[prefix + 'mask.weight'], sd[prefix + 'mask.bias'], padding=3), dim=1)
    flow = (sparse.permute(0, 1, 4, 2, 3) * mask.unsqueeze(2)).sum(dim=1).permute(0, 2, 3, 1)
    occ = None
    if lc.pf_estimate_occlusion_map:
        occ = torch.sigmoid(F.conv2d(pred, sd[prefix + 'occlusion.weight'], sd[prefix + 'occlusion.bias'], padding=3))
    return flow, occ


def bottleneck(sd, lc, img, prefix='generator.'):
    """Generator.forward_bottle / compute_fea (generator.py:95-102, 202-206)."""
    out = _conv_bn_relu(sd, prefix + 'first', img, 3)
    for i in range(lc.gen_num_down_blocks):
        out = down_block(sd, prefix + f'down_blocks.{i}', out)
    return out


def generator_forward(sd, lc, src, drv_p, src_p, bg):
    """Generator.forward (generator.py:104-144): flow predictor, then the
    forward_with_flow decoder. Returns the reference's output dict."""
    flow, occ = pixelwise_flow(sd, lc, src, drv_p, src_p, bg)
    gc = {'num_down_blocks': lc.gen_num_down_blocks, 'num_bottleneck_blocks': lc.gen_num_bottleneck_blocks}
    pred, deformed = O.decoder_forward(sd, gc, src, flow, occ)
    out = {'bottle_neck_feat': bottleneck(sd, lc, src), 'optical_flow': flow, 'deformed': deformed,
           'prediction': pred}
    if occ is not None:
        out['occlusion_map'] = occ
    return out


# ----------------------------------------------------------------------------
# FlowDiffusion.sample_one_video (VideoFlowDiffusion_multi_w_ref.py:223-316)
# ----------------------------------------------------------------------------


def encode_round(sd, lc, ucfg, vid):
    """The no_grad encoder part of sample_one_video: per cond frame idx, region
    params of the frame, bg params vs the reference frame (cond frame tc-1),
    Generator.forward; cond_fea = [bottleneck(frames 0..tc-2), bottleneck(ref) x (1 + tp)].
    Returns (ret dict of real_* tensors, x_cond, cond_fea, ref_img)."""
    tc, tp = ucfg.tc, ucfg.tp
    ref = vid[:, :, tc - 1]
    src_p = region_predictor(sd, lc, ref)
    grids, confs, outs, warps, feas = [], [], [], [], []
    for idx in range(tc):
        frame = vid[:, :, idx]
        drv_p = region_predictor(sd, lc, frame)
        bgp = bg_predictor(sd, lc, ref, frame)
        g = generator_forward(sd, lc, ref, drv_p, src_p, bgp)
        if idx != tc - 1:
            feas.append(bottleneck(sd, lc, frame))
        grids.append(g['optical_flow'].permute(0, 3, 1, 2))
        if lc.pf_estimate_occlusion_map:
            confs.append(g['occlusion_map'])
        outs.append(g['prediction'])
        warps.append(g['deformed'])
    feas += [g['bottle_neck_feat']] * (1 + tp)
    ret = {'real_vid_grid': torch.stack(grids, dim=2), 'real_out_vid': torch.stack(outs, dim=2),
           'real_warped_vid': torch.stack(warps, dim=2)}
    if lc.pf_estimate_occlusion_map:
        ret['real_vid_conf'] = torch.stack(confs, dim=2)
        x_cond = torch.cat([ret['real_vid_grid'], ret['real_vid_conf'] * 2 - 1], dim=1)
    else:
        x_cond = torch.cat([ret['real_vid_grid'], torch.zeros_like(ret['real_vid_grid'])[:, 0:1]], dim=1)
    return ret, x_cond, torch.stack(feas, dim=2), ref


def decode_round(sd, lc, ucfg, ret, pred, ref):
    """The decode part of sample_one_video: grids/conf = cat(real cond part,
    predicted part), then forward_with_flow per frame."""
    tc = ucfg.tc
    grid = torch.cat([ret['real_vid_grid'][:, :, :tc], pred[:, :2]], dim=2)
    conf = None
    if lc.pf_estimate_occlusion_map:
        conf = torch.cat([ret['real_vid_conf'][:, :, :tc], (pred[:, 2].unsqueeze(1) + 1) * 0.5], dim=2)
    gc = {'num_down_blocks': lc.gen_num_down_blocks, 'num_bottleneck_blocks': lc.gen_num_bottleneck_blocks}
    outs, warps = [], []
    for i in range(grid.shape[2]):
        p, d = O.decoder_forward(sd, gc, ref, grid[:, :, i].permute(0, 2, 3, 1),
                                 conf[:, :, i] if conf is not None else None)
        outs.append(p)
        warps.append(d)
    ret = dict(ret)
    ret['sample_vid_grid'] = grid
    if conf is not None:
        ret['sample_vid_conf'] = conf
    ret['sample_out_vid'] = torch.stack(outs, dim=2)
    ret['sample_warped_vid'] = torch.stack(warps, dim=2)
    return ret
