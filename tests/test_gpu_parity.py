"""GPU parity: the HIP path (through the C ABI) against the reference golden
vectors and the CPU oracle on the same seeded inputs.

Tolerances (fp32 everywhere; the reference's own fp32-vs-fp64 drift is 2.5e-6
per eps forward):
  eps (Unet3D output, |eps| ~ 2)    max-abs <= 1e-4
  one DDPM / DDIM update            max-abs <= 1e-5 x (1 + |eps| coefficient)
  quantile threshold                bit-exact
  DDPM step indexing / DDIM pairs   exact
"""
import importlib

import numpy as np
import pytest

from tests import parity_log
import torch

from tests.golden_inputs import (CONFIGS, PKG, VARIANTS, GOLDEN_BATCH, make_sd, unet_inputs, make_gen_sd,
                                 decoder_inputs, GEN_CFG)
from tests.test_oracle_golden import load

pytestmark = pytest.mark.gpu

pkg = importlib.import_module(PKG)
DEV = torch.device('cuda:0')
_HANDLES = {}


def handle(name, max_batch=4):
    key = (name, max_batch)
    if key not in _HANDLES:
        cfg = CONFIGS[name]
        h = pkg._lib.Handle(cfg, 1000, max_batch, 0)
        sd = make_sd(cfg)
        sd.update(pkg.schedule_buffers(1000))
        h.load_state(sd)
        h.finalize()
        _HANDLES[key] = h
    return _HANDLES[key]


def oracle():
    from oracle import extdm_oracle as O
    return O


def gpu_eps(h, x, t, cond, fea):
    out = torch.empty(x.shape, device=DEV)
    h.unet_forward(x.to(DEV), t.to(DEV), cond.to(DEV), fea.to(DEV), out)
    torch.cuda.synchronize()
    return out.cpu()


@pytest.mark.parametrize('name', ['small', 'bair'])
def test_unet_forward_vs_reference_golden(name):
    cfg = CONFIGS[name]
    x, t, cond, fea = unet_inputs(cfg)
    eps = gpu_eps(handle(name), x, t, cond, fea)
    g = load(f'unet_{name}.npz')['eps']
    err = np.abs(eps.numpy() - g).max()
    parity_log.check(err, 1e-4)


@pytest.mark.parametrize('name', VARIANTS)
def test_variant_unet_forward_vs_reference_golden(name):
    """ada (KTH), ada_u22 (Cityscapes), wo_ref (SMMNIST) denoisers."""
    cfg = CONFIGS[name]
    B = GOLDEN_BATCH.get(name, 2)
    x, t, cond, fea = unet_inputs(cfg, B=B)
    eps = gpu_eps(handle(name, max_batch=B), x, t, cond, fea)
    g = load(f'unet_{name}.npz')['eps']
    err = np.abs(eps.numpy() - g).max()
    parity_log.check(err, 2e-4)


@pytest.mark.parametrize('name', ['ada_small', 'u22_small', 'woref_small'])
def test_variant_ddpm_chain_vs_oracle(name):
    """Three DDPM steps with injected noise through the native sampler loop (graph)
    against the oracle's p_sample_loop restatement over a 3-step schedule."""
    cfg = CONFIGS[name]
    x, _, cond, fea = unet_inputs(cfg, B=2, seed=17)
    h3 = pkg._lib.Handle(cfg, 3, 2, 0)
    sd = make_sd(cfg)
    sd.update(pkg.schedule_buffers(3))
    h3.load_state(sd)
    h3.finalize()
    gen = torch.Generator().manual_seed(3)
    xT = torch.randn(x.shape, generator=gen)
    noises = torch.stack([torch.randn(x.shape, generator=gen) for _ in range(3)])
    out = torch.empty(x.shape, device=DEV)
    h3.sample(0, [2, 1, 0], None, 0., cond.to(DEV), fea.to(DEV), out, x_T=xT.to(DEV),
              noise=noises.to(DEV).contiguous(), use_graph=True)
    torch.cuda.synchronize()
    O = oracle()
    with torch.no_grad():
        ref = O.p_sample_loop(O.schedule(3), lambda xx, tt: O.unet_forward(sd, cfg.as_dict(), xx, tt, cond, fea),
                              xT, list(noises))
    err = (out.cpu() - ref).abs().max().item()
    # 3.1x the largest measured (5.1e-6, u22_small; profiles/r05_parity_errors.json)
    parity_log.check(err, 1.6e-5)


def test_unet_forward_vs_oracle_other_t():
    cfg = CONFIGS['small']
    x, _, cond, fea = unet_inputs(cfg, B=3, seed=7)
    t = torch.tensor([0, 250, 998])
    eps = gpu_eps(handle('small'), x, t, cond, fea)
    with torch.no_grad():
        ref = oracle().unet_forward(make_sd(cfg), cfg.as_dict(), x, t, cond, fea)
    parity_log.check((eps - ref).abs().max().item(), 1e-4)


@pytest.mark.parametrize('tc,latent,fs', [(3, 8, 4), (2, 24, 12), (3, 24, 12)])
def test_trajwarp_key_tiles_vs_oracle(tc, latent, fs):
    """TrajWarp cross-attention (u12:804-827) over key counts the BAIR shapes never reach:
    NK = tc * fs^2 = 48 (one full 32-key tile + a partial one), 288 (an odd count of full
    tiles: the tail after the two-tile loop) and 432 (13 full + a partial tail), through
    the whole u12 forward against the oracle."""
    cfg = pkg.spec.UnetConfig(dim=16, tc=tc, tp=4, latent=latent, fea_size=fs)
    x, t, cond, fea = unet_inputs(cfg, B=2, seed=5)
    h = pkg._lib.Handle(cfg, 1000, 2, 0)
    sd = make_sd(cfg)
    sd.update(pkg.schedule_buffers(1000))
    h.load_state(sd)
    h.finalize()
    eps = gpu_eps(h, x, t, cond, fea)
    with torch.no_grad():
        ref = oracle().unet_forward(make_sd(cfg), cfg.as_dict(), x, t, cond, fea)
    parity_log.check((eps - ref).abs().max().item(), 1e-4)


def test_batch_independence_bitwise():
    """Per-sample results do not depend on batch composition (sharding-safe)."""
    cfg = CONFIGS['small']
    x, t, cond, fea = unet_inputs(cfg, B=4, seed=3)
    t = torch.tensor([10, 20, 30, 40])
    h = handle('small')
    full = gpu_eps(h, x, t, cond, fea)
    one = gpu_eps(h, x[2:3].contiguous(), t[2:3], cond[2:3].contiguous(), fea[2:3].contiguous())
    assert torch.equal(full[2:3], one)


def test_batch_independence_bitwise_ragged_windows():
    """The same at a geometry whose STW window count per sample is not a multiple of the fused
    kernel's 8 waves per workgroup (C = 64 at latent 24, 5 frames: 3 x 6 x 6 = 108 windows), so
    workgroups span two samples: the per-wave operand exponent (stw_x3.hip e_w) keeps every
    sample's roundings its own (round-3 ADVICE)."""
    cfg = pkg.spec.UnetConfig(dim=64, tc=2, tp=3, latent=24, fea_size=12)
    x, t, cond, fea = unet_inputs(cfg, B=3, seed=9)
    t = torch.tensor([5, 500, 950])
    # sample 1 at a much smaller activation scale than its neighbours: a shared exponent would
    # move its lo roundings
    x[1] *= 1e-3
    h = pkg._lib.Handle(cfg, 1000, 3, 0)
    sd = make_sd(cfg)
    sd.update(pkg.schedule_buffers(1000))
    h.load_state(sd)
    h.finalize()
    full = gpu_eps(h, x, t, cond, fea)
    for i in range(3):
        one = gpu_eps(h, x[i:i + 1].contiguous(), t[i:i + 1], cond[i:i + 1].contiguous(), fea[i:i + 1].contiguous())
        assert torch.equal(full[i:i + 1], one), i


def test_ddpm_steps_vs_reference_golden():
    cfg = CONFIGS['small']
    x, _, cond, fea = unet_inputs(cfg)
    g = load('sampler_small.npz')
    h = handle('small')
    for ti in (999, 500, 1, 0):
        tt = torch.full((2,), ti, dtype=torch.long)
        eps = gpu_eps(h, x, tt, cond, fea).to(DEV)
        torch.manual_seed(100 + ti)
        noise = torch.randn(x.shape)
        xs = x.to(DEV).contiguous()
        h.sampler_step(0, ti, 0, 0., xs, eps, noise.to(DEV)[None].contiguous())
        torch.cuda.synchronize()
        err = np.abs(xs.cpu().numpy() - g[f'p_sample_{ti}']).max()
        # one update: 1e-6 = 4x the largest measured (2.4e-7; profiles/r05_parity_errors.json)
        parity_log.check(err, 1e-6, f't={ti}')


def test_quantile_threshold_bit_exact():
    """The fused step's radix-select threshold equals torch.quantile bit for bit."""
    cfg = CONFIGS['small']
    h = handle('small')
    sch = pkg.schedule_buffers(1000)
    gen = torch.Generator().manual_seed(1)
    n = 3 * cfg.tp * cfg.latent * cfg.latent
    for ti, scale in ((999, 1.0), (500, 3.0), (3, 0.2), (100, 50.0)):
        x = (torch.randn(3, 3, cfg.tp, cfg.latent, cfg.latent, generator=gen) * scale)
        eps = torch.randn(x.shape, generator=gen)
        x[1].view(-1)[: n // 2] = 0.25  # heavy ties
        x0 = sch['sqrt_recip_alphas_cumprod'][ti] * x - sch['sqrt_recipm1_alphas_cumprod'][ti] * eps
        ref = torch.quantile(x0.reshape(3, -1).abs(), 0.9, dim=-1).clamp(min=1.0)
        th = torch.zeros(3, device=DEV)
        xs = x.to(DEV).contiguous()
        h.sampler_step(0, ti, 0, 0., xs, eps.to(DEV).contiguous(), torch.zeros((1,) + x.shape, device=DEV), th)
        torch.cuda.synchronize()
        assert torch.equal(th.cpu(), ref), (ti, th.cpu(), ref)


@pytest.mark.parametrize('use_graph', [True, False])
def test_ddpm10_chain_vs_reference_golden(use_graph):
    cfg = CONFIGS['small']
    x, _, cond, fea = unet_inputs(cfg)
    g = load('sampler_small.npz')
    h10 = pkg._lib.Handle(cfg, 10, 2, 0)
    sd = make_sd(cfg)
    sd.update(pkg.schedule_buffers(10))
    h10.load_state(sd)
    h10.finalize()
    torch.manual_seed(7)
    xT = torch.randn(x.shape)
    noises = torch.stack([torch.randn(x.shape) for _ in range(10)])
    out = torch.empty(x.shape, device=DEV)
    h10.sample(0, list(range(9, -1, -1)), None, 0., cond.to(DEV), fea.to(DEV), out, x_T=xT.to(DEV),
               noise=noises.to(DEV).contiguous(), use_graph=use_graph)
    torch.cuda.synchronize()
    err = np.abs(out.cpu().numpy() - g['ddpm10']).max()
    # 3.7x the measured 4.1e-6 (profiles/r05_parity_errors.json)
    parity_log.check(err, 1.5e-5)


def test_ddim10_chain_vs_reference_golden():
    cfg = CONFIGS['small']
    x, _, cond, fea = unet_inputs(cfg)
    g = load('sampler_small.npz')
    h = handle('small')
    pairs = pkg.ddim_time_pairs(1000, 10)
    torch.manual_seed(11)
    xT = torch.randn(x.shape)
    noises = torch.stack([torch.randn(x.shape) for _ in range(10)])
    out = torch.empty(x.shape, device=DEV)
    h.sample(1, [p[0] for p in pairs], [p[1] for p in pairs], 1.0, cond.to(DEV), fea.to(DEV), out, x_T=xT.to(DEV),
             noise=noises.to(DEV).contiguous())
    torch.cuda.synchronize()
    err = np.abs(out.cpu().numpy() - g['ddim10']).max()
    # 3.3x the measured 9.2e-6 (profiles/r05_parity_errors.json)
    parity_log.check(err, 3e-5)


def test_graph_equals_eager_and_sharding_invariance():
    """Philox noise keyed by global sample index: a 4-sample batch equals two
    2-sample shards with sample_base 0 and 2, bit for bit; graph == eager."""
    cfg = CONFIGS['small']
    x, _, cond, fea = unet_inputs(cfg, B=4, seed=21)
    h = handle('small')
    times = list(range(999, 989, -1))
    outs = {}
    for use_graph in (True, False):
        o = torch.empty(x.shape, device=DEV)
        h.sample(0, times, None, 0., cond.to(DEV), fea.to(DEV), o, seed=1234, sample_base=0, use_graph=use_graph)
        outs[use_graph] = o.cpu()
    assert torch.equal(outs[True], outs[False])
    parts = []
    for base in (0, 2):
        o = torch.empty((2,) + tuple(x.shape[1:]), device=DEV)
        h.sample(0, times, None, 0., cond[base:base + 2].to(DEV).contiguous(), fea[base:base + 2].to(DEV).contiguous(),
                 o, seed=1234, sample_base=base)
        parts.append(o.cpu())
    assert torch.equal(torch.cat(parts), outs[True])


def test_decoder_no_occlusion_vs_reference_golden():
    src, flow, _ = decoder_inputs()
    g = load('decoder.npz')
    gen = pkg.Generator()
    out = gen.forward_with_flow(src.to(DEV), flow.to(DEV), None)
    err = np.abs(out['prediction'].cpu().numpy() - g['pred_noocc']).max()
    # 2.8x the measured 7.2e-6 (the fp32 decoder; profiles/r05_parity_errors.json)
    parity_log.check(err, 2e-5)
    assert torch.equal(out['prediction'], out['deformed'])


def test_decoder_with_occlusion_vs_reference_golden():
    """Full Generator.forward_with_flow: encoder half, warped bottleneck, 6 ResBlock2d,
    occlusion-blended skips, nearest-x2 up blocks, sigmoid head (generator.py:152-206)."""
    src, flow, occ = decoder_inputs()
    g = load('decoder.npz')
    gen = pkg.Generator()
    gen.load_state_dict(make_gen_sd())
    out = gen.forward_with_flow(src.to(DEV), flow.to(DEV), occ.to(DEV))
    err = np.abs(out['prediction'].cpu().numpy() - g['pred_occ']).max()
    # ~3x the measured 5.2e-6 / 7.2e-6 (profiles/r05_parity_errors.json)
    parity_log.check(err, 2e-5)
    err_d = np.abs(out['deformed'].cpu().numpy() - g['deformed']).max()
    parity_log.check(err_d, 2e-5)


def test_decoder_multi_frame_matches_per_frame():
    """decode_frames over T frames == T single-frame calls (encoder half hoisted)."""
    src, flow, occ = decoder_inputs()
    gen = pkg.Generator()
    gen.load_state_dict(make_gen_sd())
    fl = torch.stack([flow.permute(0, 3, 1, 2), flow.flip(1).permute(0, 3, 1, 2)], dim=2).to(DEV)
    oc = torch.stack([occ, 1 - occ], dim=2).to(DEV)
    allf = gen.decode_frames(src.to(DEV), fl, oc)
    for t in range(2):
        one = gen.decode_frames(src.to(DEV), fl[:, :, t:t + 1].contiguous(), oc[:, :, t:t + 1].contiguous())
        assert (allf[:, :, t] - one[:, :, 0]).abs().max().item() <= 1e-6


@pytest.mark.parametrize('cls,name', [('Unet3DAda', 'ada_small'), ('Unet3DAdaU22', 'u22_small'),
                                      ('Unet3DWoRef', 'woref_small')])
def test_variant_drop_in_module(cls, name):
    """The drop-in variant classes take the reference constructor (module defaults
    for window / dim_head) and reproduce the golden forward once the state is loaded."""
    cfg = CONFIGS[name]
    u = getattr(pkg, cls)(dim=cfg.dim, channels=cfg.channels, dim_mults=cfg.dim_mults, cond_num=cfg.tc,
                          pred_num=cfg.tp, framesize=cfg.latent).to(DEV)
    assert u.ucfg.window == cfg.window and u.ucfg.dim_head == cfg.dim_head
    u.load_state_dict(make_sd(cfg))
    x, t, cond, fea = unet_inputs(cfg)
    with torch.no_grad():
        eps = u(x.to(DEV), t.to(DEV), cond.to(DEV), cond_fea=fea.to(DEV))
    g = load(f'unet_{name}.npz')['eps']
    parity_log.check(np.abs(eps.cpu().numpy() - g).max(), 2e-4)


def test_decoder_multi_frame_no_occlusion_layout():
    """Without occlusion the multi-frame decode writes [B, C, T, S, S] like the
    per-frame forward_with_flow calls stacked on dim 2 (sample_one_video's layout)."""
    src, flow, _ = decoder_inputs()
    gen = pkg.Generator()
    fl = torch.stack([flow.permute(0, 3, 1, 2), flow.flip(1).permute(0, 3, 1, 2), -flow.permute(0, 3, 1, 2)],
                     dim=2).to(DEV).contiguous()
    allf = gen.decode_frames(src.to(DEV), fl)
    for t in range(3):
        one = gen.forward_with_flow(src.to(DEV), fl[:, :, t].permute(0, 2, 3, 1), None)['prediction']
        assert torch.equal(allf[:, :, t], one)


def test_drop_in_api_sample_shapes_and_determinism():
    cfg = CONFIGS['small']
    u = pkg.Unet3D(dim=cfg.dim, channels=512, dim_mults=cfg.dim_mults, cond_num=cfg.tc, pred_num=cfg.tp,
                   framesize=cfg.latent).to(DEV)
    d = pkg.GaussianDiffusion(u, image_size=cfg.latent, num_frames=cfg.tc + cfg.tp, timesteps=1000,
                              sampling_timesteps=10).to(DEV)
    x, _, cond, fea = unet_inputs(cfg)
    torch.manual_seed(5)
    a = d.sample(cond.to(DEV), cond_fea=fea.to(DEV))
    torch.manual_seed(5)
    b = d.sample(cond.to(DEV), cond_fea=fea.to(DEV))
    assert a.shape == (2, 3, cfg.tp, cfg.latent, cfg.latent)
    assert torch.equal(a, b) and torch.isfinite(a).all()


def test_range_guard_falls_back_to_fp32():
    """f16x3 rejects a sampling call whose conv operands reach |v| >= 65504 (runtime.cpp
    extdm_sample); GaussianDiffusion then re-runs it on an FP32 handle: the
    result equals an explicit FP32 run with the same seed, and the warning is raised."""
    cfg = CONFIGS['small']

    def make(precision):
        u = pkg.Unet3D(dim=cfg.dim, channels=512, dim_mults=cfg.dim_mults, cond_num=cfg.tc, pred_num=cfg.tp,
                       framesize=cfg.latent).to(DEV)
        u.precision = precision
        return pkg.GaussianDiffusion(u, image_size=cfg.latent, num_frames=cfg.tc + cfg.tp, timesteps=1000,
                                     sampling_timesteps=3).to(DEV)
    _, _, cond, fea = unet_inputs(cfg)
    fea = (fea * 1e5).to(DEV)  # TrajWarp's k / v projection inputs past the fp16 range
    d16 = make('f16x3')
    with pytest.warns(RuntimeWarning, match='65504'):
        a = d16.ddim_sample(cond.to(DEV), (2, 3, cfg.tp, cfg.latent, cfg.latent), fea, seed=11)
    # the fallback is the diffusion's state, not the shared denoiser's (round-4 ADVICE)
    assert d16._fp32_fallback and d16.denoise_fn.precision == 'f16x3'
    b = make('fp32').ddim_sample(cond.to(DEV), (2, 3, cfg.tp, cfg.latent, cfg.latent), fea, seed=11)
    assert torch.equal(torch.nan_to_num(a), torch.nan_to_num(b))
    # a second call stays on FP32 without another warning
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter('error')
        c = d16.ddim_sample(cond.to(DEV), (2, 3, cfg.tp, cfg.latent, cfg.latent), fea, seed=11)
    assert torch.equal(torch.nan_to_num(c), torch.nan_to_num(b))
    # a direct forward on the shared denoiser still runs f16x3 and reports the trip via range_flag
    x = torch.zeros(2, 3, cfg.tp, cfg.latent, cfg.latent, device=DEV)
    d16.denoise_fn(x, torch.full((2,), 5, dtype=torch.long, device=DEV), cond.to(DEV), cond_fea=fea)
    assert d16.denoise_fn.range_flag() != 0


@pytest.mark.parametrize('precision', ['f16x3', 'fp32'])
def test_ddpm1000_chain_vs_reference_golden(precision):
    """The headline metric's sampler length: a whole DDPM-1000 chain (t = 999 .. 0, the graph
    replay path) against the reference's own p_sample loop on the reduced u12 denoiser, with
    the reference's CPU noise stream injected (tests/golden/ddpm1000.npz, make_golden.py
    ddpm1000). Checked at the snapshots after t = 999, 900, 500, 100, 10 and 0 by running the
    chain piecewise from the golden state, and as one 1000-step chain from x_T. Bar: the
    single-step bar (1e-4, test_ddpm_steps_vs_reference_golden) plus 2e-6 per step of the
    segment (the survey's drift contract, 7.4e-7 per 10 steps, with margin): 2.1e-3 for the
    whole chain."""
    from tests.golden_inputs import ddpm1000_case, DDPM1000_SNAPS
    cfg, x, cond, fea, seed = ddpm1000_case()
    g = load('ddpm1000.npz')
    h = pkg._lib.Handle(cfg, 1000, x.shape[0], 0, precision=precision)
    sd = make_sd(cfg)
    sd.update(pkg.schedule_buffers(1000))
    h.load_state(sd)
    h.finalize()
    torch.manual_seed(seed)
    xT = torch.randn(x.shape)
    noises = torch.stack([torch.randn(x.shape) for _ in range(1000)])  # p_sample draws at every t
    cd, fd = cond.to(DEV), fea.to(DEV)
    out = torch.empty(x.shape, device=DEV)
    h.sample(0, list(range(999, -1, -1)), None, 0., cd, fd, out, x_T=xT.to(DEV), noise=noises.to(DEV).contiguous(),
             use_graph=True)
    torch.cuda.synchronize()
    whole = np.abs(out.cpu().numpy() - g['x_after_0']).max()
    # piecewise: each segment restarted from the golden state (isolates per-segment error)
    seg = {}
    prev, start = xT, 999
    for ts in DDPM1000_SNAPS:
        times = list(range(start, ts - 1, -1))
        nz = noises[999 - start: 999 - ts + 1]
        h.sample(0, times, None, 0., cd, fd, out, x_T=prev.to(DEV), noise=nz.to(DEV).contiguous(), use_graph=True)
        torch.cuda.synchronize()
        ref = g[f'x_after_{ts}']
        seg[ts] = (len(times), float(np.abs(out.cpu().numpy() - ref).max()))
        prev, start = torch.from_numpy(ref), ts - 1
    print(precision, 'whole chain max|diff|', whole, 'segments (steps, max|diff|)', seg)
    # bars ~3x the measured errors of both precisions (profiles/r05_parity_errors.json): every
    # segment <= 3.6e-6 (f16x3, t = 100 after 400 steps), the whole chain 5.2e-6 (fp32) / 3.9e-6
    for ts, (n, e) in seg.items():
        parity_log.check(e, 1.2e-5, f'snapshot t={ts} after {n} steps')
    parity_log.check(whole, 1.6e-5, 'whole chain')


@pytest.mark.parametrize('arch', ['u12', 'ada'])
def test_fea_phase_fs32_vs_oracle(arch):
    """init_conv's cond_fea branch at fea_size 32, latent 64, which no BASELINE config reaches
    (round-4 ADVICE: the phase-composed route was gated on for fs 32 without a test): u12 and ada
    forwards against the oracle, and the route the handle takes there.
    Bench layer 11 (the edge launches) exists only while the phase-composed route is on."""
    if arch == 'u12':
        cfg = pkg.spec.UnetConfig(dim=64, tc=2, tp=2, latent=64, fea_size=32)
    else:
        cfg = pkg.spec.UnetConfig.for_arch(pkg.spec.ARCH_ADA, tc=2, tp=2, latent=64, fea_size=32)
    x, t, cond, fea = unet_inputs(cfg, B=1, seed=9)
    h = pkg._lib.Handle(cfg, 1000, 1, 0)
    sd = make_sd(cfg)
    sd.update(pkg.schedule_buffers(1000))
    h.load_state(sd)
    h.finalize()
    eps = gpu_eps(h, x, t, cond, fea)
    # the route: at fs 32 the two-phase 128 x 256 tile's X window (12 rows x 36 = 432 staging
    # slots > 400) is not covered, so fea_phase_on (runtime.cpp) keeps the bilinear + 7x7 route
    # — decided once per handle by a dry run of both launchers, no hard failure (round-4 ADVICE);
    # ada's branch reads only cond_fea and runs once per call in the cond cache (fea_hoist_on)
    msg = 'phase-composed cond_fea branch is off' if arch == 'u12' else 'hoisted out of the step'
    with pytest.raises(RuntimeError, match=msg):
        h.bench_layer(1, 11, 1)
    with torch.no_grad():
        ref = oracle().unet_forward(make_sd(cfg), cfg.as_dict(), x, t, cond, fea)
    err = (eps - ref).abs().max().item()
    print(f'{arch} latent 64 / fea 32: max|err| {err:.3e}')
    parity_log.check(err, 1e-4)
