"""GPU: single attention layers (extdm_attn_layer) against the CPU oracle — STW window
attention (shifted / unshifted) and temporal attention, in both precisions. BAIR levels
0-1 (C = 64 / 128) run the fused f16x3 kernels (stw_x3.hip) in F16X3, level 2 (C = 256)
the unfused route with the f16x3 attention core (attn_core.hip).
Bar: max-abs <= 6e-6 on the layer output (|out| ~ 1-4; 3x the largest measured, 1.9e-6:
profiles/r05_parity_errors.json)."""
import importlib

import pytest

from tests import parity_log
import torch

from tests.golden_inputs import CONFIGS, PKG, make_sd

pytestmark = pytest.mark.gpu
ATT_BAR = 6e-6  # f16x3 / fp32 attention layers vs the oracle (module docstring)
pkg = importlib.import_module(PKG)
DEV = torch.device('cuda:0')
_H = {}


def handle(name, precision):
    key = (name, precision)
    if key not in _H:
        cfg = CONFIGS[name]
        h = pkg._lib.Handle(cfg, 1000, 2, 0, precision=precision)
        sd = make_sd(cfg)
        sd.update(pkg.schedule_buffers(1000))
        h.load_state(sd)
        h.finalize()
        _H[key] = (h, sd)
    return _H[key]


# (layer prefix, level, shifted)
LAYERS = [('downs.0.1', 0, True), ('downs.0.3', 0, False), ('downs.1.1', 1, True), ('downs.2.3', 2, False),
          ('init_temporal_attn', 0, None)]


@pytest.mark.parametrize('precision', ['f16x3', 'fp32'])
@pytest.mark.parametrize('prefix,level,shifted', LAYERS)
def test_attention_layer_vs_oracle(prefix, level, shifted, precision, monkeypatch):
    monkeypatch.delenv('EXTDM_NO_X3_ATTN', raising=False)  # read per call (runtime.cpp x3_attn_ok)
    from oracle import extdm_oracle as O
    cfg = CONFIGS['bair']
    h, sd = handle('bair', precision)
    C = cfg.dim * (1 if level == 0 else cfg.dim_mults[level])
    L = cfg.latent >> level
    gen = torch.Generator().manual_seed(5 + level)
    x = torch.randn(2, C, cfg.frames, L, L, generator=gen) * 1.5 + 0.3
    out = torch.empty(x.shape, device=DEV)
    h.attn_layer(prefix, x.to(DEV), out, shifted=bool(shifted))
    torch.cuda.synchronize()
    with torch.no_grad():
        if shifted is None:
            ref = O.temporal_attention(sd, prefix, x, O.time_pos_bias(sd, cfg.frames), cfg.heads, cfg.dim_head)
        else:
            win = tuple(cfg.window)
            ref = O.stw_attention(sd, prefix, x, win, tuple(w // 2 for w in win) if shifted else (0, 0, 0),
                                  cfg.heads, cfg.dim_head)
    err = (out.cpu() - ref).abs().max().item()
    # bit-stable across launches (the -O3 build of stw_x3.hip was not: build.py OPT)
    out2 = torch.empty(x.shape, device=DEV)
    h.attn_layer(prefix, x.to(DEV), out2, shifted=bool(shifted))
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), out2.cpu())
    parity_log.check(err, ATT_BAR)


@pytest.mark.parametrize('prefix,level,shifted', [('downs.0.1', 0, True), ('downs.2.3', 2, False),
                                                  ('init_temporal_attn', 0, None)])
def test_attention_core_heads6_vs_oracle(prefix, level, shifted):
    """heads = 6 (heads % 4 != 0): the f16x3 attention core walks heads over 4 waves per block,
    so two waves get a second head and two do not (the round-2 ADVICE wave-barrier fix,
    attn_core.hip: no block barrier inside the head loop). The fused kernels take heads = 8
    only, so every attention layer of this config runs the unfused route through the core."""
    import dataclasses
    from oracle import extdm_oracle as O
    cfg = dataclasses.replace(CONFIGS['bair'], heads=6)
    key = ('bair_h6', 'f16x3')
    if key not in _H:
        h = pkg._lib.Handle(cfg, 1000, 2, 0, precision='f16x3')
        sd = make_sd(cfg)
        sd.update(pkg.schedule_buffers(1000))
        h.load_state(sd)
        h.finalize()
        _H[key] = (h, sd)
    h, sd = _H[key]
    C = cfg.dim * (1 if level == 0 else cfg.dim_mults[level])
    L = cfg.latent >> level
    gen = torch.Generator().manual_seed(15 + level)
    x = torch.randn(2, C, cfg.frames, L, L, generator=gen) * 1.5 + 0.3
    out = torch.empty(x.shape, device=DEV)
    h.attn_layer(prefix, x.to(DEV), out, shifted=bool(shifted))
    torch.cuda.synchronize()
    with torch.no_grad():
        if shifted is None:
            ref = O.temporal_attention(sd, prefix, x, O.time_pos_bias(sd, cfg.frames), cfg.heads, cfg.dim_head)
        else:
            win = tuple(cfg.window)
            ref = O.stw_attention(sd, prefix, x, win, tuple(w // 2 for w in win) if shifted else (0, 0, 0),
                                  cfg.heads, cfg.dim_head)
    err = (out.cpu() - ref).abs().max().item()
    out2 = torch.empty(x.shape, device=DEV)
    h.attn_layer(prefix, x.to(DEV), out2, shifted=bool(shifted))
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), out2.cpu())
    parity_log.check(err, ATT_BAR)


@pytest.mark.parametrize('prefix,shifted', [('downs.0.1', True), ('downs.0.3', False)])
def test_window32_tile_odd_frames_vs_oracle(prefix, shifted):
    """SMMNIST's wo_ref denoiser at its own shapes: 2x4x4 windows over 9 + 10 = 19 frames, padded to
    20, so the last window row holds a padded frame. Round 6: the fused kernel's LDS tile path
    (attn_x3_kernel TILE) covers it (rows of the padded frame loaded from frame D - 1, normalised to
    0 like the reference's zero padding, never stored); before, an odd frame count fell back to
    per-lane 4-B loads and stores."""
    import dataclasses
    from oracle import extdm_oracle as O
    cfg = dataclasses.replace(CONFIGS['woref_smmnist'], tp=10)  # the SMMNIST bench: 10 -> 10
    key = ('woref_t19', 'f16x3')
    if key not in _H:
        h = pkg._lib.Handle(cfg, 1000, 2, 0, precision='f16x3')
        sd = make_sd(cfg)
        sd.update(pkg.schedule_buffers(1000))
        h.load_state(sd)
        h.finalize()
        _H[key] = (h, sd)
    h, sd = _H[key]
    assert cfg.frames == 19 and cfg.latent == 32
    gen = torch.Generator().manual_seed(41)
    x = torch.randn(2, cfg.dim, cfg.frames, cfg.latent, cfg.latent, generator=gen) * 1.5 + 0.3
    out = torch.empty(x.shape, device=DEV)
    h.attn_layer(prefix, x.to(DEV), out, shifted=shifted)
    torch.cuda.synchronize()
    with torch.no_grad():
        win = tuple(cfg.window)
        ref = O.stw_attention(sd, prefix, x, win, tuple(w // 2 for w in win) if shifted else (0, 0, 0),
                              cfg.heads, cfg.dim_head)
    err = (out.cpu() - ref).abs().max().item()
    out2 = torch.empty(x.shape, device=DEV)
    h.attn_layer(prefix, x.to(DEV), out2, shifted=shifted)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), out2.cpu())
    parity_log.check(err, ATT_BAR, f'wo_ref {cfg.frames} frames')


# 64-token windows (ada / ada_u22 4x4x4): the fused stw64_x3 route. ada_kth: dim_head 16 (two
# heads per 32-row unit), T = 30 -> padded to 32 frames; u22_city: dim_head 32, T = 7 -> 8
# (a padded frame inside every window of the last window row). `level`: the latent halvings
# (C 64 / 128 from the weights; ups.2.1 is C 64 at latent / 2).
W64 = [('ada_kth', 'downs.0.1', 0, True), ('ada_kth', 'downs.0.3', 0, False), ('ada_kth', 'downs.1.1', 1, True),
       ('u22_city', 'downs.0.1', 0, True), ('u22_city', 'downs.1.3', 1, False), ('u22_city', 'ups.2.1', 1, True)]


def _w64_case(name, prefix, level, shifted, precision):
    from oracle import extdm_oracle as O
    cfg = CONFIGS[name]
    h, sd = handle(name, precision)
    C = sd[prefix + '.fn.fn.attn.qkv.weight'].shape[1]  # ups.i sit one level above their channels
    L = cfg.latent >> level
    gen = torch.Generator().manual_seed(25 + level)
    x = torch.randn(2, C, cfg.frames, L, L, generator=gen) * 1.5 + 0.3
    out = torch.empty(x.shape, device=DEV)
    h.attn_layer(prefix, x.to(DEV), out, shifted=shifted)
    torch.cuda.synchronize()
    win = tuple(cfg.window)
    with torch.no_grad():
        ref = O.stw_attention(sd, prefix, x, win, tuple(w // 2 for w in win) if shifted else (0, 0, 0),
                              cfg.heads, cfg.dim_head)
    out2 = torch.empty(x.shape, device=DEV)
    h.attn_layer(prefix, x.to(DEV), out2, shifted=shifted)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), out2.cpu())  # bit-stable across launches
    return x, out.cpu(), ref


@pytest.mark.parametrize('name,prefix,level,shifted', W64)
def test_window64_attention_vs_oracle(name, prefix, level, shifted):
    """f16x3 (fp32-faithful): the same bar as the <= 32-token windows."""
    x, out, ref = _w64_case(name, prefix, level, shifted, 'f16x3')
    err = (out - ref).abs().max().item()
    print(f'{name} {prefix} f16x3 max|err| {err:.3e}')
    parity_log.check(err, ATT_BAR)


# ada's C = 256 levels (dim_head 16, 64-token windows): the unfused route with the f16x3 attention
# core at DH = 16 (attn_core.hip), LN -> qkv 1x1 conv -> core -> proj 1x1 conv + residual
W64_CORE = [('ada_kth', 'downs.2.1', 2, True), ('ada_kth', 'downs.2.3', 2, False)]


@pytest.mark.parametrize('name,prefix,level,shifted', W64_CORE)
def test_window64_dim16_core_vs_oracle(name, prefix, level, shifted):
    x, out, ref = _w64_case(name, prefix, level, shifted, 'f16x3')
    err = (out - ref).abs().max().item()
    print(f'{name} {prefix} f16x3 core max|err| {err:.3e}')
    parity_log.check(err, ATT_BAR)


@pytest.mark.parametrize('name,prefix,level,shifted', W64)
def test_window64_attention_bf16_vs_oracle(name, prefix, level, shifted):
    """bf16 attention contractions (BF16_ATTN): q, k, v and P rounded to bf16 (2^-9 relative
    each). Bar: max-abs <= 1e-2 x max|attention increment| (ref - x)."""
    x, out, ref = _w64_case(name, prefix, level, shifted, 'bf16_attn')
    err = (out - ref).abs().max().item()
    inc = (ref - x).abs().max().item()
    print(f'{name} {prefix} bf16_attn max|err| {err:.3e} = {err / inc:.2e} x max|increment|')
    parity_log.check(err, 1e-2 * inc, f'bf16, max|increment| {inc:.3e}')
    assert err > 1e-7  # a different arithmetic from the fp32-faithful mode


# temporal attention at the other configs' frame counts: KTH 30 (dim_head 16), wo_ref 14 (the golden
# config's tc - 1 + tp), Cityscapes 7 — the LDS tile path with 32 / 16 / 8 frame slots per pixel (one, two
# or four pixels per wave; 8 since round 6) and the slots past D masked (stw_x3.hip T1)
TEMPORAL = [('ada_kth', 'init_temporal_attn'), ('woref_smmnist', 'init_temporal_attn'),
            ('u22_city', 'init_temporal_attn')]


@pytest.mark.parametrize('name,prefix', TEMPORAL)
def test_temporal_frame_counts_vs_oracle(name, prefix):
    from oracle import extdm_oracle as O
    cfg = CONFIGS[name]
    h, sd = handle(name, 'f16x3')
    C, L = cfg.dim, cfg.latent
    gen = torch.Generator().manual_seed(41)
    x = torch.randn(2, C, cfg.frames, L, L, generator=gen) * 1.5 + 0.3
    out = torch.empty(x.shape, device=DEV)
    h.attn_layer(prefix, x.to(DEV), out, shifted=False)
    torch.cuda.synchronize()
    with torch.no_grad():
        ref = O.temporal_attention(sd, prefix, x, O.time_pos_bias(sd, cfg.frames), cfg.heads, cfg.dim_head)
    err = (out.cpu() - ref).abs().max().item()
    out2 = torch.empty(x.shape, device=DEV)
    h.attn_layer(prefix, x.to(DEV), out2, shifted=False)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), out2.cpu())
    print(f'{name} {prefix} D={cfg.frames} max|err| {err:.3e}')
    parity_log.check(err, ATT_BAR, f'D = {cfg.frames}')
