"""Model configuration and state_dict layout of the ExtDM sampling path.

`unet_spec(cfg)` lists the Unet3D state_dict entries (name, shape, dtype) in the
exact order the reference registers them, for each of the four denoisers
(model/BaseDM_adaptor/DenoiseNet_STWAtt_w_w_ref_adaptor_cross_multi_traj_u12.py:864-1003,
..._traj_ada.py:865-1018, ..._traj_ada_u22.py:1009-1170,
DenoiseNet_STWAtt_w_wo_ref_adaptor_cross_multi.py:755-904), so reference DM
checkpoints (`checkpoint['diffusion']`, keys `denoise_fn.*`) load
strict-compatible and synthetic weights are generated in reference order.
`generator_spec(gcfg)` does the same for the LFAE Generator decoder
(model/LFAE/generator.py:26-62, util.py:69-149).
"""
import math
from dataclasses import dataclass, field

ARCH_U12 = 'DenoiseNet_STWAtt_w_w_ref_adaptor_cross_multi_traj_u12'
ARCH_U22 = 'DenoiseNet_STWAtt_w_w_ref_adaptor_cross_multi_traj_u22'  # byte-identical to u12
ARCH_ADA = 'DenoiseNet_STWAtt_w_w_ref_adaptor_cross_multi_traj_ada'
ARCH_ADA_U22 = 'DenoiseNet_STWAtt_w_w_ref_adaptor_cross_multi_traj_ada_u22'
ARCH_WO_REF = 'DenoiseNet_STWAtt_w_wo_ref_adaptor_cross_multi'
# ids of include/extdm.h EXTDM_ARCH_*
ARCH_IDS = {ARCH_U12: 0, ARCH_U22: 0, ARCH_ADA: 1, ARCH_ADA_U22: 2, ARCH_WO_REF: 3}
ARCH_SHORT = {ARCH_U12: 'u12', ARCH_U22: 'u12', ARCH_ADA: 'ada', ARCH_ADA_U22: 'ada_u22', ARCH_WO_REF: 'wo_ref'}
# constructor defaults that differ per module (window_size, attn_dim_head)
ARCH_DEFAULTS = {ARCH_U12: ((2, 4, 4), 32), ARCH_U22: ((2, 4, 4), 32), ARCH_ADA: ((4, 4, 4), 16),
                 ARCH_ADA_U22: ((4, 4, 4), 32), ARCH_WO_REF: ((2, 4, 4), 32)}


@dataclass
class UnetConfig:
    """Constructor surface of Unet3D as FlowDiffusion builds it
    (VideoFlowDiffusion_multi_w_ref.py:80-94; _u22.py:199-213; multi1248.py:70-84).
    `fea_size` is the cond_fea H = W: the LFAE bottleneck (latent / 2) for the
    feature-branch denoisers, the latent itself for wo_ref (multi1248.py:243-245)."""
    dim: int = 64
    channels: int = 512
    dim_mults: tuple = (1, 2, 4, 4)
    window: tuple = (2, 4, 4)
    heads: int = 8
    dim_head: int = 32
    tc: int = 2
    tp: int = 14
    latent: int = 32           # flow / latent H = W
    fea_size: int = 16         # cond_fea spatial size
    fea_ch: int = 256
    arch: str = ARCH_U12

    @classmethod
    def for_arch(cls, arch, **kw):
        """Defaults of the named reference module, then overrides."""
        win, dh = ARCH_DEFAULTS[arch]
        base = dict(window=win, dim_head=dh, arch=arch)
        if arch in (ARCH_ADA_U22, ARCH_WO_REF):
            base['channels'] = 3 + 256
        if arch == ARCH_WO_REF:
            base['dim_mults'] = (1, 2, 4, 8)
        base.update(kw)
        if arch == ARCH_WO_REF and 'fea_size' not in kw:
            base['fea_size'] = base.get('latent', 32)
        return cls(**base)

    @property
    def short(self):
        return ARCH_SHORT[self.arch]

    @property
    def tm(self):
        """cond frames the denoiser sees (wo_ref drops the last: wo_ref.py:911)."""
        return self.tc - 1 if self.arch == ARCH_WO_REF else self.tc

    @property
    def frames(self):
        return self.tm + self.tp

    def levels(self):
        dims = [self.dim] + [self.dim * m for m in self.dim_mults]
        return list(zip(dims[:-1], dims[1:]))

    def as_dict(self):
        return {'dim': self.dim, 'dim_mults': tuple(self.dim_mults), 'window': tuple(self.window),
                'heads': self.heads, 'dim_head': self.dim_head, 'tc': self.tc, 'tp': self.tp,
                'arch': self.short}


def adaptor_layers(tm, tp):
    """compute_layer (u12:644-648)."""
    L = max(1, int(math.ceil(math.log2((tp + 1) / tm))))
    return L, (2 ** L - 1) * tm


def _resnet(out, p, din, dout, temb_dim):
    if temb_dim:
        out += [(f'{p}.mlp.1.weight', (dout * 2, temb_dim)), (f'{p}.mlp.1.bias', (dout * 2,))]
    for b, ci in (('block1', din), ('block2', dout)):
        out += [(f'{p}.{b}.proj.weight', (dout, ci, 1, 3, 3)), (f'{p}.{b}.proj.bias', (dout,)),
                (f'{p}.{b}.norm.weight', (dout,)), (f'{p}.{b}.norm.bias', (dout,))]
    if din != dout:
        out += [(f'{p}.res_conv.weight', (dout, din, 1, 1, 1)), (f'{p}.res_conv.bias', (dout,))]


def _stw(out, p, d, cfg):
    a = f'{p}.fn.fn.attn'
    w = cfg.window
    nt = (2 * w[0] - 1) * (2 * w[1] - 1) * (2 * w[2] - 1)
    N = w[0] * w[1] * w[2]
    hid = cfg.heads * cfg.dim_head
    out += [(f'{a}.relative_position_bias_table', (nt, cfg.heads)),
            (f'{a}.relative_position_index', (N, N), 'int64'),
            (f'{a}.rotary_emb.freqs', (min(32, cfg.dim_head) // 2,)),
            (f'{a}.qkv.weight', (3 * hid, d)),
            (f'{a}.proj.weight', (d, hid)), (f'{a}.proj.bias', (d,)),
            (f'{p}.fn.norm.gamma', (1, d, 1, 1, 1))]


def _adaptor(out, p, d, cfg):
    L, Fr = adaptor_layers(cfg.tm, cfg.tp)
    ap = f'{p}.adaptors'
    out += [(f'{ap}.predictor.fn.fn.weight', (d, d, 1, 1, 1)), (f'{ap}.predictor.fn.fn.bias', (d,)),
            (f'{ap}.predictor.fn.norm.gamma', (1, d, 1, 1, 1))]
    kt = 3 if cfg.short == 'ada_u22' else 1  # ada_u22 extrapolates with full 3x3x3 convs (ada_u22.py:537)
    for l in range(L):
        out += [(f'{ap}.extrapolators.{l}.fn.weight', (d, d, kt, 3, 3))]
    out += [(f'{p}.Tmodulator.weight', (d * cfg.tp, d * Fr, 1, 1)), (f'{p}.Tmodulator.bias', (d * cfg.tp,)),
            (f'{p}.fuser.fn.weight', (d, 2 * d, 1, 1, 1)), (f'{p}.fuser.fn.bias', (d,)),
            (f'{p}.fuser.norm.gamma', (1, 2 * d, 1, 1, 1))]


def _temporal(out, p, d, cfg):
    """Residual(PreNorm(d, EinopsToAndFrom(AttentionLayer))) (u12:903-915)."""
    hid = cfg.heads * cfg.dim_head
    a = f'{p}.fn.fn.fn'
    out += [(f'{a}.norm.weight', (d,)), (f'{a}.norm.bias', (d,)),
            (f'{a}.attn.rotary_emb.freqs', (min(32, cfg.dim_head) // 2,)),
            (f'{a}.attn.to_qkv.weight', (3 * hid, d)), (f'{a}.attn.to_out.weight', (d, hid)),
            (f'{p}.fn.norm.gamma', (1, d, 1, 1, 1))]


def unet_spec(cfg: UnetConfig):
    """Ordered (name, shape, dtype) list of the Unet3D state_dict of cfg.arch."""
    arch = cfg.short
    u22 = arch == 'ada_u22'
    out = []
    d0 = cfg.dim
    tdim = cfg.dim * 4
    if u22:  # direct Parameters come first in state_dict order (ada_u22.py:1120-1121)
        out += [('alpha', (cfg.heads,)), ('beta', (cfg.heads,))]
    out += [('time_rel_pos_bias.relative_attention_bias.weight', (32, cfg.heads))]
    if u22:
        out += [('rel_pos_bias_thw.relative_attention_bias.weight', (32, cfg.heads))]
    out += [('init_conv.weight', (d0, cfg.channels, 1, 7, 7)), ('init_conv.bias', (d0,))]
    if arch != 'wo_ref':
        out += [('init_noise_conv.weight', (256, 3, 1, 7, 7)), ('init_noise_conv.bias', (256,))]
    _temporal(out, 'init_temporal_attn', d0, cfg)
    if arch == 'u12':
        _adaptor(out, 'init_adaptor', 256, cfg)
        for n in ('q', 'k', 'v', 'o'):
            out += [(f'init_traj.cross_att.linear_{n}.weight', (256, 256)),
                    (f'init_traj.cross_att.linear_{n}.bias', (256,))]
        out += [('init_traj.fuser.weight', (256, 512, 1, 1, 1)), ('init_traj.fuser.bias', (256,))]
    elif arch in ('ada', 'ada_u22'):
        _temporal(out, 'cond_temporal_attn', 256, cfg)
        _adaptor(out, 'cond_adaptor', 256, cfg)
    out += [('time_mlp.1.weight', (tdim, cfg.dim)), ('time_mlp.1.bias', (tdim,)),
            ('time_mlp.3.weight', (tdim, tdim)), ('time_mlp.3.bias', (tdim,))]
    lv = cfg.levels()
    samp = '6' if u22 else '5'
    for i, (din, dout) in enumerate(lv):
        p = f'downs.{i}'
        _resnet(out, p + '.0', din, dout, tdim)
        _stw(out, p + '.1', dout, cfg)
        _resnet(out, p + '.2', dout, dout, tdim)
        _stw(out, p + '.3', dout, cfg)
        if i > 1 or u22:
            _adaptor(out, p + '.4', dout, cfg)
        if u22:
            _temporal(out, p + '.5', dout, cfg)
        if i < len(lv) - 1:
            out += [(f'{p}.{samp}.weight', (dout, dout, 1, 4, 4)), (f'{p}.{samp}.bias', (dout,))]
    # the `ups` ModuleList is registered before mid_block1 (u12:946-947)
    for i, (din, dout) in enumerate(reversed(lv)):
        p = f'ups.{i}'
        _resnet(out, p + '.0', dout * 2, din, tdim)
        _stw(out, p + '.1', din, cfg)
        _resnet(out, p + '.2', din, din, tdim)
        _stw(out, p + '.3', din, cfg)
        if i > 1:
            _adaptor(out, p + '.4', din, cfg)
        if u22:
            _temporal(out, p + '.5', din, cfg)
        if i < len(lv) - 1:
            out += [(f'{p}.{samp}.weight', (din, din, 1, 4, 4)), (f'{p}.{samp}.bias', (din,))]
    md = lv[-1][1]
    _resnet(out, 'mid_block1', md, md, tdim)
    _stw(out, 'mid_attn1', md, cfg)
    _resnet(out, 'mid_block2', md, md, tdim)
    _stw(out, 'mid_attn2', md, cfg)
    _adaptor(out, 'mid_adaptor', md, cfg)
    for head, oc in (('final_conv', 2), ('occlusion_map', 1)):
        _resnet(out, head + '.0', cfg.dim * 2, cfg.dim, 0)
        out += [(f'{head}.1.weight', (oc, cfg.dim, 1, 1, 1)), (f'{head}.1.bias', (oc,))]
    return [(e[0], tuple(e[1]), e[2] if len(e) > 2 else 'float32') for e in out]


@dataclass
class GeneratorConfig:
    """LFAE Generator decoder surface (config/DM/*.yaml flow_params.generator_params)."""
    num_channels: int = 3
    block_expansion: int = 64
    max_features: int = 512
    num_down_blocks: int = 2
    num_bottleneck_blocks: int = 6
    image: int = 64

    def as_dict(self):
        return {'num_down_blocks': self.num_down_blocks, 'num_bottleneck_blocks': self.num_bottleneck_blocks}


def _bn(out, p, c):
    out += [(f'{p}.weight', (c,)), (f'{p}.bias', (c,)), (f'{p}.running_mean', (c,)),
            (f'{p}.running_var', (c,)), (f'{p}.num_batches_tracked', (), 'int64')]


def generator_spec(g: GeneratorConfig, prefix='', lfae=None):
    """Generator entries in reference registration order (generator.py:26-62).
    With `lfae` (an LfaeConfig) the pixelwise_flow_predictor, registered first,
    is included; without it only the decoder-side entries (first, down_blocks,
    up_blocks, bottleneck, final) are listed."""
    out = []
    if lfae is not None:
        _pixelwise_flow_predictor(out, f'{prefix}pixelwise_flow_predictor', lfae)
    be, mf = g.block_expansion, g.max_features
    out += [(f'{prefix}first.conv.weight', (be, g.num_channels, 7, 7)), (f'{prefix}first.conv.bias', (be,))]
    _bn(out, f'{prefix}first.norm', be)
    for i in range(g.num_down_blocks):
        ci, co = min(mf, be * 2 ** i), min(mf, be * 2 ** (i + 1))
        out += [(f'{prefix}down_blocks.{i}.conv.weight', (co, ci, 3, 3)), (f'{prefix}down_blocks.{i}.conv.bias', (co,))]
        _bn(out, f'{prefix}down_blocks.{i}.norm', co)
    for i in range(g.num_down_blocks):
        ci = min(mf, be * 2 ** (g.num_down_blocks - i))
        co = min(mf, be * 2 ** (g.num_down_blocks - i - 1))
        out += [(f'{prefix}up_blocks.{i}.conv.weight', (co, ci, 3, 3)), (f'{prefix}up_blocks.{i}.conv.bias', (co,))]
        _bn(out, f'{prefix}up_blocks.{i}.norm', co)
    c = min(mf, be * 2 ** g.num_down_blocks)
    for i in range(g.num_bottleneck_blocks):
        p = f'{prefix}bottleneck.r{i}'
        out += [(f'{p}.conv1.weight', (c, c, 3, 3)), (f'{p}.conv1.bias', (c,)),
                (f'{p}.conv2.weight', (c, c, 3, 3)), (f'{p}.conv2.bias', (c,))]
        _bn(out, f'{p}.norm1', c)
        _bn(out, f'{p}.norm2', c)
    out += [(f'{prefix}final.weight', (g.num_channels, be, 7, 7)), (f'{prefix}final.bias', (g.num_channels,))]
    return [(e[0], tuple(e[1]), e[2] if len(e) > 2 else 'float32') for e in out]


# ---------------------------------------------------------------------------
# LFAE encoder side: RegionPredictor, BGMotionPredictor,
# PixelwiseFlowPredictor — model/LFAE/{region_predictor,bg_motion_predictor,
# pixelwise_flow_predictor,util}.py
# ---------------------------------------------------------------------------

@dataclass
class LfaeConfig:
    """flow_params.model_params of config/DM/*.yaml (defaults: bair.yaml:34-68)."""
    num_regions: int = 10
    num_channels: int = 3
    estimate_affine: bool = True
    revert_axis_swap: bool = True
    image: int = 64
    # bg_predictor_params
    bg_block_expansion: int = 32
    bg_max_features: int = 1024
    bg_num_blocks: int = 5
    bg_type: str = 'affine'
    # region_predictor_params
    rp_temperature: float = 0.1
    rp_block_expansion: int = 32
    rp_max_features: int = 1024
    rp_scale_factor: float = 0.5
    rp_num_blocks: int = 5
    rp_pca_based: bool = True
    rp_pad: int = 0
    # generator_params
    gen_block_expansion: int = 64
    gen_max_features: int = 512
    gen_num_down_blocks: int = 2
    gen_num_bottleneck_blocks: int = 6
    # generator_params.pixelwise_flow_predictor_params
    pf_block_expansion: int = 64
    pf_max_features: int = 1024
    pf_num_blocks: int = 5
    pf_scale_factor: float = 0.5
    pf_use_deformed_source: bool = True
    pf_use_covar_heatmap: bool = True
    pf_estimate_occlusion_map: bool = True
    pf_region_var: float = 0.01

    @classmethod
    def from_config(cls, config, estimate_occlusion_map=None):
        """From a loaded config/DM/*.yaml dict. `estimate_occlusion_map` overrides the
        YAML like valid.py:81 does from the CLI flag."""
        m = config['flow_params']['model_params']
        bg, rp, gp = m['bg_predictor_params'], m['region_predictor_params'], m['generator_params']
        pf = gp['pixelwise_flow_predictor_params']
        c = cls(num_regions=m['num_regions'], num_channels=m['num_channels'],
                estimate_affine=m['estimate_affine'], revert_axis_swap=m['revert_axis_swap'],
                image=config['dataset_params']['frame_shape'],
                bg_block_expansion=bg['block_expansion'], bg_max_features=bg['max_features'],
                bg_num_blocks=bg['num_blocks'], bg_type=bg.get('bg_type', 'zero'),
                rp_temperature=rp['temperature'], rp_block_expansion=rp['block_expansion'],
                rp_max_features=rp['max_features'], rp_scale_factor=rp.get('scale_factor', 1),
                rp_num_blocks=rp['num_blocks'], rp_pca_based=rp.get('pca_based', False), rp_pad=rp.get('pad', 3),
                gen_block_expansion=gp['block_expansion'], gen_max_features=gp['max_features'],
                gen_num_down_blocks=gp['num_down_blocks'], gen_num_bottleneck_blocks=gp['num_bottleneck_blocks'],
                pf_block_expansion=pf['block_expansion'], pf_max_features=pf['max_features'],
                pf_num_blocks=pf['num_blocks'], pf_scale_factor=pf.get('scale_factor', 1),
                pf_use_deformed_source=pf.get('use_deformed_source', True),
                pf_use_covar_heatmap=pf.get('use_covar_heatmap', False),
                pf_estimate_occlusion_map=pf.get('estimate_occlusion_map', False),
                pf_region_var=pf.get('region_var', 0.01))
        if estimate_occlusion_map is not None:
            c.pf_estimate_occlusion_map = bool(estimate_occlusion_map)
        return c

    def generator(self):
        return GeneratorConfig(num_channels=self.num_channels, block_expansion=self.gen_block_expansion,
                               max_features=self.gen_max_features, num_down_blocks=self.gen_num_down_blocks,
                               num_bottleneck_blocks=self.gen_num_bottleneck_blocks, image=self.image)

    @property
    def pf_in_features(self):
        return (self.num_regions + 1) * (self.num_channels * int(self.pf_use_deformed_source) + 1)

    @property
    def bg_outputs(self):
        return {'zero': 0, 'shift': 2, 'affine': 6, 'perspective': 8}[self.bg_type]


def aa_kernel_size(scale):
    """AntiAliasInterpolation2d kernel size for `scale` (util.py:224-233)."""
    sigma = (1 / scale - 1) / 2
    return 2 * round(sigma * 4) + 1


def _conv_bn(out, p, ci, co, k):
    out += [(f'{p}.conv.weight', (co, ci, k, k)), (f'{p}.conv.bias', (co,))]
    _bn(out, f'{p}.norm', co)


def _hg_encoder(out, p, be, cin, nb, mf):
    """util.Encoder (util.py:152-168)."""
    for i in range(nb):
        ci = cin if i == 0 else min(mf, be * 2 ** i)
        _conv_bn(out, f'{p}.down_blocks.{i}', ci, min(mf, be * 2 ** (i + 1)), 3)


def _hourglass(out, p, be, cin, nb, mf):
    """util.Hourglass (util.py:171-222); out_filters = be + cin."""
    _hg_encoder(out, f'{p}.encoder', be, cin, nb, mf)
    for j, i in enumerate(range(nb)[::-1]):
        ci = (1 if i == nb - 1 else 2) * min(mf, be * 2 ** (i + 1))
        _conv_bn(out, f'{p}.decoder.up_blocks.{j}', ci, min(mf, be * 2 ** i), 3)


def _pixelwise_flow_predictor(out, p, c: LfaeConfig):
    cin = c.pf_in_features
    _hourglass(out, f'{p}.hourglass', c.pf_block_expansion, cin, c.pf_num_blocks, c.pf_max_features)
    of = c.pf_block_expansion + cin
    out += [(f'{p}.mask.weight', (c.num_regions + 1, of, 7, 7)), (f'{p}.mask.bias', (c.num_regions + 1,))]
    if c.pf_estimate_occlusion_map:
        out += [(f'{p}.occlusion.weight', (1, of, 7, 7)), (f'{p}.occlusion.bias', (1,))]
    if c.pf_scale_factor != 1:
        k = aa_kernel_size(c.pf_scale_factor)
        out += [(f'{p}.down.weight', (c.num_channels, 1, k, k))]


def region_predictor_spec(c: LfaeConfig, prefix=''):
    """RegionPredictor (region_predictor.py:28-60) in registration order."""
    out = []
    _hourglass(out, f'{prefix}predictor', c.rp_block_expansion, c.num_channels, c.rp_num_blocks, c.rp_max_features)
    of = c.rp_block_expansion + c.num_channels
    out += [(f'{prefix}regions.weight', (c.num_regions, of, 7, 7)), (f'{prefix}regions.bias', (c.num_regions,))]
    if c.estimate_affine and not c.rp_pca_based:
        out += [(f'{prefix}jacobian.weight', (4, of, 7, 7)), (f'{prefix}jacobian.bias', (4,))]
    if c.rp_scale_factor != 1:
        k = aa_kernel_size(c.rp_scale_factor)
        out += [(f'{prefix}down.weight', (c.num_channels, 1, k, k))]
    return [(e[0], tuple(e[1]), e[2] if len(e) > 2 else 'float32') for e in out]


def bg_predictor_spec(c: LfaeConfig, prefix=''):
    """BGMotionPredictor (bg_motion_predictor.py:16-44) in registration order."""
    out = []
    if c.bg_type != 'zero':
        _hg_encoder(out, f'{prefix}encoder', c.bg_block_expansion, 2 * c.num_channels, c.bg_num_blocks,
                    c.bg_max_features)
        fin = min(c.bg_max_features, c.bg_block_expansion * 2 ** c.bg_num_blocks)
        out += [(f'{prefix}fc.weight', (c.bg_outputs, fin)), (f'{prefix}fc.bias', (c.bg_outputs,))]
    return [(e[0], tuple(e[1]), e[2] if len(e) > 2 else 'float32') for e in out]
