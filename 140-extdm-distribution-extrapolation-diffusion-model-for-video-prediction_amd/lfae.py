"""Drop-in mirrors of the LFAE modules and the FlowDiffusion sampling wrapper,
backed by libextdm_hip.so.

  RegionPredictor     model/LFAE/region_predictor.py:28-150 (PCA-based)
  BGMotionPredictor   model/LFAE/bg_motion_predictor.py:10-64
  Generator           model/LFAE/generator.py:15-206 (+ PixelwiseFlowPredictor,
                      pixelwise_flow_predictor.py:16-153)
  FlowDiffusion       model/BaseDM_adaptor/VideoFlowDiffusion_multi_w_ref.py:18-316
                      (u12 / u22 / ada denoisers; the wo_ref wrapper multi1248.py:213-295
                      via `wrapper='multi1248'`)
  autoregressive_sample   scripts/DM/valid.py:141-186

Constructor signatures, output dict keys and state_dict layouts follow the
reference, so AE checkpoints ('generator', 'region_predictor', 'bg_predictor')
load with the reference's strictness. Every forward runs on the HIP library;
CPU tensors raise.
"""
import dataclasses

import torch
from torch import nn

from . import _lib
from .models import (UNET3D_BY_MODULE, GaussianDiffusion, _register_tree)
from .spec import (GeneratorConfig, LfaeConfig, UnetConfig, ARCH_U12, ARCH_ADA_U22, ARCH_WO_REF, bg_predictor_spec,
                   generator_spec, region_predictor_spec)
from .weights import synth_state_dict


def _need_device(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError('ExtDM HIP path needs tensors on a ROCm device (no CPU fallback)')


class _NativeModule(nn.Module):
    """A module whose forward runs on its own native handle (weights under `PREFIX`)."""
    PREFIX = ''

    def _setup(self, lcfg, spec, seed):
        self.lcfg = lcfg
        _register_tree(self, spec, synth_state_dict(spec, seed=seed))
        self._handle = None

    def _state_version(self):
        return tuple((p.data_ptr(), p._version) for p in self.parameters())

    def _h(self, device, N, T=1):
        """Native handle sized for N images (and T frames per decode call)."""
        dev = device.index or 0
        h = self._handle
        ver = self._state_version()
        if h is None or h[0] != dev or h[1] < N or h[2] < T or h[3] != ver:
            lc = self.lcfg
            flow = int(lc.image * lc.pf_scale_factor) if lc.pf_scale_factor != 1 else lc.image // 2
            same = h is not None and h[0] == dev
            N2, T2 = max(N, h[1] if same else 0), max(T, 2, h[2] if same else 0)
            ucfg = UnetConfig(tc=1, tp=T2 - 1, latent=flow)
            nh = _lib.Handle(ucfg, 1000, N2, dev, gcfg=lc.generator())
            nh.set_lfae(lc)
            nh.load_state({self.PREFIX + k: v for k, v in self.state_dict().items()})
            nh.finalize()
            self._handle = h = (dev, N2, T2, ver, nh)
        return h[4]


class RegionPredictor(_NativeModule):
    """RegionPredictor (region_predictor.py:28-150). Only the PCA-based variant
    the configs use (pca_based=True) is implemented; returns shift, covar,
    heatmap, affine, u, d like the reference."""
    PREFIX = 'region_predictor.'

    def __init__(self, block_expansion, num_regions, num_channels, max_features, num_blocks, temperature,
                 estimate_affine=False, scale_factor=1, pca_based=False, fast_svd=False, pad=3, image_size=64,
                 seed=2469):
        super().__init__()
        if not pca_based:
            raise NotImplementedError('only the PCA-based region predictor is configured (config/DM/*.yaml)')
        lc = LfaeConfig(num_regions=num_regions, num_channels=num_channels, estimate_affine=estimate_affine,
                        image=image_size, rp_temperature=temperature, rp_block_expansion=block_expansion,
                        rp_max_features=max_features, rp_scale_factor=scale_factor, rp_num_blocks=num_blocks,
                        rp_pca_based=pca_based, rp_pad=pad)
        self._setup(lc, region_predictor_spec(lc), seed)

    @torch.no_grad()
    def forward(self, x):
        _need_device(x)
        x = x.float().contiguous()
        N, R = x.shape[0], self.lcfg.num_regions
        h = self._h(x.device, N)
        hw = h.region_hw()
        o = {k: torch.empty(s, device=x.device) for k, s in
             (('shift', (N, R, 2)), ('covar', (N, R, 2, 2)), ('affine', (N, R, 2, 2)), ('u', (N, R, 2, 2)),
              ('sv', (N, R, 2)), ('heatmap', (N, R, hw, hw)))}
        h.region_params(x, o['shift'], o['covar'], o['affine'], o['u'], o['sv'], o['heatmap'])
        return {'shift': o['shift'], 'covar': o['covar'], 'heatmap': o['heatmap'], 'affine': o['affine'],
                'u': o['u'], 'd': torch.diag_embed(o['sv'])}


class BGMotionPredictor(_NativeModule):
    """BGMotionPredictor (bg_motion_predictor.py:10-64): a 3x3 background transform."""
    PREFIX = 'bg_predictor.'

    def __init__(self, block_expansion, num_channels, max_features, num_blocks, bg_type='zero', image_size=64,
                 seed=2470):
        super().__init__()
        assert bg_type in ['zero', 'shift', 'affine', 'perspective']
        lc = LfaeConfig(num_channels=num_channels, image=image_size, bg_block_expansion=block_expansion,
                        bg_max_features=max_features, bg_num_blocks=num_blocks, bg_type=bg_type)
        self.bg_type = bg_type
        self._setup(lc, bg_predictor_spec(lc), seed)

    @torch.no_grad()
    def forward(self, source_image, driving_image):
        _need_device(source_image, driving_image)
        src = source_image.float().contiguous()
        drv = driving_image.float().contiguous()
        out = torch.empty(src.shape[0], 3, 3, device=src.device)
        self._h(src.device, src.shape[0]).bg_params(src, drv, out)
        return out


class Generator(_NativeModule):
    """LFAE Generator (generator.py:15-206). With pixelwise_flow_predictor_params
    it is the full module (forward = flow prediction + warp decoder); without,
    the decoder half used by sample_one_video's forward_with_flow."""
    PREFIX = 'generator.'

    def __init__(self, num_channels=3, num_regions=10, block_expansion=64, max_features=512, num_down_blocks=2,
                 num_bottleneck_blocks=6, pixelwise_flow_predictor_params=None, skips=True, revert_axis_swap=True,
                 image_size=64, seed=4321, **unused):
        super().__init__()
        if not skips:
            raise NotImplementedError('the reference configs use skips=True')
        pf = dict(pixelwise_flow_predictor_params or {})
        lc = LfaeConfig(num_regions=num_regions, num_channels=num_channels, revert_axis_swap=revert_axis_swap,
                        image=image_size, gen_block_expansion=block_expansion, gen_max_features=max_features,
                        gen_num_down_blocks=num_down_blocks, gen_num_bottleneck_blocks=num_bottleneck_blocks,
                        pf_block_expansion=pf.get('block_expansion', 64), pf_max_features=pf.get('max_features', 1024),
                        pf_num_blocks=pf.get('num_blocks', 5), pf_scale_factor=pf.get('scale_factor', 1),
                        pf_use_deformed_source=pf.get('use_deformed_source', True),
                        pf_use_covar_heatmap=pf.get('use_covar_heatmap', False),
                        pf_estimate_occlusion_map=pf.get('estimate_occlusion_map', False),
                        pf_region_var=pf.get('region_var', 0.01))
        self.has_flow_predictor = pixelwise_flow_predictor_params is not None
        self.gcfg = lc.generator()
        self._setup(lc, generator_spec(self.gcfg, lfae=lc if self.has_flow_predictor else None), seed)

    @torch.no_grad()
    def forward(self, source_image, driving_region_params, source_region_params, bg_params=None):
        """generator.py:104-144."""
        if not self.has_flow_predictor:
            raise RuntimeError('Generator.forward needs pixelwise_flow_predictor_params')
        _need_device(source_image)
        src = source_image.float().contiguous()
        N, C, S, _ = src.shape
        h = self._h(src.device, N)
        fh = h.flow_hw()
        flow = torch.empty(N, 2, fh, fh, device=src.device)
        occ = torch.empty(N, 1, fh, fh, device=src.device) if self.lcfg.pf_estimate_occlusion_map else None
        cont = lambda d: {k: d[k].float().contiguous() for k in ('shift', 'covar', 'affine')}
        bg = bg_params.float().contiguous() if bg_params is not None else None
        h.flow_predict(src, cont(driving_region_params), cont(source_region_params), bg, flow, occ)
        pred = torch.empty(N, C, 1, S, S, device=src.device)
        warped = torch.empty_like(pred)
        h.decode(src, flow[:, :, None], pred, occ=occ[:, :, None] if occ is not None else None, warped=warped)
        out = {'bottle_neck_feat': self.forward_bottle(src), 'deformed': warped[:, :, 0],
               'optical_flow': flow.permute(0, 2, 3, 1)}
        if occ is not None:
            out['occlusion_map'] = occ
        out['prediction'] = pred[:, :, 0]
        return out

    @torch.no_grad()
    def forward_bottle(self, source_image):
        """generator.py:95-102: the bottleneck feature of the encoder half."""
        _need_device(source_image)
        src = source_image.float().contiguous()
        N, _, S, _ = src.shape
        g = self.gcfg
        c = min(g.max_features, g.block_expansion * 2 ** g.num_down_blocks)
        out = torch.empty(N, c, S >> g.num_down_blocks, S >> g.num_down_blocks, device=src.device)
        self._h(src.device, N).bottleneck(src, out)
        return out

    compute_fea = forward_bottle

    @torch.no_grad()
    def forward_with_flow(self, source_image, optical_flow, occlusion_map):
        """Reference signature (generator.py:152): optical_flow (B, h, w, 2),
        occlusion_map (B, 1, h, w) or None. Returns 'prediction' and 'deformed'."""
        flow = optical_flow.permute(0, 3, 1, 2)[:, :, None]
        occ = occlusion_map[:, :, None] if occlusion_map is not None else None
        pred, warped = self.decode_frames(source_image, flow, occ, with_warped=True)
        return {'prediction': pred[:, :, 0], 'deformed': warped[:, :, 0]}

    @torch.no_grad()
    def decode_frames(self, source_image, flow, occ=None, with_warped=False):
        """All frames at once: source_image (B,C,S,S), flow (B,2,T,h,w), occ (B,1,T,h,w)
        or None -> prediction (B,C,T,S,S) [, deformed]. The encoder half runs once per clip."""
        _need_device(source_image, flow, occ)
        src = source_image.float().contiguous()
        fl = flow.float().contiguous()
        oc = occ.float().contiguous() if occ is not None else None
        B, C, S, _ = src.shape
        T = fl.shape[2]
        pred = torch.empty(B, C, T, S, S, device=src.device, dtype=torch.float32)
        warped = torch.empty_like(pred) if with_warped else None
        self._h(src.device, B, T).decode(src, fl, pred, occ=oc, warped=warped)
        return (pred, warped) if with_warped else pred


class FlowDiffusion(nn.Module):
    """FlowDiffusion (VideoFlowDiffusion_multi_w_ref.py:18-118), sampling half.

    `wrapper` picks the reference wrapper whose sample_one_video is mirrored:
    'multi_w_ref' (default; u12/u22/ada, channels 256+256, init_noise_conv path),
    'multi_w_ref_u22' (ada_u22, channels 3+256; VideoFlowDiffusion_multi_w_ref_u22.py:143-510
    without its hard-wired cuda:0/cuda:1 model split) or 'multi1248' (wo_ref,
    channels 3+256, dim_mults (1,2,4,8))."""

    def __init__(self, config, pretrained_pth="", is_train=False, ddim_sampling_eta=1., timesteps=1000,
                 dim_mults=(1, 2, 4, 4), learn_null_cond=False, use_deconv=True, padding_mode="zeros",
                 withFea=True, Unet3D_architecture="DenoiseNet_STWAtt_w_w_ref_adaptor_cross_multi_traj_ada",
                 wrapper='multi_w_ref'):
        super().__init__()
        if is_train:
            raise NotImplementedError('training (FlowDiffusion.forward / p_losses) is out of scope')
        fp = config['flow_params']['model_params']
        dp = config['diffusion_params']['model_params']
        ds = config['dataset_params']
        self.lcfg = LfaeConfig.from_config(config)
        self.estimate_occlusion_map = self.lcfg.pf_estimate_occlusion_map
        self.use_residual_flow = dp['use_residual_flow']
        if self.use_residual_flow:
            raise NotImplementedError('use_residual_flow=True is not used by any reference config')
        self.wrapper = wrapper
        if wrapper == 'multi1248' and not self.estimate_occlusion_map:
            # multi1248.py:236 reads generated["occlusion_map"] unconditionally
            raise KeyError('occlusion_map: the multi1248 wrapper needs estimate_occlusion_map=True')
        if wrapper == 'multi_w_ref_u22' and not self.estimate_occlusion_map:
            # multi_w_ref_u22.py:496-498 decodes with occlusion_map=sample_conf.to(...): None has no .to
            raise AttributeError("'NoneType' object has no attribute 'to': the multi_w_ref_u22 wrapper needs "
                                 "estimate_occlusion_map=True")
        S = ds['frame_shape']
        self.generator = Generator(num_regions=fp['num_regions'], num_channels=fp['num_channels'],
                                   revert_axis_swap=fp['revert_axis_swap'], image_size=S, **fp['generator_params'])
        self.region_predictor = RegionPredictor(num_regions=fp['num_regions'], num_channels=fp['num_channels'],
                                                estimate_affine=fp['estimate_affine'], image_size=S,
                                                **fp['region_predictor_params'])
        self.bg_predictor = BGMotionPredictor(num_channels=fp['num_channels'], image_size=S,
                                              **fp['bg_predictor_params'])
        if pretrained_pth:
            ck = torch.load(pretrained_pth, map_location='cpu', weights_only=True)
            self.generator.load_state_dict(ck['generator'], strict=False)
            self.region_predictor.load_state_dict(ck['region_predictor'])
            self.bg_predictor.load_state_dict(ck['bg_predictor'])
        tc, tp = ds['train_params']['cond_frames'], ds['train_params']['pred_frames']
        if wrapper == 'multi1248':
            arch, channels = ARCH_WO_REF, 3 + 256
        elif wrapper == 'multi_w_ref_u22':
            # hard-imports ada_u22 whatever Unet3D_architecture says (multi_w_ref_u22.py:16, 199-213)
            arch, channels = ARCH_ADA_U22, 3 + 256
        else:
            arch, channels = Unet3D_architecture, 256 + 256
        unet_cls = UNET3D_BY_MODULE[arch]
        self.unet = unet_cls(dim=64, channels=channels, out_grid_dim=2, out_conf_dim=1, dim_mults=dim_mults,
                             use_bert_text_cond=False, learn_null_cond=learn_null_cond, use_final_activation=False,
                             use_deconv=use_deconv, padding_mode=padding_mode, cond_num=tc, pred_num=tp,
                             framesize=int(S * fp['region_predictor_params']['scale_factor']))
        self.diffusion = GaussianDiffusion(self.unet, image_size=S // 2, num_frames=tc + tp,
                                           sampling_timesteps=dp['sampling_timesteps'], timesteps=timesteps,
                                           loss_type=dp['loss_type'], use_dynamic_thres=True,
                                           null_cond_prob=dp['null_cond_prob'], ddim_sampling_eta=ddim_sampling_eta)
        self.cond_frame_num, self.pred_frame_num = tc, tp
        self.frame_num = tc + tp

    @torch.no_grad()
    def encode(self, real_vid):
        """The encoder part of sample_one_video (multi_w_ref.py:223-275 /
        multi1248.py:213-257): per cond frame, region and background params vs
        the reference frame (cond frame tc-1), Generator.forward; the conditioning
        x_cond and cond_fea. All tc frames go through each module in one batched call."""
        tc, tp = self.cond_frame_num, self.pred_frame_num
        B = real_vid.shape[0]
        vid = real_vid.float()
        ref = vid[:, :, tc - 1].contiguous()
        frames = vid.permute(2, 0, 1, 3, 4).reshape(tc * B, *vid.shape[1:2], *vid.shape[3:]).contiguous()
        refs = ref.repeat(tc, 1, 1, 1)
        src_p = self.region_predictor(ref)
        src_p = {k: v.repeat(tc, *([1] * (v.dim() - 1))) for k, v in src_p.items()}
        drv_p = self.region_predictor(frames)
        bg = self.bg_predictor(refs, frames)
        g = self.generator(refs, source_region_params=src_p, driving_region_params=drv_p, bg_params=bg)
        tb = lambda x: x.reshape(tc, B, *x.shape[1:]).movedim(0, 2)  # (tc*B, ...) -> (B, ..., tc, ...)
        ret = {'real_vid_grid': tb(g['optical_flow'].permute(0, 3, 1, 2)).contiguous()}
        if self.estimate_occlusion_map:
            ret['real_vid_conf'] = tb(g['occlusion_map']).contiguous()
        ret['real_out_vid'] = tb(g['prediction']).contiguous()
        ret['real_warped_vid'] = tb(g['deformed']).contiguous()
        # cond_fea: forward_bottle of cond frames 0..tc-2, then the last generator call's
        # bottle_neck_feat (the bottleneck of the reference frame) repeated
        ref_fea = g['bottle_neck_feat'][(tc - 1) * B:]
        early = self.generator.forward_bottle(frames[:(tc - 1) * B]) if tc > 1 else ref_fea[:0]
        early = early.reshape(tc - 1, B, *ref_fea.shape[1:])
        if self.wrapper == 'multi1248':
            # ... x tp, bilinear to the flow size (multi1248.py:240-245), on the HIP library: the
            # tc - 1 early maps and ONE resize of the repeated reference map per output frame
            # (a frame stride of 0), written straight into the [B, C, tc - 1 + tp, fs, fs] tensor
            fs = ret['real_vid_grid'].shape[-1]
            # (fp32 with contiguous H x W planes, as the kernel takes them: a no-op for the
            # native generator's output, a conversion for an fp16 / channels-last bottleneck)
            early_t = early.permute(1, 2, 0, 3, 4).float().contiguous()  # [B, C, tc - 1, h, w]
            ref_fea = ref_fea.float().contiguous()
            fea = _lib.bilinear_frames(early_t if tc > 1 else None, ref_fea.unsqueeze(2).expand(-1, -1, tp, -1, -1),
                                       tc - 1, tc - 1 + tp, (fs, fs))
        else:
            feas = [early[i] for i in range(tc - 1)] + [ref_fea] * (1 + tp)
            fea = torch.stack(feas, dim=2)
        if self.estimate_occlusion_map:
            x_cond = torch.cat((ret['real_vid_grid'], ret['real_vid_conf'] * 2 - 1), dim=1)
        else:
            x_cond = torch.cat((ret['real_vid_grid'], torch.zeros_like(ret['real_vid_grid'])[:, 0:1]), dim=1)
        return ret, x_cond.contiguous(), fea.contiguous(), ref

    @torch.no_grad()
    def decode(self, ret, pred, ref):
        """The decode part of sample_one_video (multi_w_ref.py:281-316): grids /
        conf = cat(real cond part, predicted part), forward_with_flow for every frame
        (one batched native call; the encoder half runs once per clip)."""
        tc = self.cond_frame_num
        grid = torch.cat([ret['real_vid_grid'][:, :, :tc], pred[:, :2]], dim=2).contiguous()
        conf = None
        if self.estimate_occlusion_map:
            conf = torch.cat([ret['real_vid_conf'][:, :, :tc], (pred[:, 2].unsqueeze(1) + 1) * 0.5], dim=2)
            conf = conf.contiguous()
        out, warped = self.generator.decode_frames(ref, grid, conf, with_warped=True)
        ret = dict(ret)
        ret['sample_vid_grid'] = grid
        if conf is not None:
            ret['sample_vid_conf'] = conf
        ret['sample_out_vid'] = out
        ret['sample_warped_vid'] = warped
        return ret

    def sample_one_video(self, cond_scale, real_vid, **sample_kw):
        """multi_w_ref.py:223-316. `sample_kw` (x_T, noise, seed, sample_base,
        round_idx) reach the native sampler (GaussianDiffusion.sample)."""
        _need_device(real_vid)
        ret, x_cond, fea, ref = self.encode(real_vid)
        self.diffusion.max_batch = max(self.diffusion.max_batch, x_cond.shape[0])
        pred = self.diffusion.sample(x_cond, cond_fea=fea, batch_size=1, cond_scale=cond_scale, **sample_kw)
        return self.decode(ret, pred, ref)


class _WrapperFlowDiffusion(FlowDiffusion):
    """FlowDiffusion with the wrapper fixed by the class, as the reference fixes it by the
    module its FlowDiffusion is imported from (scripts/DM/valid.py imports
    model.BaseDM_adaptor.<DM_arch>.FlowDiffusion)."""
    WRAPPER = 'multi_w_ref'

    def __init__(self, *args, **kwargs):
        kwargs.setdefault('wrapper', self.WRAPPER)
        if kwargs['wrapper'] != self.WRAPPER:
            raise ValueError(f'{type(self).__name__} mirrors the {self.WRAPPER} wrapper, not {kwargs["wrapper"]}')
        super().__init__(*args, **kwargs)


class FlowDiffusionMultiWRef(_WrapperFlowDiffusion):
    """VideoFlowDiffusion_multi_w_ref.FlowDiffusion (:18-316)."""
    WRAPPER = 'multi_w_ref'


class FlowDiffusionMultiWRefU22(_WrapperFlowDiffusion):
    """VideoFlowDiffusion_multi_w_ref_u22.FlowDiffusion (:143-510)."""
    WRAPPER = 'multi_w_ref_u22'


class FlowDiffusionMulti1248(_WrapperFlowDiffusion):
    """VideoFlowDiffusion_multi1248.FlowDiffusion (:213-295)."""
    WRAPPER = 'multi1248'


# reference module name (config `DM_arch`, valid.py's import) -> FlowDiffusion class
FLOW_DIFFUSION_BY_MODULE = {'VideoFlowDiffusion_multi_w_ref': FlowDiffusionMultiWRef,
                            'VideoFlowDiffusion_multi_w_ref_u22': FlowDiffusionMultiWRefU22,
                            'VideoFlowDiffusion_multi1248': FlowDiffusionMulti1248}


@torch.no_grad()
def autoregressive_sample(model, real_vids, total_pred_frames, num_sample_video=1, cond_scale=1.0, seed=None,
                          sample_base=0, round_noise=None):
    """The eval driver's generation loop (scripts/DM/valid.py:141-186): clips
    repeated n times as '(b n)', NUM_AUTOREG = ceil(total / tp) rounds of
    sample_one_video, each conditioned on the last tc decoded frames of the
    previous round. Returns cat(real cond frames, predictions)[:, :, :tc + total].
    With `seed`, round r draws its noise from the counter-based stream keyed by
    (seed, global sample index = sample_base + i, round r), so shards of a batch
    reproduce the unsharded run. `round_noise[r]` = (x_T, noise) injects round r's
    noise instead (parity tests replaying the reference's CPU stream)."""
    from math import ceil
    tc, tp = model.cond_frame_num, model.pred_frame_num
    vids = real_vids.repeat_interleave(num_sample_video, dim=0)
    cur = vids[:, :, :tc].contiguous()
    preds = []
    for r in range(ceil(total_pred_frames / tp)):
        kw = {} if seed is None else {'seed': seed, 'sample_base': sample_base, 'round_idx': r}
        if round_noise is not None:
            kw = {'x_T': round_noise[r][0], 'noise': round_noise[r][1]}
        out = model.sample_one_video(cond_scale=cond_scale, real_vid=cur, **kw)['sample_out_vid']
        preds.append(out[:, :, -tp:])
        cur = out[:, :, -tc:].contiguous()
    pred = torch.cat(preds, dim=2)
    return torch.cat([vids[:, :, :tc], pred[:, :, :total_pred_frames]], dim=2)
