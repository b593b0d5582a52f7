"""ctypes binding of libextdm_hip.so (include/extdm.h). The library is the
product path: if it is missing or no HIP device is visible, every entry point
raises — there is no CPU or eager-PyTorch fallback."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('EXTDM_LIB') or os.path.join(HERE, 'libextdm_hip.so')

# every symbol include/extdm.h declares
EXPORTS = ['extdm_create', 'extdm_destroy', 'extdm_last_error', 'extdm_load_weight', 'extdm_finalize',
           'extdm_workspace_bytes', 'extdm_unet_forward', 'extdm_sample', 'extdm_sampler_step', 'extdm_record_thresholds', 'extdm_bench_layer', 'extdm_bench_layer_kernel',
           'extdm_decode', 'extdm_set_lfae', 'extdm_region_params', 'extdm_region_hw', 'extdm_bg_params',
           'extdm_flow_predict', 'extdm_flow_hw', 'extdm_bottleneck', 'extdm_range_flag',
           'extdm_attn_layer', 'extdm_frame_metrics_workspace', 'extdm_frame_metrics', 'extdm_bilinear_frames']

BG_TYPES = {'zero': 0, 'shift': 1, 'affine': 2, 'perspective': 3}

SAMPLER_DDPM = 0
SAMPLER_DDIM = 1

# include/extdm.h EXTDM_PRECISION_*: arithmetic of the direct convolutions
PRECISIONS = {'fp32': 0, 'f16x3': 1, 'bf16_attn': 2}
DEFAULT_PRECISION = os.environ.get('EXTDM_PRECISION', 'f16x3')

class ExtdmConfig(ctypes.Structure):
    _fields_ = [('arch', ctypes.c_int), ('dim', ctypes.c_int), ('channels', ctypes.c_int),
                ('dim_mults', ctypes.c_int * 4), ('n_levels', ctypes.c_int), ('window', ctypes.c_int * 3),
                ('heads', ctypes.c_int), ('dim_head', ctypes.c_int), ('tc', ctypes.c_int), ('tp', ctypes.c_int),
                ('latent', ctypes.c_int), ('fea_size', ctypes.c_int), ('fea_ch', ctypes.c_int),
                ('timesteps', ctypes.c_int), ('max_batch', ctypes.c_int), ('device', ctypes.c_int),
                ('image', ctypes.c_int), ('num_channels', ctypes.c_int), ('gen_block_expansion', ctypes.c_int),
                ('gen_max_features', ctypes.c_int), ('gen_num_down_blocks', ctypes.c_int),
                ('gen_num_bottleneck_blocks', ctypes.c_int), ('precision', ctypes.c_int)]


class ExtdmLfaeConfig(ctypes.Structure):
    _fields_ = [('num_regions', ctypes.c_int), ('num_channels', ctypes.c_int), ('image', ctypes.c_int),
                ('revert_axis_swap', ctypes.c_int), ('rp_temperature', ctypes.c_float),
                ('rp_scale_factor', ctypes.c_float), ('rp_pad', ctypes.c_int), ('rp_num_blocks', ctypes.c_int),
                ('rp_pca_based', ctypes.c_int), ('bg_type', ctypes.c_int), ('bg_num_blocks', ctypes.c_int),
                ('pf_scale_factor', ctypes.c_float), ('pf_region_var', ctypes.c_float),
                ('pf_num_blocks', ctypes.c_int), ('pf_use_covar_heatmap', ctypes.c_int),
                ('pf_use_deformed_source', ctypes.c_int)]


_lib = None


def load():
    """Load the shared library and declare the signatures."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f'ExtDM HIP library not built: {LIB_PATH} (run __graft_entry__.build())')
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, f32, u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_uint64
    L.extdm_create.argtypes = [ctypes.POINTER(ExtdmConfig), ctypes.POINTER(vp)]
    L.extdm_create.restype = i32
    L.extdm_destroy.argtypes = [vp]
    L.extdm_destroy.restype = None
    L.extdm_last_error.argtypes = []
    L.extdm_last_error.restype = ctypes.c_char_p
    L.extdm_load_weight.argtypes = [vp, ctypes.c_char_p, vp, i32, ctypes.POINTER(i64), i32]
    L.extdm_load_weight.restype = i32
    L.extdm_finalize.argtypes = [vp]
    L.extdm_finalize.restype = i32
    L.extdm_workspace_bytes.argtypes = [vp]
    L.extdm_workspace_bytes.restype = i64
    L.extdm_unet_forward.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp]
    L.extdm_unet_forward.restype = i32
    L.extdm_sample.argtypes = [vp, i32, i32, i32, ctypes.POINTER(i32), ctypes.POINTER(i32), f32, vp, vp, vp, vp,
                               u64, i32, i32, vp, i32, vp]
    L.extdm_sample.restype = i32
    L.extdm_sampler_step.argtypes = [vp, i32, i32, i32, i32, f32, vp, vp, vp, vp, vp]
    L.extdm_sampler_step.restype = i32
    L.extdm_record_thresholds.argtypes = [vp, vp, i64]
    L.extdm_record_thresholds.restype = i32
    L.extdm_bench_layer.argtypes = [vp, i32, i32, i32, ctypes.POINTER(f32), ctypes.POINTER(ctypes.c_double)]
    L.extdm_bench_layer.restype = i32
    L.extdm_bench_layer_kernel.argtypes = [vp, i32, ctypes.c_char_p, i32]
    L.extdm_bench_layer_kernel.restype = i32
    L.extdm_decode.argtypes = [vp, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp]
    L.extdm_decode.restype = i32
    L.extdm_set_lfae.argtypes = [vp, ctypes.POINTER(ExtdmLfaeConfig)]
    L.extdm_set_lfae.restype = i32
    L.extdm_region_params.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, vp, vp]
    L.extdm_region_params.restype = i32
    L.extdm_region_hw.argtypes = [vp]
    L.extdm_region_hw.restype = i32
    L.extdm_bg_params.argtypes = [vp, i32, vp, vp, vp, vp]
    L.extdm_bg_params.restype = i32
    L.extdm_flow_predict.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.extdm_flow_predict.restype = i32
    L.extdm_flow_hw.argtypes = [vp]
    L.extdm_flow_hw.restype = i32
    L.extdm_bottleneck.argtypes = [vp, i32, vp, vp, vp]
    L.extdm_bottleneck.restype = i32
    L.extdm_attn_layer.argtypes = [vp, ctypes.c_char_p, i32, i32, i32, i32, i32, i32, vp, vp, vp]
    L.extdm_attn_layer.restype = i32
    L.extdm_range_flag.argtypes = [vp, i32, vp]
    L.extdm_range_flag.restype = i32
    L.extdm_frame_metrics_workspace.argtypes = [i32, i32, i32, i32, i32]
    L.extdm_frame_metrics_workspace.restype = ctypes.c_size_t
    L.extdm_frame_metrics.argtypes = [vp, vp, i32, i32, i32, i32, i32, ctypes.c_long, ctypes.c_long, ctypes.c_long,
                                      vp, vp, vp, vp]
    L.extdm_frame_metrics.restype = i32
    lg = ctypes.c_long
    L.extdm_bilinear_frames.argtypes = [vp, i32, i32, i32, i32, i32, vp, lg, lg, lg, vp, lg, lg, lg, i32, i32, i32, vp]
    L.extdm_bilinear_frames.restype = i32
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise RuntimeError('extdm: ' + load().extdm_last_error().decode())


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def bilinear_frames(a, b, t_split, T, size):
    """Bilinear resize (align_corners=False) into a new contiguous [B, C, T, size, size] tensor:
    frames t < t_split from a[:, :, t], the rest from b[:, :, t - t_split] (b may have a frame
    stride of 0, e.g. an expand()ed single frame). a / b: CUDA fp32 [B, C, t, H, W] with
    contiguous H*W planes (extdm_bilinear_frames)."""
    import torch
    src = a if a is not None else b
    Bn, C, _, H, W = src.shape
    out = torch.empty(Bn, C, T, size[0], size[1], device=src.device, dtype=torch.float32)
    for x in (a, b):
        if x is not None:
            if not x.is_cuda:
                raise RuntimeError('ExtDM HIP path needs tensors on a ROCm device (no CPU fallback)')
            if x.dtype != torch.float32 or x.stride(-1) != 1 or x.stride(-2) != x.shape[-1] or x.shape[-2:] != (H, W):
                raise ValueError('bilinear_frames: fp32 [B, C, t, H, W] with contiguous planes expected')
    sa = a.stride()[:3] if a is not None else (0, 0, 0)
    sb = b.stride()[:3] if b is not None else (0, 0, 0)
    with torch.cuda.device(src.device):
        check(load().extdm_bilinear_frames(_ptr(out), Bn, C, T, size[0], size[1], _ptr(a), *sa, _ptr(b), *sb, t_split,
                                           H, W, _stream()))
    return out


def _stream():
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _require_device(*tensors):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError('ExtDM HIP path needs tensors on a ROCm device (no CPU fallback)')
        if not t.is_contiguous() or t.dtype.is_floating_point and t.dtype != __import__('torch').float32:
            raise RuntimeError('ExtDM HIP path needs contiguous float32 tensors')


class Handle:
    """One native model instance (Unet3D weights + diffusion buffers [+ decoder])."""

    def __init__(self, ucfg, timesteps, max_batch, device=0, gcfg=None, precision=None):
        L = load()
        c = ExtdmConfig()
        from .spec import ARCH_IDS
        c.arch = ARCH_IDS[ucfg.arch]
        c.dim = ucfg.dim
        c.channels = ucfg.channels
        mults = list(ucfg.dim_mults)
        for i, m in enumerate(mults):
            c.dim_mults[i] = m
        c.n_levels = len(mults)
        for i, w in enumerate(ucfg.window):
            c.window[i] = w
        c.heads = ucfg.heads
        c.dim_head = ucfg.dim_head
        c.tc, c.tp = ucfg.tc, ucfg.tp
        c.latent = ucfg.latent
        c.fea_size = ucfg.fea_size
        c.fea_ch = ucfg.fea_ch
        c.timesteps = timesteps
        c.max_batch = max_batch
        c.device = device
        if gcfg is None:
            from .spec import GeneratorConfig
            gcfg = GeneratorConfig(image=2 * ucfg.latent)
        c.image = gcfg.image
        c.num_channels = gcfg.num_channels
        c.gen_block_expansion = gcfg.block_expansion
        c.gen_max_features = gcfg.max_features
        c.gen_num_down_blocks = gcfg.num_down_blocks
        c.gen_num_bottleneck_blocks = gcfg.num_bottleneck_blocks
        self.precision = precision or DEFAULT_PRECISION
        if self.precision not in PRECISIONS:
            raise ValueError(f'precision must be one of {sorted(PRECISIONS)}, got {self.precision!r}')
        c.precision = PRECISIONS[self.precision]
        self.cfg = ucfg
        self.max_batch = max_batch
        self.timesteps = timesteps
        h = ctypes.c_void_p()
        check(L.extdm_create(ctypes.byref(c), ctypes.byref(h)))
        self.h = h
        self.n = 3 * ucfg.tp * ucfg.latent * ucfg.latent

    def __del__(self):
        if getattr(self, 'h', None) and _lib is not None:
            _lib.extdm_destroy(self.h)
            self.h = None

    def load_state(self, sd):
        """sd: name -> CPU tensor (float32 or int64)."""
        import torch
        L = load()
        for name, t in sd.items():
            t = t.detach().to('cpu').contiguous()
            if t.dtype == torch.int64:
                dt = 1
            else:
                t = t.to(torch.float32)
                dt = 0
            shape = (ctypes.c_int64 * max(1, t.dim()))(*t.shape)
            check(L.extdm_load_weight(self.h, name.encode(), ctypes.c_void_p(t.data_ptr()), dt, shape, t.dim()))

    def finalize(self):
        check(load().extdm_finalize(self.h))

    def workspace_bytes(self):
        return int(load().extdm_workspace_bytes(self.h))

    def unet_forward(self, x, t, cond, fea, out):
        _require_device(x, cond, fea, out)
        check(load().extdm_unet_forward(self.h, x.shape[0], _ptr(x), _ptr(t), _ptr(cond), _ptr(fea), _ptr(out),
                                        _stream()))

    def sample(self, sampler, times, times_next, eta, x_cond, cond_fea, out, x_T=None, noise=None, seed=0,
               sample_base=0, round_idx=0, use_graph=True):
        _require_device(x_cond, cond_fea, out, x_T, noise)
        S = len(times)
        ta = (ctypes.c_int * S)(*times)
        tn = (ctypes.c_int * S)(*(times_next if times_next is not None else [0] * S))
        check(load().extdm_sample(self.h, out.shape[0], sampler, S, ta, tn, float(eta), _ptr(x_cond),
                                  _ptr(cond_fea), _ptr(x_T), _ptr(noise), ctypes.c_uint64(seed), sample_base,
                                  round_idx, _ptr(out), 1 if use_graph else 0, _stream()))

    def sampler_step(self, sampler, t, t_next, eta, x, eps, noise=None, thresh_out=None):
        _require_device(x, eps, noise, thresh_out)
        check(load().extdm_sampler_step(self.h, x.shape[0], sampler, int(t), int(t_next), float(eta), _ptr(x),
                                        _ptr(eps), _ptr(noise), _ptr(thresh_out), _stream()))

    def record_thresholds(self, buf):
        """Record every later sample() call's per-step thresholds into buf[k * B + b] (device
        fp32; None stops). The tensor must stay alive while recording is on."""
        _require_device(buf)
        self._thresh_buf = buf
        check(load().extdm_record_thresholds(self.h, _ptr(buf), 0 if buf is None else buf.numel()))

    def range_flag(self, reset=True):
        """1 if an f16x3 conv input reached |v| >= 65504 since the last reset."""
        rc = load().extdm_range_flag(self.h, 1 if reset else 0, _stream())
        if rc < 0:
            check(rc)
        return rc

    def attn_layer(self, prefix, x, out, shifted=False):
        """One attention layer (STW or temporal) of the forward: x, out (B,C,T,H,W)."""
        _require_device(x, out)
        B, C, T, H, W = x.shape
        check(load().extdm_attn_layer(self.h, prefix.encode(), B, C, T, H, W, int(shifted), _ptr(x), _ptr(out),
                                      _stream()))

    def bench_layer(self, B, layer=0, iters=20):
        ms, fl = ctypes.c_float(), ctypes.c_double()
        check(load().extdm_bench_layer(self.h, B, layer, iters, ctypes.byref(ms), ctypes.byref(fl)))
        return float(ms.value), float(fl.value)

    def bench_layer_kernel(self, layer):
        """The kernel template the last bench_layer(layer) launched ('' if not recorded)."""
        buf = ctypes.create_string_buffer(256)
        check(load().extdm_bench_layer_kernel(self.h, layer, buf, 256))
        return buf.value.decode()

    # ---- LFAE encoder (include/extdm.h) ----
    def set_lfae(self, lc):
        c = ExtdmLfaeConfig()
        c.num_regions, c.num_channels, c.image = lc.num_regions, lc.num_channels, lc.image
        c.revert_axis_swap = int(lc.revert_axis_swap)
        c.rp_temperature, c.rp_scale_factor = lc.rp_temperature, lc.rp_scale_factor
        c.rp_pad, c.rp_num_blocks, c.rp_pca_based = lc.rp_pad, lc.rp_num_blocks, int(lc.rp_pca_based)
        c.bg_type, c.bg_num_blocks = BG_TYPES[lc.bg_type], lc.bg_num_blocks
        c.pf_scale_factor, c.pf_region_var = lc.pf_scale_factor, lc.pf_region_var
        c.pf_num_blocks = lc.pf_num_blocks
        c.pf_use_covar_heatmap, c.pf_use_deformed_source = int(lc.pf_use_covar_heatmap), int(lc.pf_use_deformed_source)
        check(load().extdm_set_lfae(self.h, ctypes.byref(c)))

    def region_hw(self):
        return int(load().extdm_region_hw(self.h))

    def flow_hw(self):
        return int(load().extdm_flow_hw(self.h))

    def region_params(self, img, shift, covar, affine, u=None, sv=None, heat=None):
        _require_device(img, shift, covar, affine, u, sv, heat)
        check(load().extdm_region_params(self.h, img.shape[0], _ptr(img), _ptr(shift), _ptr(covar), _ptr(affine),
                                         _ptr(u), _ptr(sv), _ptr(heat), _stream()))

    def bg_params(self, src, drv, out):
        _require_device(src, drv, out)
        check(load().extdm_bg_params(self.h, out.shape[0], _ptr(src), _ptr(drv), _ptr(out), _stream()))

    def flow_predict(self, src, drv, srcp, bg, flow, occ=None):
        """drv / srcp: dicts with contiguous 'shift', 'covar', 'affine' device tensors."""
        _require_device(src, bg, flow, occ, *[d[k] for d in (drv, srcp) for k in ('shift', 'covar', 'affine')])
        check(load().extdm_flow_predict(self.h, src.shape[0], _ptr(src), _ptr(drv['shift']), _ptr(drv['covar']),
                                        _ptr(drv['affine']), _ptr(srcp['shift']), _ptr(srcp['covar']),
                                        _ptr(srcp['affine']), _ptr(bg), _ptr(flow), _ptr(occ), _stream()))

    def bottleneck(self, img, out):
        _require_device(img, out)
        check(load().extdm_bottleneck(self.h, img.shape[0], _ptr(img), _ptr(out), _stream()))

    def decode(self, ref, flow, out, occ=None, warped=None):
        """ref (B,C,S,S), flow (B,2,T,fh,fw), occ (B,1,T,fh,fw) or None -> out (B,C,T,S,S)."""
        _require_device(ref, flow, out, occ, warped)
        B, C, S, _ = ref.shape
        T, fh, fw = flow.shape[2], flow.shape[3], flow.shape[4]
        check(load().extdm_decode(self.h, B, C, T, S, fh, fw, _ptr(ref), _ptr(flow), _ptr(occ), _ptr(out),
                                  _ptr(warped), _stream()))
