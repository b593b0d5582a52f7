"""ctypes binding of libextdm_hip.so (include/extdm.h). The library is the
product path: if it is missing or no HIP device is visible, every entry point
raises — there is no CPU or eager-PyTorch fallback."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'libextdm_hip.so')

# every symbol include/extdm.h declares
EXPORTS = ['extdm_create', 'extdm_destroy', 'extdm_last_error', 'extdm_load_weight', 'extdm_finalize',
           'extdm_workspace_bytes', 'extdm_unet_forward', 'extdm_sample', 'extdm_sampler_step', 'extdm_bench_layer',
           'extdm_decode']

SAMPLER_DDPM = 0
SAMPLER_DDIM = 1


class ExtdmConfig(ctypes.Structure):
    _fields_ = [('arch', ctypes.c_int), ('dim', ctypes.c_int), ('channels', ctypes.c_int),
                ('dim_mults', ctypes.c_int * 4), ('n_levels', ctypes.c_int), ('window', ctypes.c_int * 3),
                ('heads', ctypes.c_int), ('dim_head', ctypes.c_int), ('tc', ctypes.c_int), ('tp', ctypes.c_int),
                ('latent', ctypes.c_int), ('fea_size', ctypes.c_int), ('fea_ch', ctypes.c_int),
                ('timesteps', ctypes.c_int), ('max_batch', ctypes.c_int), ('device', ctypes.c_int),
                ('image', ctypes.c_int), ('num_channels', ctypes.c_int), ('gen_block_expansion', ctypes.c_int),
                ('gen_max_features', ctypes.c_int), ('gen_num_down_blocks', ctypes.c_int),
                ('gen_num_bottleneck_blocks', ctypes.c_int)]


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
    L.extdm_bench_layer.argtypes = [vp, i32, i32, i32, ctypes.POINTER(f32), ctypes.POINTER(ctypes.c_double)]
    L.extdm_bench_layer.restype = i32
    L.extdm_decode.argtypes = [vp, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp]
    L.extdm_decode.restype = i32
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise RuntimeError('extdm: ' + load().extdm_last_error().decode())


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


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

    def __init__(self, ucfg, timesteps, max_batch, device=0, gcfg=None):
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

    def bench_layer(self, B, layer=0, iters=20):
        ms, fl = ctypes.c_float(), ctypes.c_double()
        check(load().extdm_bench_layer(self.h, B, layer, iters, ctypes.byref(ms), ctypes.byref(fl)))
        return float(ms.value), float(fl.value)

    def decode(self, ref, flow, out, occ=None, warped=None):
        """ref (B,C,S,S), flow (B,2,T,fh,fw), occ (B,1,T,fh,fw) or None -> out (B,C,T,S,S)."""
        _require_device(ref, flow, out, occ, warped)
        B, C, S, _ = ref.shape
        T, fh, fw = flow.shape[2], flow.shape[3], flow.shape[4]
        check(load().extdm_decode(self.h, B, C, T, S, fh, fw, _ptr(ref), _ptr(flow), _ptr(occ), _ptr(out),
                                  _ptr(warped), _stream()))
