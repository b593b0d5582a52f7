"""Build libextdm_hip.so (gfx950) in-tree with hipcc: the .so travels with the
repository snapshot to the GPU box. No torch extension machinery is involved.

`build(variant=..., opt=..., extra=..., csrc=...)` builds an A/B copy of the library
into _variants/<variant>/ (per-file optimisation levels / extra flags, or the sources of
another revision in csrc) for the GPU measurement scripts (EXTDM_LIB selects it at run
time)."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
REPO = os.path.dirname(HERE)
INCLUDE = os.path.join(REPO, 'include')
LIB = os.path.join(HERE, 'libextdm_hip.so')
SOURCES = ['conv.hip', 'conv_halo.hip', 'conv_x3.hip', 'pw_x3.hip', 'conv_gemm_x3.hip', 'conv_narrow.hip', 'norm.hip', 'attn.hip', 'attn_core.hip', 'stw_fused.hip',
           'stw_x3.hip', 'stw64_x3.hip', 'cross_x3.hip', 'xpath_x3.hip', 'fea_x3.hip', 'metrics.hip', 'sampler.hip', 'decoder.hip', 'lfae.hip', 'runtime.cpp']
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
FLAGS = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-ffp-contract=off', '-I', INCLUDE, '-I', CSRC]
# Per-file flags. The fused f16x3 attention kernels (many independent fp32 lanes of
# work between MFMAs) must not be SLP-vectorised: at -O3 the SLP pass turns their
# scalar fp32 arithmetic into v_pk_mul_f32 / v_pk_add_f32 pairs (DESIGN.md §4.0 build
# note), which also pushes the 8-wave C = 64 kernels past 256 VGPRs into scratch.
# The attention kernels run softmax / splits on MFMA accumulators: with hipcc's default
# AGPR accumulators every such value is copied out (v_accvgpr_read) and back (the cross
# kernel's key-tile loop: 112 copies in 441 instructions); the VGPR form of the MFMAs keeps
# them in VGPRs (the convs' accumulators only meet VALU in the epilogue and keep AGPRs).
VGPR_MFMA = ['-mllvm', '-amdgpu-mfma-vgpr-form=1']
PER_FILE = {'stw_x3.hip': ['-fno-slp-vectorize'] + VGPR_MFMA, 'stw64_x3.hip': ['-fno-slp-vectorize'] + VGPR_MFMA, 'cross_x3.hip': ['-fno-slp-vectorize'] + VGPR_MFMA,
            'attn_core.hip': VGPR_MFMA,
            # the scaled-lo gather split as v_mul + v_fma_mixlo per value (SLP packed it into
            # v_pk_mul / v_pk_fma_f32 with the hi converted back: ~9 VALU per pair)
            'xpath_x3.hip': ['-fno-slp-vectorize'],
            # the SLP-packed form of the sampler's four-wide update (v_pk_mul_f32 on SGPR pairs
            # around the IEEE divisions) returned wrong values in 16-lane groups of one
            # component in ~9 % of launches while a second process ran on the GPU; scalar
            # fp32: 0 in 175 000 (tests/test_gpu_sampler.py)
            'sampler.hip': ['-fno-slp-vectorize'],
            # scalar v_fma_f32 chains (SLP paired them into v_pk_fma_f32 with lane shuffles)
            'conv_narrow.hip': ['-fno-slp-vectorize']}
OPT = {}


def _needs(obj, src):
    if not os.path.exists(obj):
        return True
    deps = [src, os.path.join(os.path.dirname(src), 'kernels.h'), os.path.join(os.path.dirname(src), 'attn_x3_ops.h'), os.path.join(INCLUDE, 'extdm.h'), os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > os.path.getmtime(obj) for d in deps)


def _compile(src, objdir, opt, per_file, extra, csrc=CSRC):
    obj = os.path.join(objdir, src + '.o')
    s = os.path.join(csrc, src)
    if _needs(obj, s):
        flags = [opt.get(src, f) if f == '-O3' else (csrc if f == CSRC else f) for f in FLAGS]
        flags += per_file.get(src, []) + extra.get(src, [])
        cmd = [HIPCC] + flags + (['-x', 'hip'] if src.endswith('.cpp') else []) + ['-c', s, '-o', obj]
        subprocess.run(cmd, check=True)
    return obj


def build(verbose=False, variant=None, opt=None, per_file=None, extra=None, csrc=None):
    if variant:
        objdir = os.path.join(REPO, '_variants', variant, 'obj')
        lib = os.path.join(REPO, '_variants', variant, 'libextdm_hip.so')
    else:
        objdir, lib = os.path.join(CSRC, 'build'), LIB
    opt = OPT if opt is None else opt
    per_file = PER_FILE if per_file is None else per_file
    extra = extra or {}
    os.makedirs(objdir, exist_ok=True)
    jobs = int(os.environ.get('MAX_JOBS', '8'))
    with ThreadPoolExecutor(max_workers=min(jobs, len(SOURCES))) as ex:
        objs = list(ex.map(lambda s: _compile(s, objdir, opt, per_file, extra, csrc or CSRC), SOURCES))
    if not os.path.exists(lib) or any(os.path.getmtime(o) > os.path.getmtime(lib) for o in objs):
        subprocess.run([HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', '-o', lib] + objs, check=True)
    if verbose:
        print('built', lib)
    return lib


if __name__ == '__main__':
    build(verbose=True)
    sys.exit(0)
