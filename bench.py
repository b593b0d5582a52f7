"""ExtDM sampling throughput on MI355X: predicted frames/sec/node.

Workload (BASELINE.json configs[1]): BAIR 64x64 ch3, 2 -> 28 (tc = 2, tp = 14
per autoregressive round x 2 rounds), DDPM 1000 steps, u12 Unet3D (dim 64,
dim_mults 1,2,4,4) behind the multi_w_ref FlowDiffusion wrapper, random-init
weights, synthetic clips resident in HBM, 128 clips per GPU (WORKLOADS['bair']). BAIR eval default: no occlusion map
(valid_DM_bair.sh omits --estimate_occlusion_map).

Step accounting. A "step" is one reverse-diffusion step of the per-GPU clip
batch: one replay of the captured hipGraph (Unet3D forward + fused
threshold / posterior / noise update, Diffusion.py:169-189). One generation =
the eval driver's full 2 -> 28 run (scripts/DM/valid.py:141-186 through the
package's autoregressive_sample): per round the LFAE encoder on the tc cond
frames, the DDPM-1000 reverse loop, the flow-warp decode of the round's
tc + tp frames; then (N > 1) the RCCL all-gather of the generated videos.
  * `--warmup W`: W untimed graph replays (a W-step reverse loop, plus one
    untimed encoder / decoder pass that builds every native handle);
  * `--steps K`: the timed region is ceil(K / steps_per_generation) >= 1
    COMPLETE generations — a partial generation would not deliver frames —
    so the reported `steps` is the number of reverse-diffusion steps actually
    timed (2000 per generation) and `ms_per_step` = timed wall / steps.
`value` = predicted frames delivered / timed wall (max over ranks).

Multi-GPU: `--gpus N` without a torch.distributed launcher spawns N child ranks
(one process per GPU, LOCAL_RANK = GPU index) before any GPU call; under
torch.distributed.run the launcher's WORLD_SIZE / RANK / LOCAL_RANK are used.
Clip batches are sharded (weak scaling, B clips per rank); the noise is a
counter-based Philox stream keyed by (seed, global sample index, round, step),
so a clip's result does not depend on the shard it lands on.

`--dist-backend gloo` runs the same rank path over gloo (collectives staged through
host memory; ranks share the GPUs round-robin) to rehearse N > 1 on one GPU.

Other BASELINE workloads: `--config {kth,cityscapes,ucf,smmnist}` (WORKLOADS below:
each dataset's tc / tp / rounds / sampler, its wrapper and denoiser variant, a per-GPU
batch), one bench line each; BAIR stays the default the driver runs.

Output: rank 0 prints (and flushes) a JSON line as soon as the timed region and
the roofline launch timing are done, marked "partial": true, then the complete
line with `cpu_baseline` once the CPU port has been timed. The last line is the
result.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--config NAME]
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
PKG = '140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd'
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense fp32 matrix peak
# f16x3: three v_mfma_f32_32x32x16_f16 per fp32 product; fp16 dense MFMA peak 2516.6 TF/s
# (32x32x16 = 32768 FLOP per 32 cycles per SIMD, 1024 SIMDs, 2.4 GHz) / 3
F16X3_PEAK_TFLOPS = 2516.6 / 3
BF16_PEAK_TFLOPS = 2516.6  # dense bf16 MFMA (v_mfma_f32_32x32x16_bf16), same rate as fp16
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak
PEAKS = {'fp32': FP32_MFMA_PEAK_TFLOPS, 'f16x3': F16X3_PEAK_TFLOPS, 'bf16': BF16_PEAK_TFLOPS}
# kernel families by the arithmetic their MFMAs run (template arguments decide where listed in
# kernel_arith): fp32 MFMA kernels, and the f16x3 ones
FP32_FAMILIES = ('attn_fused_kernel', 'window_attn_kernel', 'cross_attn_kernel', 'conv_kernel', 'conv_halo_kernel',
                 'conv_gemm_kernel')
X3_FAMILIES = ('conv_x3_kernel', 'conv_gemm_x3_kernel', 'xpath_x3_kernel', 'noise_pool_x3_kernel',
               'cross_attn_x3_kernel', 'cross_attn_x3p_kernel', 'fea_side_x3_kernel', 'pw_x3_kernel')


def _template(kname):
    """('ident', [template args]) of 'ident<a, b, ...>' (args [] without a template list)."""
    base = kname.split(' (')[0].strip()
    if '<' not in base:
        return base, []
    ident, rest = base.split('<', 1)
    return ident.strip(), [a.strip() for a in rest.rsplit('>', 1)[0].split(',')]


def kernel_arith(kname, precision):
    """The arithmetic of a launched kernel, from its template: 'fp32' (fp32 MFMA), 'f16x3' (three
    fp16 MFMAs per fp32 product), 'bf16', or 'f16x3+bf16' (the fused attention kernels in
    BF16_ATTN: qkv / proj on f16x3, QK^T / PV on bf16).
      attn_core_kernel<MODE, X3, NT, DH>     X3 true: f16x3, false: bf16
      attn_x3_kernel<C, MODE, DH, NW, TILE, BF>, stw64_x3_kernel<C, DH, NW, BF, TILE>
                                             BF false: f16x3, true: f16x3+bf16
    Other families by name (FP32_FAMILIES / X3_FAMILIES); unknown names by the handle's precision."""
    ident, args = _template(kname)
    if ident == 'attn_core_kernel' and len(args) in (3, 4):
        return 'f16x3' if args[1] == 'true' else 'bf16'
    if ident == 'attn_x3_kernel' and len(args) == 6:
        return 'f16x3+bf16' if args[5] == 'true' else 'f16x3'
    if ident == 'stw64_x3_kernel' and len(args) in (4, 5):
        return 'f16x3+bf16' if args[3] == 'true' else 'f16x3'
    if ident in FP32_FAMILIES:
        return 'fp32'
    if ident in X3_FAMILIES:
        return 'f16x3'
    return 'fp32' if precision == 'fp32' else 'f16x3'


def kernel_peak(arith, core_frac=0.0):
    """Dense MFMA peak (TFLOP/s) for that arithmetic. 'f16x3+bf16': the FLOP-weighted harmonic
    mean of the f16x3 and bf16 peaks (the time the work takes at peak), core_frac = the share of
    the FLOPs in the bf16 QK^T / PV contractions."""
    if arith == 'f16x3+bf16':
        return 1.0 / ((1.0 - core_frac) / F16X3_PEAK_TFLOPS + core_frac / BF16_PEAK_TFLOPS)
    return PEAKS[arith]


# BASELINE.json configs as bench workloads (tc / tp per round, rounds =
# ceil(total_pred / tp); the sampler of the dataset's eval script). `batch` = clips per GPU:
# the BASELINE batch split over its GPU count where it names one (KTH: 64 on 4 GPUs), else the
# batch past which the per-clip step cost stops falling (round 6, profiles/r06_batch_cfg.txt: ms per
# clip-step Cityscapes 1.10 / 0.45 / 0.38 at 8 / 32 / 64, UCF 9.70 / 8.93 at 4 / 8, SMMNIST 0.519 /
# 0.495 at 64 / 128). The BAIR line is the metric (configs[1]).
WORKLOADS = {
    # BAIR: 128 clips per GPU (round 5 sweep, DDIM-20 generations on one box: 0.413 / 0.396 / 0.391 /
    # 0.397 ms per clip-step at B = 64 / 128 / 192 / 256 — the small levels' launches fill the chip
    # better; 128 keeps one DDPM-1000 generation near 100 s)
    'bair': dict(image=64, tc=2, tp=14, total_pred=28, sampling_steps=1000, timesteps=1000, batch=128, occ=False,
                 precision=None, baseline='configs[1]: BAIR 64x64 ch3, cond=2 pred=14, DDPM 1000 steps, 1xMI355X'),
    'kth': dict(image=64, tc=10, tp=20, total_pred=40, sampling_steps=100, timesteps=1000, batch=16, occ=False,
                precision=None, cpu_steady=2, baseline='configs[2]: KTH 64x64 ch1, cond=10 pred=40, DDIM 100 steps, batch=64 on 4 GPUs',
                lead=(6, 'level-0 shifted STW attention (ada 4x4x4 windows, dim_head 16), fused LN/qkv/RoPE/softmax/PV/proj')),
    'cityscapes': dict(image=128, tc=2, tp=5, total_pred=28, sampling_steps=1000, timesteps=1000, batch=128, occ=True,
                       precision=None, cpu_steady=2, baseline='configs[3]: Cityscapes 128x128 ch3, cond=2 pred=28, DDPM 1000 steps',
                       lead=(6, 'level-0 shifted STW attention (ada_u22 4x4x4 windows, dim_head 32), fused LN/qkv/RoPE/softmax/PV/proj')),
    'ucf': dict(image=256, tc=4, tp=12, total_pred=12, sampling_steps=10, timesteps=1000, batch=8, occ=True,
                precision='bf16_attn', cpu_steady=1, cpu_steps_max=1, baseline='configs[4]: UCF-101 256x256 ch3, cond=4 pred=12, bf16 MFMA attention',
                lead=(6, 'level-0 shifted STW attention (ada_u22 4x4x4 windows), fused, bf16 QK^T / PV')),
    'smmnist': dict(image=64, tc=10, tp=10, total_pred=10, sampling_steps=100, timesteps=100, batch=128, occ=True,
                    precision=None, baseline='configs[0]: SMMNIST 64x64 ch1, cond=10 pred=10, DDPM 100 steps',
                    lead=(6, 'level-0 shifted STW attention (C 64, 2x4x4 windows), fused LN/qkv/proj')),
}
# `lead`: the bench_layer id of the workload's kernel with the largest share of GPU time in its own
# DDIM-20 profile (profiles/r0N_cfgprof_<config>_kernel_stats.csv); it heads that config's roofline.
# The launched template is read back from the library (extdm_bench_layer_kernel). BAIR's is LAYERS[0].


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--config', default='bair', choices=sorted(WORKLOADS),
                    help='BASELINE workload (bair = configs[1], the metric; the others: bench lines of their own)')
    ap.add_argument('--dist-backend', default='nccl', choices=['nccl', 'gloo'],
                    help='torch.distributed backend for N > 1 (gloo: test the rank path on one GPU)')
    ap.add_argument('--steps', type=int, default=None,
                    help='reverse-diffusion steps to time, rounded up to whole generations (default: one)')
    ap.add_argument('--warmup', type=int, default=5, help='untimed graph replays')
    ap.add_argument('--batch', type=int, default=None, help='clips per GPU (default: the workload\'s)')
    ap.add_argument('--sampling-steps', type=int, default=None,
                    help='default: the workload\'s sampler (BAIR: DDPM-1000, the metric); fewer = DDIM-S sweeps')
    ap.add_argument('--total-pred', type=int, default=None)
    ap.add_argument('--tp', type=int, default=None)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-steps', type=int, default=5, help='timed oracle steps per CPU batch point')
    ap.add_argument('--precision', default=None, choices=['fp32', 'f16x3', 'bf16_attn'],
                    help='conv / attention arithmetic (include/extdm.h EXTDM_PRECISION_*); default: package default')
    ap.add_argument('--no-roofline', action='store_true', help='test-only: skip the per-kernel roofline timing')
    ap.add_argument('--dump', default=None, help='test-only: save the gathered videos of the last generation here')
    ap.add_argument('--stub', action='store_true',
                    help='test-only: CPU/gloo stand-in workload that exercises the launcher and rank plumbing')
    a = ap.parse_args(argv)
    w = WORKLOADS[a.config]
    for k in ('batch', 'sampling_steps', 'total_pred', 'tp'):
        if getattr(a, k) is None:
            setattr(a, k, w[k])
    return a


# ------------------------------------------------------------------ launcher
def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv):
    """One child process per GPU (RANK = LOCAL_RANK = i, WORLD_SIZE = n) started
    before this process touches the GPU. A failing rank stops the others (their
    exact PIDs); returns the first non-zero exit status, else 0."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    return rc


# ------------------------------------------------------------------ workloads
def synthetic_clips(B, tc, S, seed):
    """Conditioning clips U[0,1) from NumPy PCG64."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(rng.random((B, 3, tc, S, S), dtype=np.float32))


CONFIG_NAMES = {'bair': 'BAIR 64x64 ch3', 'kth': 'KTH 64x64 ch1 (as 3 ch)', 'cityscapes': 'Cityscapes 128x128 ch3',
                'ucf': 'UCF-101 256x256 ch3', 'smmnist': 'SMMNIST 64x64 ch1 (as 3 ch)'}


def layer_what(layer, u, shapes):
    return _layer_what(layer, u, shapes) or None


def _layer_what(layer, u, shapes):
    """What bench layer `layer` (runtime.cpp extdm_bench_layer) runs for denoiser config `u`
    (spec.UnetConfig), with the operand shapes read from the denoiser's state_dict (`shapes`:
    name -> shape); None where the layer does not exist in this denoiser."""
    T, L, fs, d0 = u.frames, u.latent, u.fea_size, u.dim
    win = 'x'.join(str(min(w, e)) for w, e in zip(u.window, (T, L, L)))
    heads = f'{u.heads} heads x {u.dim_head}'

    def sh(name):
        return shapes.get(name)
    if layer == 0:
        if u.short == 'u12':
            return (f'init_conv cond_fea branch, phase-composed: 2 row parities x 2 column phases, 1x5x5 over the '
                    f'{fs}x{fs} map, {u.fea_ch} -> {d0} ch, {u.tp} frames')
        w = sh('init_conv.weight')
        return w and f'init_conv {w[1]} -> {w[0]} ch 1x7x7 over {T} frames of {L}x{L} px'
    if layer == 11:
        return (f'init_conv cond_fea branch edge corrections (2 line launches K = 5 x {u.fea_ch} + corners)'
                if u.short == 'u12' else None)
    if layer in (1, 5):
        w = sh('downs.0.0.block2.proj.weight')
        how = 'fp32 input staged' if layer == 1 else 'pre-split operand by LDS-DMA'
        blk = 'block1-shape' if layer == 1 else 'block2'
        return w and f'level-0 ResnetBlock {blk} conv {w[1]}->{w[0]} 1x3x3 at {L}x{L} px, {T} frames, {how}'
    if layer == 6:
        return (f'level-0 shifted-window attention (STW, C {d0}, {win} windows, {heads}), fused '
                f'LN/qkv/RoPE/softmax/PV/proj')
    if layer == 7:
        return f'init_temporal_attn (C {d0}, {T} frames, {heads})'
    if layer == 8:
        return (f'TrajWarp cross-attention core ({u.tp * fs * fs} queries x {u.tc * fs * fs} keys, 8 heads)'
                if u.short == 'u12' else None)
    if layer == 4:
        w = sh('ups.3.0.res_conv.weight')
        return w and f'level-0 res_conv {w[1]}->{w[0]} 1x1x1 at {L}x{L} px, {T} frames'
    if layer == 9:
        return f'init_conv x-branch as one composed 13x13 conv 3->{d0}, K = 3x169' if u.short in ('u12', 'ada') else None
    if layer == 10:
        w = sh('init_noise_conv.weight')
        return w and u.short == 'u12' and f'init_noise_conv 3->{w[0]} 1x7x7 + MaxPool(1,2,2), K = 3x49'
    if layer == 12:
        w = sh('init_traj.cross_att.linear_q.weight')
        return w and f'TrajWarp linear_q {w[1]}->{w[0]} 1x1 + ReLU over {u.tp} x {fs}x{fs} px, weights register-resident (pw_x3)'
    if layer == 13:
        w = sh('downs.2.4.Tmodulator.weight')
        return w and (f'level-2 MotionAdaptor Tmodulator, 1x1 over (T C) = {w[1]} -> {w[0]} channels of '
                      f'{L // 4}x{L // 4} px')
    if layer in (14, 16):
        return f"{'the level-0 STW layer' if layer == 14 else 'init_temporal_attn'}'s qkv 1x1 conv"
    if layer in (15, 17):
        return f"{'the level-0 STW layer' if layer == 15 else 'init_temporal_attn'}'s proj 1x1 conv + residual"
    return None


def metric_label(config, meta_metric, sampler, name, tc, total_pred, baseline):
    """BASELINE.json's metric for the BAIR line; the other workloads' lines name their own."""
    if config == 'bair':
        return meta_metric
    return (f'predicted frames/sec/GPU ({sampler}) {name} {tc}->{total_pred} — bench line of {baseline}, '
            f'not the headline metric')


class NativeWorkload:
    """The product path: FlowDiffusion + autoregressive_sample on the HIP library, for one of
    the BASELINE workloads (WORKLOADS[args.config])."""

    def __init__(self, args, dev, world, rank):
        import importlib
        pkg = importlib.import_module(PKG)
        self.pkg, self.args, self.dev, self.world, self.rank = pkg, args, dev, world, rank
        self.w = w = WORKLOADS[args.config]
        B = args.batch
        wrapper, unet_arch = pkg.configs.dm_arch(args.config)
        cfg = pkg.configs.dm_config(args.config, pred_frames=args.tp, sampling_timesteps=args.sampling_steps,
                                    estimate_occlusion_map=w['occ'])
        cfg['dataset_params']['frame_shape'] = w['image']  # UCF-101 at 256 (BASELINE configs[4]; the YAML says 64)
        fd = pkg.FlowDiffusion(config=cfg, is_train=False, Unet3D_architecture=unet_arch, wrapper=wrapper,
                               timesteps=w['timesteps']).to(dev)
        fd.diffusion.max_batch = B
        self.precision = args.precision or w['precision'] or pkg._lib.DEFAULT_PRECISION
        fd.unet.precision = self.precision
        self.fd = fd
        self.tc, self.tp = fd.cond_frame_num, fd.pred_frame_num
        self.rounds = -(-args.total_pred // self.tp)
        self.steps_per_generation = self.rounds * args.sampling_steps
        self.frames_per_generation = world * B * args.total_pred
        self.start, _ = pkg.dist.shard(world * B, world, rank)  # weak scaling: B clips per rank
        # the global batch from one seed, sliced per rank: a clip's input (and, with the noise
        # keyed by global sample index, its output) does not depend on the rank count
        self.clips = synthetic_clips(world * B, self.tc, w['image'], 1234)[self.start:self.start + B].to(dev)
        self.h = None

    def prime(self, warmup):
        """Untimed: build every native handle (weights packed, workspace planned),
        capture the step graph and replay it `warmup` times, run encoder + decoder."""
        fd, B, pkg = self.fd, self.args.batch, self.pkg
        ret, x_cond, fea, ref = fd.encode(self.clips)
        self.h = h = fd.diffusion._native(B, self.dev, fea.shape[-1])
        prime = torch.empty(B, 3, self.tp, x_cond.shape[3], x_cond.shape[4], device=self.dev)
        n = max(1, min(warmup, fd.diffusion.num_timesteps))
        T = fd.diffusion.num_timesteps
        h.sample(pkg._lib.SAMPLER_DDPM, list(range(T - 1, T - 1 - n, -1)), None, 0., x_cond, fea, prime, seed=1,
                 sample_base=self.start)
        fd.decode(ret, prime, ref)
        torch.cuda.synchronize()

    def generation(self, idx):
        out = self.pkg.autoregressive_sample(self.fd, self.clips, self.args.total_pred, num_sample_video=1,
                                             seed=1234 + idx, sample_base=self.start)
        return self.pkg.dist.gather_shards(out.contiguous(), self.world * self.args.batch, self.world)

    def sync(self):
        torch.cuda.synchronize()

    def check(self, out):
        assert out.shape[0] == self.world * self.args.batch and torch.isfinite(out).all()

    def describe(self):
        a, B, w = self.args, self.args.batch, self.w
        T = self.fd.diffusion.num_timesteps
        sampler = f'DDPM {T}' if a.sampling_steps >= T else f'DDIM {a.sampling_steps} (of {T})'
        names = CONFIG_NAMES
        unet = self.fd.unet.__class__.__name__
        return {
            'dtype': {'fp32': 'fp32', 'f16x3': 'fp32 (f16x3 split-MFMA convs + attention, fp32 accumulate)',
                      'bf16_attn': 'fp32 convs as f16x3; attention QK^T / PV in bf16 MFMA (fp32 accumulate)'}[
                          self.precision],
            'data': 'synthetic (U[0,1) PCG64 clips, seeded random-init weights; no dataset/checkpoint offline)',
            'config': {'workload': f'{names[a.config]} {self.tc}->{a.total_pred} (tp={self.tp} x {self.rounds} rounds), '
                                   f'{sampler} steps, {unet} ({self.fd.wrapper} wrapper), LFAE encoder + flow-warp '
                                   f'decoder, occlusion map {"on" if w["occ"] else "off (eval default)"}',
                       'baseline_config': w['baseline'], 'bench_config': a.config,
                       'global_batch': self.world * B, 'batch_per_gpu': B, 'sampling_steps': a.sampling_steps,
                       'rounds': self.rounds, 'parallelism': f'clip-shard x{self.world} (+gather to rank 0)',
                       'workspace_gb': round(self.h.workspace_bytes() / 2 ** 30, 2)}}

    # extdm_bench_layer ids (runtime.cpp) of the kernels reported for BAIR, dominant first: the
    # kernel with the largest share of a step's GPU time (the phase-composed cond_fea conv), its edge
    # corrections, the level-0 ResnetBlock 3x3 convs (block1 stages an fp32 input, block2 (5) copies
    # block1's pre-split operand), the level-0 attention launches: shifted-window attention (6), the
    # temporal attention (7) and TrajWarp's cross-attention core (8), the level-0 1x1 res_conv
    # (HBM-bound: 3 FLOP-equivalents of f16x3 MFMA per 4-B element moved is far below the machine
    # balance), the x-branch's low-K gathers (9, 10), TrajWarp's linear (12) and the level-2
    # Tmodulator (13). `kernel`: the launched template (None: read back from the library,
    # extdm_bench_layer_kernel — the attention layers' route and the conv tiles' template arguments
    # are chosen per launch); the PMC traffic of profiles/pmc_layer<id>.json counts only
    # when it names this template and was measured on this exact library build (lib_sha16).
    LAYERS = [(0, 'mfma', None,
               'init_conv cond_fea branch, phase-composed: 2 row parities x 2 column phases x 64 rows, 1x5x5 over the 16x16 map, 256 ch'),
              (11, 'mfma', 'fea_side_x3_kernel',
               'init_conv cond_fea branch edge corrections (2 line launches K = 5 x 256, 512 rows + corners)'),
              (1, 'mfma', None,
               'level-0 ResnetBlock block1 conv 64->64 1x3x3, fp32 input staged'),
              (6, 'mfma', None,
               'level-0 shifted-window attention (STW, C 64, 2x4x4 windows, 8 heads x 32), fused LN/qkv/proj'),
              (5, 'mfma', None,
               'level-0 ResnetBlock block2 conv 64->64 1x3x3, pre-split operand by LDS-DMA'),
              (7, 'mfma', None, 'init_temporal_attn (C 64, 16 frames, 8 heads x 32)'),
              (8, 'mfma', 'cross_attn_x3p_kernel<1>', 'TrajWarp cross-attention core (3584 queries x 512 keys, 8 heads)'),
              (4, 'hbm', None,
               'level-0 res_conv 128->64 1x1x1'),
              (9, 'mfma', 'xpath_x3_kernel', 'init_conv x-branch as one composed 13x13 conv 3->64, K = 3x169'),
              (10, 'mfma', 'noise_pool_x3_kernel', 'init_noise_conv 3->256 1x7x7 + MaxPool(1,2,2), K = 3x49'),
              (12, 'hbm', 'pw_x3_kernel',
               'TrajWarp linear_q 256->256 1x1 + ReLU, weights register-resident (pw_x3)'),
              (13, 'mfma', None,
               'level-2 MotionAdaptor Tmodulator, 1x1 over (T C) = 3584 -> 3584 channels of 8x8 px')]
    # the unfused core route's other launches, reported beside layer 6 / 7 when that route is taken
    CORE_SPLIT = {6: [(14, 'the level-0 STW layer\'s qkv 1x1 conv'), (15, 'its proj 1x1 conv + residual')],
                  7: [(16, 'init_temporal_attn\'s qkv 1x1 conv'), (17, 'its to_out 1x1 conv + residual')]}
    # Layers whose HBM reads are whole-line coalesced streams (every wave instruction reads >= 256
    # contiguous bytes: buffer loads of 64 consecutive pixels, 1-KB LDS-DMA pieces): their PMC
    # FETCH_SIZE gets the gfx950 x2 correction (MI355X_MICROARCH.md HBM), calibrated on pw_x3 (layer
    # 12), which reads each of its 234.9 MB of input exactly once: raw FETCH 118.8 MB (0.506x). Not
    # doubled (reported raw, uncalibrated): the x-branch gathers (9, 10: overlapping per-lane 32-B
    # windows), the temporal attention (7: 16-B pieces four pixels wide, one frame apart) and the
    # per-lane attention kernels (stw64_x3, attn_x3 without its tile path: 4-B loads per lane).
    WIDE_READS = {0, 1, 4, 5, 8, 11, 12, 13}
    # HBM-bound entries: (input + output channels, spatial size per frame, frames) of the algorithmic bytes
    HBM_BYTES = {4: lambda u, T, sh: (sum(sh['ups.3.0.res_conv.weight'][:2]), u.latent ** 2, T),
                 12: lambda u, T, sh: (sum(sh['init_traj.cross_att.linear_q.weight'][:2]), u.fea_size ** 2, u.tp)}

    @staticmethod
    def wide_reads(layer, kname):
        if layer == 6:  # the STW tile path stages x by 1-KB LDS-DMA pieces
            ident, args = _template(kname)
            return ident == 'attn_x3_kernel' and len(args) == 6 and args[4] == 'true'
        return layer in NativeWorkload.WIDE_READS

    def pmc_path(self, layer):
        """profiles/pmc_layer<id>.json (BAIR) or profiles/pmc_<config>_layer<id>.json."""
        c = self.args.config
        return os.path.join(REPO, 'profiles', f'pmc_layer{layer}.json' if c == 'bair' else f'pmc_{c}_layer{layer}.json')

    def _traffic(self, layer, kname):
        """HBM bytes per launch from the committed PMC passes (scripts_gpu/pmc_layers.sh), only
        when they were taken on this library build, config batch and precision and name the
        launched template."""
        pmc = self.pmc_path(layer)
        try:
            j = json.load(open(pmc))
        except (ValueError, OSError):
            return None, 'no PMC file'
        if int(j.get('batch', -1)) != self.args.batch or j.get('precision') != self.precision:
            return None, 'PMC batch / precision differ'
        if j.get('lib_sha16') != lib_sha16():
            return None, 'PMC taken on another library build (stale)'
        if not kname or kname not in j.get('kernel_name', ''):
            return None, 'PMC kernel signature differs'
        if 'fetch_rule' not in j:
            return None, 'PMC file predates the raw / corrected FETCH split'
        src = (f"profiles/{os.path.basename(pmc)}: FETCH {j['fetch_bytes_raw_per_launch']} B raw, "
               f"{j['fetch_rule']}; WRITE {j['write_bytes_per_launch']} B")
        return j.get('hbm_bytes_per_launch'), src

    def attn_core_frac(self, layer):
        """Share of an attention layer's FLOPs in QK^T / PV: per token 4 N hid of 2 C 3 hid + 4 N hid
        + 2 hid C (N = window tokens at level 0, or frames) = 4 N / (8 C + 4 N)."""
        u = self.fd.unet.ucfg
        T = u.frames
        C = u.dim
        if layer in (6, 14, 15):
            ws = list(u.window)
            ext = [T, u.latent, u.latent]
            N = 1
            for w, e in zip(ws, ext):
                N *= min(w, e)
        else:
            N = T
        return 4.0 * N / (8.0 * C + 4.0 * N)

    def layer_ids(self):
        """(id, bound, static template or None, what) in report order: this workload's lead first;
        `what` from this denoiser's own config and weight shapes (layer_what), layers it lacks left out."""
        layers = list(self.LAYERS)
        lead = self.w.get('lead')
        if lead:
            i = next(k for k, e in enumerate(layers) if e[0] == lead[0])
            layers = [(lead[0], layers[i][1], None, lead[1])] + layers[:i] + layers[i + 1:]
        shapes = {k: tuple(v.shape) for k, v in self.fd.unet.state_dict().items()}
        out = []
        for lid, bound, kname, _ in layers:
            what = layer_what(lid, self.fd.unet.ucfg, shapes)
            if what:
                out.append((lid, bound, kname, what))
        return out

    def roofline(self):
        """Per kernel, timed over 20 launches of the exact forward launch with HIP events on the
        handle's stream (extdm_bench_layer). MFMA-bound: FLOP per launch / time against the dense
        MFMA peak of the arithmetic that kernel runs (kernel_arith: its template; f16x3 = dense fp16
        / 3, bf16 = dense bf16, fp32 = dense fp32, f16x3+bf16 the FLOP-weighted mix). HBM-bound:
        algorithmic bytes per launch (fp32 input + output elements, 4 B each, weights aside) / time
        against 8 TB/s. The first entry is the dominant kernel; the others ride along."""
        B = self.args.batch
        u = self.fd.unet.ucfg
        T = u.frames
        out = []
        todo = list(self.layer_ids())
        while todo:
            layer, bound, kname, what = todo.pop(0)
            if layer == 5 and self.precision == 'fp32':
                continue
            try:
                ms_layer, flops = self.h.bench_layer(B, layer, 20)
            except RuntimeError:  # the layer does not exist in this denoiser variant / precision / route
                continue
            launched = self.h.bench_layer_kernel(layer)
            if launched:
                kname = launched
            if kname is None:
                kname = ''
            if layer in self.CORE_SPLIT and launched.startswith('attn_core_kernel'):
                # the unfused route: this entry is the core launch alone; its convs follow
                what = what + ' — unfused route: the attention core launch alone'
                shapes = {k: tuple(v.shape) for k, v in self.fd.unet.state_dict().items()}
                todo[0:0] = [(i, 'mfma', None, layer_what(i, u, shapes)) for i, _ in self.CORE_SPLIT[layer]]
            arith = kernel_arith(kname, self.precision) if kname else ('fp32' if self.precision == 'fp32' else 'f16x3')
            traffic, src = self._traffic(layer, kname)
            if bound == 'mfma':
                frac_core = self.attn_core_frac(layer) if arith == 'f16x3+bf16' else 0.0
                kpeak = kernel_peak(arith, frac_core)
                achieved = flops / (ms_layer * 1e-3) / 1e12
                e = {'bound': 'mfma', 'achieved': round(achieved, 2), 'peak': round(kpeak, 1), 'unit': 'TFLOP/s',
                     'frac': round(achieved / kpeak, 4), 'flop_per_launch': flops, 'arith': arith}
                if frac_core:
                    e['peak_note'] = (f'f16x3 qkv/proj + bf16 QK^T/PV: {frac_core:.3f} of the FLOPs at {BF16_PEAK_TFLOPS}, '
                                      f'the rest at {F16X3_PEAK_TFLOPS:.1f} TFLOP/s (FLOP-weighted harmonic peak)')
            else:
                shapes = {k: tuple(v.shape) for k, v in self.fd.unet.state_dict().items()}
                ch, hw, nt = self.HBM_BYTES[layer](u, T, shapes)
                nbytes = 4 * B * nt * hw * ch
                achieved = nbytes / (ms_layer * 1e-3) / 1e9
                e = {'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(achieved / HBM_PEAK_GBS, 4), 'bytes_per_launch': nbytes, 'arith': arith}
            e.update({'kernel': f"{kname or '(1x1 conv)'} ({what}, {arith})", 'layer': layer, 'traffic': traffic,
                      'traffic_src': src, 'launch_ms': round(ms_layer, 4)})
            out.append(e)
        if not out:
            return None
        res = out[0]
        res['others'] = out[1:]
        return res

    def cpu_baseline(self):
        return cpu_baseline(self.fd, self.rounds, self.args.sampling_steps,
                            min(self.args.cpu_steps, self.w.get('cpu_steps_max', self.args.cpu_steps)), self.w,
                            steady_batch=self.w.get('cpu_steady', 4))


def lib_sha16():
    """First 16 hex digits of sha256 of the loaded HIP library (EXTDM_LIB or the in-tree one)."""
    import hashlib
    path = os.environ.get('EXTDM_LIB') or os.path.join(REPO, PKG, 'libextdm_hip.so')
    try:
        return hashlib.sha256(open(path, 'rb').read()).hexdigest()[:16]
    except OSError:
        return None


class StubWorkload:
    """CPU stand-in for tests (tests/test_bench_launcher.py): same rank plumbing
    (shard, gloo all-gather, max-over-ranks), a result that depends only on the
    global sample index, no GPU."""

    def __init__(self, args, dev, world, rank):
        import importlib
        self.D = importlib.import_module(PKG + '.dist')
        self.args, self.world, self.rank = args, world, rank
        self.start, self.count = self.D.shard(world * args.batch, world, rank)
        self.steps_per_generation = 4
        self.frames_per_generation = world * args.batch * args.total_pred
        self.precision = 'fp32'

    def prime(self, warmup):
        pass

    def generation(self, idx):
        ids = torch.arange(self.start, self.start + self.count, dtype=torch.float32)
        out = ids.view(-1, 1, 1).expand(-1, 3, 2).contiguous()
        time.sleep(0.05)
        return self.D.gather_shards(out, self.world * self.args.batch, self.world)

    def sync(self):
        pass

    def check(self, out):
        n = self.world * self.args.batch
        assert torch.equal(out[:, 0, 0], torch.arange(n, dtype=torch.float32))

    def describe(self):
        return {'dtype': 'fp32', 'data': 'stub', 'config': {'workload': 'stub', 'global_batch': self.world *
                                                             self.args.batch, 'batch_per_gpu': self.args.batch,
                                                             'parallelism': f'clip-shard x{self.world}'}}

    def roofline(self):
        return None

    def cpu_baseline(self):
        return None


def cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def cgroup_cpus():
    """CPUs' worth of time the cgroup grants this process (cpu.max quota / period; cgroup v1
    cfs quota), or None when unlimited / unknown."""
    try:
        q, p = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            return max(1, math.ceil(int(q) / int(p)))
        return None
    except (OSError, ValueError):
        pass
    try:
        q = int(open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us').read())
        p = int(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read())
        return max(1, math.ceil(q / p)) if q > 0 else None
    except (OSError, ValueError):
        return None


def cpu_threads():
    """Host cores this process may run on (sched affinity, capped by the cgroup CPU quota: on
    the GPU box 256 cores are visible but the container is granted a 16-CPU share, and 256
    threads on it took 87 s for the oracle's encoder round), and the OMP_NUM_THREADS slice
    where one is set. Returns (visible cores, usable cores, slice)."""
    visible = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else (os.cpu_count() or 1)
    quota = cgroup_cpus()
    usable = min(visible, quota) if quota else visible
    env = os.environ.get('OMP_NUM_THREADS')
    threads = min(usable, int(env)) if env and env.isdigit() and int(env) > 0 else usable
    return visible, usable, threads


def cpu_baseline(fd, rounds, steps_per_round, n_steps, w, steady_batch=4):
    """The oracle (PyTorch-CPU restatement of the reference, kind "port") timed on this
    box's host cores (torch.set_num_threads(<all host cores>))
    at B = 1 and at a steady batch: one round's LFAE encoder and decode (B = 1, scaled by B),
    n_steps reverse steps (Unet forward + the DDPM / DDIM update; median, with the spread)
    per batch point, extrapolated to the workload's rounds x steps. `value` = the better
    all-cores batch point; where OMP_NUM_THREADS sets a smaller slice, B = 1 is also timed on
    that slice (reported beside it, not the value). Oracle use is confined to this untimed leg."""
    from oracle import extdm_oracle as O
    from oracle import lfae_oracle as LO
    visible, cores, slice_threads = cpu_threads()
    threads = cores
    torch.set_num_threads(threads)
    ucfg = fd.unet.ucfg
    lc = fd.lcfg
    sd = {f'generator.{k}': v.detach().cpu() for k, v in fd.generator.state_dict().items()}
    sd.update({f'region_predictor.{k}': v.detach().cpu() for k, v in fd.region_predictor.state_dict().items()})
    sd.update({f'bg_predictor.{k}': v.detach().cpu() for k, v in fd.bg_predictor.state_dict().items()})
    usd = {k: v.detach().cpu() for k, v in fd.unet.state_dict().items()}
    T_sched = fd.diffusion.num_timesteps
    sch = O.schedule(T_sched)
    ddim = steps_per_round < T_sched
    vid = synthetic_clips(1, ucfg.tc, lc.image, 99)
    with torch.no_grad():
        t0 = time.perf_counter()
        ret, x_cond, fea, ref = LO.encode_round(sd, lc, ucfg, vid)
        t_enc = time.perf_counter() - t0
        print(f'cpu baseline: encoder round {t_enc:.2f} s', file=sys.stderr, flush=True)
        if fd.wrapper == 'multi1248':  # cond_fea at flow size, tc - 1 + tp frames (multi1248.py:240-245)
            fea = torch.randn(1, fea.shape[1], ucfg.tc - 1 + ucfg.tp, ucfg.latent, ucfg.latent)
        x = torch.randn(1, 3, ucfg.tp, ucfg.latent, ucfg.latent)
        t0 = time.perf_counter()
        LO.decode_round(sd, lc, ucfg, ret, x, ref)
        t_dec = time.perf_counter() - t0
        pairs = O.ddim_pairs(T_sched, steps_per_round) if ddim else None
        # a warm step + n_steps timed ones, all inside the sampler's step list
        n_steps = max(1, min(n_steps, (len(pairs) if ddim else T_sched) - 1))
        # B = 1, 2 and the steady batch: on the GPU box's host the oracle's per-clip cost is lowest at
        # B = 2 and rises past it (B = 4: 3x the CPU-seconds of B = 2 for 2x the work, no cgroup
        # throttling — a cache effect, profiles/r06_cpu_scaling.log); every point is reported and
        # the value is the best of them
        bs = sorted({1, min(2, steady_batch), steady_batch}) if steady_batch > 1 else [1]
        runs = [(threads, B) for B in bs]
        if slice_threads < threads:
            runs.append((slice_threads, 1))
        points = []
        for nth, B in runs:
            torch.set_num_threads(nth)
            xc, fb, xb = x_cond.expand(B, *x_cond.shape[1:]), fea.expand(B, *fea.shape[1:]), x.expand(B, *x.shape[1:])

            def step(k, xb):
                ti = pairs[k][0] if ddim else T_sched - 1 - k
                t = torch.full((B,), ti, dtype=torch.long)
                eps = O.unet_forward(usd, ucfg.as_dict(), xb, t, xc, fb)
                if ddim:
                    return O.ddim_step(sch, xb, eps, pairs[k][0], pairs[k][1], torch.randn_like(xb))
                return O.ddpm_step(sch, xb, eps, t, torch.randn_like(xb))
            xb = step(0, xb)  # warm
            per = []
            for k in range(n_steps):
                t0 = time.perf_counter()
                xb = step(k + 1, xb)
                per.append(time.perf_counter() - t0)
                # progress on stderr (stdout carries the one JSON line)
                print(f'cpu baseline: {nth} threads, B={B}: step {k + 1}/{n_steps} {per[-1]:.2f} s', file=sys.stderr,
                      flush=True)
            t_step = float(np.median(per))
            total = rounds * B * (t_enc + t_dec) + rounds * steps_per_round * t_step
            points.append({'threads': nth, 'batch': B, 'frames_per_s': round(rounds * ucfg.tp * B / total, 5),
                           's_per_step': round(t_step, 4), 's_per_step_min_max': [round(min(per), 4), round(max(per), 4)]})
        torch.set_num_threads(threads)
    best = max((p for p in points if p['threads'] == threads), key=lambda p: p['frames_per_s'])
    return {'value': best['frames_per_s'], 'unit': 'frames/s', 'cores': cores, 'threads': threads,
            'kind': 'port', 'cpu_model': cpu_model(), 'batch_points': points,
            'visible_cores': visible, 'cgroup_cpus': cgroup_cpus(),
            'baseline_method': 'r06: every host core the process may use (sched affinity capped by the cgroup '
                               'CPU quota) at B = 1, 2 and the steady batch, value = the best per-clip point (the '
                               'oracle\'s per-clip cost is lowest at B = 2 on this host and rises past it: a cache '
                               'effect, not cgroup throttling, profiles/r06_cpu_scaling.log) + the OMP_NUM_THREADS '
                               f'slice at B=1 where smaller; median of {n_steps} timed steps per point',
            'sample': f'oracle (PyTorch-CPU fp32) on {threads} threads = every usable host core ({visible} '
                      f'visible, cgroup quota {cgroup_cpus()}): encoder round '
                      f'({t_enc:.3f} s) and decode round ({t_dec:.3f} s) at B=1, {n_steps} '
                      f'{"DDIM" if ddim else "DDPM"} steps per batch point (B = '
                      f'{", ".join(str(p["batch"]) for p in points if p["threads"] == threads)}'
                      + (f'; B=1 also on the {slice_threads}-thread OMP_NUM_THREADS slice' if slice_threads < threads else '')
                      + f'); extrapolated to {rounds} rounds x {steps_per_round} steps; value = the better '
                      f'all-cores batch point (B={best["batch"]})'}


# ------------------------------------------------------------------ rank body
def run_rank(args):
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    import torch.distributed as dist
    if args.stub:
        dev = torch.device('cpu')
        if world > 1:
            dist.init_process_group('gloo')
        wl = StubWorkload(args, dev, world, rank)
    else:
        # one GPU per rank; with fewer GPUs than ranks (the gloo rehearsal on a 1-GPU box) the
        # ranks share them round-robin (device_count does not initialise the GPU)
        dev = torch.device('cuda', local % max(1, torch.cuda.device_count()))
        torch.cuda.set_device(dev)
        if world > 1:
            if args.dist_backend == 'nccl':
                dist.init_process_group('nccl', device_id=dev)
            else:
                dist.init_process_group('gloo')
        wl = NativeWorkload(args, dev, world, rank)
    D = importlib_dist()
    wl.prime(args.warmup)
    gens = max(1, math.ceil((args.steps or 1) / wl.steps_per_generation))
    if world > 1:
        dist.barrier()
    wl.sync()
    t0 = time.perf_counter()
    for g in range(gens):
        out = wl.generation(g)
    wl.sync()
    if world > 1:
        dist.barrier()
    el = D.max_over_ranks(time.perf_counter() - t0, device=dev if args.dist_backend == 'nccl' else None)
    steps = gens * wl.steps_per_generation
    value = wl.frames_per_generation * gens / el
    result = None
    if rank == 0:
        wl.check(out)
        if args.dump:
            torch.save(out.detach().cpu(), args.dump)
        meta = json.load(open(os.path.join(REPO, 'BASELINE.json')))
        T_ = wl.fd.diffusion.num_timesteps if hasattr(wl, 'fd') else 0
        sampler_ = f'DDPM {T_}' if args.sampling_steps >= T_ else f'DDIM {args.sampling_steps}'
        label = meta['metric'] if args.stub else metric_label(
            args.config, meta['metric'], sampler_, CONFIG_NAMES[args.config], wl.tc, args.total_pred,
            wl.w['baseline'].split(':')[0])
        result = {'metric': label, 'value': round(value, 4), 'unit': 'frames/s', 'n_gpus': world,
                  'steps': steps, 'warmup': args.warmup, 'ms_per_step': round(el / steps * 1e3, 4),
                  'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None}
        result.update(wl.describe())
        result['generations'] = gens
        result['requested_steps'] = args.steps if args.steps is not None else wl.steps_per_generation
        result['timed_s'] = round(el, 3)
        result['roofline'] = None if args.no_roofline else wl.roofline()
        result['partial'] = True
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()  # the other ranks stay up until rank 0 has printed
    if rank == 0:
        if not args.no_cpu_baseline and world == 1:
            result['cpu_baseline'] = wl.cpu_baseline()
        result['partial'] = False
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return result


def importlib_dist():
    import importlib
    return importlib.import_module(PKG + '.dist')


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, argv))
    return run_rank(args)


if __name__ == '__main__':
    main()
