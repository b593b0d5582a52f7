"""ExtDM sampling throughput on MI355X: predicted frames/sec/node.

Workload (BASELINE.json configs[1]): BAIR 64x64 ch3, 2 -> 28 (tc = 2, tp = 14
per autoregressive round x 2 rounds), DDPM 1000 steps, u12 Unet3D (dim 64,
dim_mults 1,2,4,4) behind the multi_w_ref FlowDiffusion wrapper, random-init
weights, synthetic clips resident in HBM. BAIR eval default: no occlusion map
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

Output: rank 0 prints (and flushes) a JSON line as soon as the timed region and
the roofline launch timing are done, marked "partial": true, then the complete
line with `cpu_baseline` once the CPU port has been timed. The last line is the
result.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
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
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=2000,
                    help='reverse-diffusion steps to time, rounded up to whole generations (>= 1)')
    ap.add_argument('--warmup', type=int, default=5, help='untimed graph replays')
    ap.add_argument('--batch', type=int, default=64, help='clips per GPU')
    ap.add_argument('--sampling-steps', type=int, default=1000,
                    help='1000 = DDPM-1000 (the metric); fewer = DDIM-S (profiling sweeps only)')
    ap.add_argument('--total-pred', type=int, default=28)
    ap.add_argument('--tp', type=int, default=14)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-steps', type=int, default=8)
    ap.add_argument('--precision', default=None, choices=['fp32', 'f16x3'],
                    help='conv / attention arithmetic (include/extdm.h EXTDM_PRECISION_*); default: package default')
    ap.add_argument('--stub', action='store_true',
                    help='test-only: CPU/gloo stand-in workload that exercises the launcher and rank plumbing')
    return ap.parse_args(argv)


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


class NativeWorkload:
    """The product path: FlowDiffusion + autoregressive_sample on the HIP library."""

    def __init__(self, args, dev, world, rank):
        import importlib
        pkg = importlib.import_module(PKG)
        self.pkg, self.args, self.dev, self.world, self.rank = pkg, args, dev, world, rank
        B = args.batch
        wrapper, unet_arch = pkg.configs.dm_arch('bair')
        cfg = pkg.configs.dm_config('bair', pred_frames=args.tp, sampling_timesteps=args.sampling_steps,
                                    estimate_occlusion_map=False)
        fd = pkg.FlowDiffusion(config=cfg, is_train=False, Unet3D_architecture=unet_arch, wrapper=wrapper).to(dev)
        fd.diffusion.max_batch = B
        self.precision = args.precision or pkg._lib.DEFAULT_PRECISION
        fd.unet.precision = self.precision
        self.fd = fd
        self.tc, self.tp = fd.cond_frame_num, fd.pred_frame_num
        self.rounds = -(-args.total_pred // self.tp)
        self.steps_per_generation = self.rounds * args.sampling_steps
        self.frames_per_generation = world * B * args.total_pred
        self.clips = synthetic_clips(B, self.tc, 64, 1234 + rank).to(dev)
        self.start, _ = pkg.dist.shard(world * B, world, rank)  # weak scaling: B clips per rank
        self.h = None

    def prime(self, warmup):
        """Untimed: build every native handle (weights packed, workspace planned),
        capture the step graph and replay it `warmup` times, run encoder + decoder."""
        fd, B, pkg = self.fd, self.args.batch, self.pkg
        ret, x_cond, fea, ref = fd.encode(self.clips)
        self.h = h = fd.diffusion._native(B, self.dev)
        prime = torch.empty(B, 3, self.tp, x_cond.shape[3], x_cond.shape[4], device=self.dev)
        n = max(1, warmup)
        h.sample(pkg._lib.SAMPLER_DDPM, list(range(999, 999 - n, -1)), None, 0., x_cond, fea, prime, seed=1,
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
        a, B = self.args, self.args.batch
        sampler = 'DDPM 1000' if a.sampling_steps >= 1000 else f'DDIM {a.sampling_steps}'
        return {
            'dtype': 'fp32' if self.precision == 'fp32' else
                     'fp32 (f16x3 split-MFMA convs + attention, fp32 accumulate)',
            'data': 'synthetic (U[0,1) PCG64 clips, seeded random-init weights; no dataset/checkpoint offline)',
            'config': {'workload': f'BAIR 64x64 ch3 {self.tc}->{a.total_pred} (tp={self.tp} x {self.rounds} rounds), '
                                   f'{sampler} steps, u12 Unet3D dim 64 mults (1,2,4,4), LFAE encoder + '
                                   f'flow-warp decoder, no occlusion map (BAIR eval default)',
                       'global_batch': self.world * B, 'batch_per_gpu': B, 'sampling_steps': a.sampling_steps,
                       'rounds': self.rounds, 'parallelism': f'clip-shard x{self.world} (+RCCL all-gather)',
                       'workspace_gb': round(self.h.workspace_bytes() / 2 ** 30, 2)}}

    # extdm_bench_layer ids (runtime.cpp) of the kernels reported, dominant first: the
    # level-0 ResnetBlock 3x3 conv (64 -> 64 at 32x32, the largest share of GPU time per
    # step, profiles/r02_*_kernel_stats.csv; block1's conv stages an fp32 input, block2's
    # copies block1's pre-split operand, id 5), init_conv's cond_fea branch (256 -> 64,
    # 7x7; the x-branch is the composed xpath_x3 kernel) and the level-0 1x1 res_conv
    # (128 -> 64), which is HBM-bound: 3 FLOP-equivalents of f16x3 MFMA per 4-B element
    # moved is far below the machine balance, so it is priced against HBM bytes.
    LAYERS = [(1, 'mfma', 'conv_x3_kernel<3,1,64,256,1,4,4,2,SPAN,NS=2>', 'level-0 ResnetBlock block1 conv 64->64 1x3x3, fp32 input staged', 64, 64),
              (5, 'mfma', 'conv_x3_kernel<3,1,64,256,1,4,4,2,SPAN,XOP>', 'level-0 ResnetBlock block2 conv 64->64 1x3x3, pre-split operand by LDS-DMA', 64, 64),
              (0, 'mfma', 'conv_x3_kernel<7,1,64,512,1,8,16,1>', 'init_conv cond_fea branch 256->64 1x7x7', 256, 64),
              (4, 'hbm', 'conv_x3_kernel<1,1,64,128,2,4,4,2>', 'level-0 res_conv 128->64 1x1x1', 128, 64)]

    def _traffic(self, layer):
        """HBM bytes per launch from the committed PMC passes (scripts_gpu/pmc_layers.sh)."""
        pmc = os.path.join(REPO, 'profiles', f'pmc_layer{layer}.json')
        try:
            j = json.load(open(pmc))
            if int(j.get('batch', -1)) == self.args.batch and j.get('precision') == self.precision:
                return j.get('hbm_bytes_per_launch')
        except (ValueError, OSError):
            pass
        return None

    def roofline(self):
        """Per kernel, timed over 20 launches of the exact forward launch with HIP events
        on the handle's stream (extdm_bench_layer). MFMA-bound: FLOP per launch / time
        against the f16x3 peak (dense fp16 MFMA / 3). HBM-bound: algorithmic bytes per
        launch (fp32 input + output elements, 4 B each, weights aside) / time against
        8 TB/s. The first entry is the dominant kernel; the others ride along."""
        B = self.args.batch
        peak = F16X3_PEAK_TFLOPS if self.precision == 'f16x3' else FP32_MFMA_PEAK_TFLOPS
        u = self.fd.unet.ucfg
        T = self.tc + self.tp
        out = []
        for layer, bound, kname, what, cin, cout in self.LAYERS:
            if layer == 5 and self.precision != 'f16x3':
                continue
            ms_layer, flops = self.h.bench_layer(B, layer, 20)
            traffic = self._traffic(layer)
            if bound == 'mfma':
                achieved = flops / (ms_layer * 1e-3) / 1e12
                e = {'bound': 'mfma', 'achieved': round(achieved, 2), 'peak': round(peak, 1), 'unit': 'TFLOP/s',
                     'frac': round(achieved / peak, 4), 'flop_per_launch': flops}
            else:
                nbytes = 4 * B * T * u.latent * u.latent * (cin + cout)
                achieved = nbytes / (ms_layer * 1e-3) / 1e9
                e = {'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(achieved / HBM_PEAK_GBS, 4), 'bytes_per_launch': nbytes}
            e.update({'kernel': f'{kname} ({what}, {self.precision})', 'traffic': traffic,
                      'launch_ms': round(ms_layer, 4)})
            out.append(e)
        res = out[0]
        res['others'] = out[1:]
        return res

    def cpu_baseline(self):
        return cpu_baseline(self.fd, self.rounds, self.args.sampling_steps, self.args.cpu_steps)


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


def cpu_baseline(fd, rounds, steps_per_round, n_steps):
    """The oracle (PyTorch-CPU restatement of the reference, kind "port") timed on
    this box's host cores at B = 1: one round's LFAE encoder, n_steps DDPM steps
    (Unet forward + p_sample update) and one round's decode, extrapolated to the
    same 2 -> 28 workload. Oracle use is confined to this untimed checker leg."""
    from oracle import extdm_oracle as O
    from oracle import lfae_oracle as LO
    ucfg = fd.unet.ucfg
    lc = fd.lcfg
    sd = {f'generator.{k}': v.detach().cpu() for k, v in fd.generator.state_dict().items()}
    sd.update({f'region_predictor.{k}': v.detach().cpu() for k, v in fd.region_predictor.state_dict().items()})
    sd.update({f'bg_predictor.{k}': v.detach().cpu() for k, v in fd.bg_predictor.state_dict().items()})
    usd = {k: v.detach().cpu() for k, v in fd.unet.state_dict().items()}
    sch = O.schedule(1000)
    vid = synthetic_clips(1, ucfg.tc, lc.image, 99)
    with torch.no_grad():
        t0 = time.perf_counter()
        ret, x_cond, fea, ref = LO.encode_round(sd, lc, ucfg, vid)
        t_enc = time.perf_counter() - t0
        x = torch.randn(1, 3, ucfg.tp, ucfg.latent, ucfg.latent)
        t = torch.full((1,), 999, dtype=torch.long)
        O.ddpm_step(sch, x, O.unet_forward(usd, ucfg.as_dict(), x, t, x_cond, fea), t, torch.randn_like(x))  # warm
        per = []
        for k in range(n_steps):
            t = torch.full((1,), 998 - k, dtype=torch.long)
            t0 = time.perf_counter()
            x = O.ddpm_step(sch, x, O.unet_forward(usd, ucfg.as_dict(), x, t, x_cond, fea), t, torch.randn_like(x))
            per.append(time.perf_counter() - t0)
        t_step = float(np.median(per))
        t0 = time.perf_counter()
        LO.decode_round(sd, lc, ucfg, ret, x, ref)
        t_dec = time.perf_counter() - t0
    total = rounds * (t_enc + steps_per_round * t_step + t_dec)
    return {'value': round(rounds * ucfg.tp / total, 5), 'unit': 'frames/s', 'cores': torch.get_num_threads(),
            'kind': 'port', 'cpu_model': cpu_model(),
            'sample': f'oracle (PyTorch-CPU fp32) B=1: encoder round ({t_enc:.3f} s), {n_steps} DDPM steps '
                      f'(median {t_step:.3f} s/step, range {min(per):.3f}-{max(per):.3f}), decode round '
                      f'({t_dec:.3f} s); extrapolated to {rounds} rounds x {steps_per_round} steps'}


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
        torch.cuda.set_device(local)
        dev = torch.device('cuda', local)
        if world > 1:
            dist.init_process_group('nccl', device_id=dev)
        wl = NativeWorkload(args, dev, world, rank)
    D = importlib_dist()
    wl.prime(args.warmup)
    gens = max(1, math.ceil(args.steps / wl.steps_per_generation))
    if world > 1:
        dist.barrier()
    wl.sync()
    t0 = time.perf_counter()
    for g in range(gens):
        out = wl.generation(g)
    wl.sync()
    if world > 1:
        dist.barrier()
    el = D.max_over_ranks(time.perf_counter() - t0, device=dev)
    steps = gens * wl.steps_per_generation
    value = wl.frames_per_generation * gens / el
    result = None
    if rank == 0:
        wl.check(out)
        meta = json.load(open(os.path.join(REPO, 'BASELINE.json')))
        result = {'metric': meta['metric'], 'value': round(value, 4), 'unit': 'frames/s', 'n_gpus': world,
                  'steps': steps, 'warmup': args.warmup, 'ms_per_step': round(el / steps * 1e3, 4),
                  'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None}
        result.update(wl.describe())
        result['generations'] = gens
        result['requested_steps'] = args.steps
        result['timed_s'] = round(el, 3)
        result['roofline'] = wl.roofline()
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
