"""ExtDM sampling throughput on MI355X: predicted frames/sec/node.

Workload (BASELINE.json configs[1]): BAIR 64x64 ch3, 2 -> 28 (tc = 2, tp = 14
per autoregressive round x 2 rounds), DDPM 1000 steps, u12 Unet3D (dim 64,
dim_mults 1,2,4,4) behind the multi_w_ref FlowDiffusion wrapper, random-init
weights, synthetic clips resident in HBM. BAIR eval default: no occlusion map
(valid_DM_bair.sh omits --estimate_occlusion_map).

One bench "step" = the eval driver's full 2 -> 28 generation of the per-GPU clip
batch (scripts/DM/valid.py:141-186 through the package's autoregressive_sample):
per round the LFAE encoder on the tc cond frames (region / background / flow
predictors, bottleneck features), the DDPM-1000 reverse loop (one captured
hipGraph step replayed 1000x: Unet3D forward + fused threshold/posterior/noise
step) and the flow-warp decode of the round's tc + tp frames; then (N > 1) an
RCCL all-gather of the generated videos to every rank.

Clip batches are sharded over ranks (weak scaling, one process per GPU); the
noise is a counter-based Philox stream keyed by (seed, global sample index,
round, step), so a clip's result does not depend on the shard it lands on.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
"""
import argparse
import json
import os
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=1)
    ap.add_argument('--warmup', type=int, default=0)
    ap.add_argument('--batch', type=int, default=64, help='clips per GPU')
    ap.add_argument('--sampling-steps', type=int, default=1000,
                    help='1000 = DDPM-1000 (the metric); fewer = DDIM-S (profiling sweeps only)')
    ap.add_argument('--total-pred', type=int, default=28)
    ap.add_argument('--tp', type=int, default=14)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-steps', type=int, default=4)
    ap.add_argument('--precision', default=None, choices=['fp32', 'f16x3'],
                    help='conv arithmetic (include/extdm.h EXTDM_PRECISION_*); default: the package default')
    return ap.parse_args()


def synthetic_clips(B, tc, S, seed):
    """Conditioning clips U[0,1) from NumPy PCG64."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(rng.random((B, 3, tc, S, S), dtype=np.float32))


def cpu_baseline(pkg, fd, rounds, steps_per_round, n_steps):
    """The oracle (PyTorch-CPU restatement of the reference) timed on this box's
    host cores at B = 1: one round's LFAE encoder, n_steps DDPM steps (Unet
    forward + p_sample update) and one round's decode, extrapolated to the same
    2 -> 28 workload."""
    import dataclasses
    from oracle import extdm_oracle as O
    from oracle import lfae_oracle as LO
    ucfg = fd.unet.ucfg
    lc = dataclasses.replace(fd.lcfg)
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
        t0 = time.perf_counter()
        for k in range(n_steps):
            t = torch.full((1,), 998 - k, dtype=torch.long)
            x = O.ddpm_step(sch, x, O.unet_forward(usd, ucfg.as_dict(), x, t, x_cond, fea), t, torch.randn_like(x))
        t_step = (time.perf_counter() - t0) / n_steps
        t0 = time.perf_counter()
        LO.decode_round(sd, lc, ucfg, ret, x, ref)
        t_dec = time.perf_counter() - t0
    total = rounds * (t_enc + steps_per_round * t_step + t_dec)
    return {'value': rounds * ucfg.tp / total, 'unit': 'frames/s', 'cores': torch.get_num_threads(),
            'kind': 'port',
            'sample': f'oracle B=1: encoder round ({t_enc:.3f} s), {n_steps} DDPM steps ({t_step:.3f} s/step), '
                      f'decode round ({t_dec:.3f} s); extrapolated to {rounds} rounds x {steps_per_round} steps'}


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('nccl', device_id=dev)
    import importlib
    pkg = importlib.import_module(PKG)
    B, S_steps = args.batch, args.sampling_steps
    wrapper, unet_arch = pkg.configs.dm_arch('bair')
    cfg = pkg.configs.dm_config('bair', pred_frames=args.tp, sampling_timesteps=S_steps,
                                estimate_occlusion_map=False)
    fd = pkg.FlowDiffusion(config=cfg, is_train=False, Unet3D_architecture=unet_arch, wrapper=wrapper).to(dev)
    fd.diffusion.max_batch = B
    precision = args.precision or pkg._lib.DEFAULT_PRECISION
    fd.unet.precision = precision
    tc, tp = fd.cond_frame_num, fd.pred_frame_num
    rounds = -(-args.total_pred // tp)
    clips = synthetic_clips(B, tc, 64, 1234 + rank).to(dev)

    D = pkg.dist
    start, count = D.shard(world * B, world, rank)  # weak scaling: B clips per rank

    def one_step(step_idx):
        out = pkg.autoregressive_sample(fd, clips, args.total_pred, num_sample_video=1, seed=1234 + step_idx,
                                        sample_base=start)
        return D.gather_shards(out.contiguous(), world * B, world)  # RCCL all-gather over xGMI

    # prime (untimed): build every native handle, load kernels, capture + replay the
    # step graph once on a 2-step schedule, run the encoder and the decoder
    ret, x_cond, fea, ref = fd.encode(clips)
    h = fd.diffusion._native(B, dev)
    prime = torch.empty(B, 3, tp, x_cond.shape[3], x_cond.shape[4], device=dev)
    h.sample(pkg._lib.SAMPLER_DDPM, [999, 998], None, 0., x_cond, fea, prime, seed=1, sample_base=start)
    fd.decode(ret, prime, ref)
    for w in range(args.warmup):
        one_step(-1 - w)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        out = one_step(k)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = D.max_over_ranks(time.perf_counter() - t0, device=dev)
    frames = world * B * args.total_pred * args.steps
    value = frames / el

    result = None
    if rank == 0:
        assert torch.isfinite(out).all()
        ms_layer, flops = h.bench_layer(B, 0, 20)
        achieved = flops / (ms_layer * 1e-3) / 1e12
        if precision == 'f16x3':
            kname, peak = 'conv_x3_kernel<7,64,512,1,8,16,1> (init_conv 512->64, 1x7x7, f16x3)', F16X3_PEAK_TFLOPS
        else:
            kname, peak = 'conv_halo_kernel<7,64,1,128> (init_conv 512->64, 1x7x7, fp32 MFMA)', FP32_MFMA_PEAK_TFLOPS
        traffic = None
        pmc = os.path.join(REPO, 'profiles', 'pmc_init_conv.json')
        if os.path.exists(pmc):
            try:
                j = json.load(open(pmc))
                if int(j.get('batch', -1)) == B and j.get('precision', 'fp32') == precision:
                    traffic = j.get('hbm_bytes_per_launch')
            except (ValueError, OSError):
                traffic = None
        meta = json.load(open(os.path.join(REPO, 'BASELINE.json')))
        sampler = 'DDPM 1000' if S_steps >= 1000 else f'DDIM {S_steps}'
        result = {
            'metric': meta['metric'], 'value': round(value, 4), 'unit': 'frames/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(el / args.steps * 1e3, 2),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
            'dtype': 'fp32' if precision == 'fp32' else 'fp32 (f16x3 split-MFMA convs + attention, fp32 accumulate)',
            'data': 'synthetic (U[0,1) PCG64 clips, seeded random-init weights; no dataset/checkpoint offline)',
            'config': {'workload': f'BAIR 64x64 ch3 {tc}->{args.total_pred} (tp={tp} x {rounds} rounds), '
                                   f'{sampler} steps, u12 Unet3D dim 64 mults (1,2,4,4), LFAE encoder + '
                                   f'flow-warp decoder, no occlusion map (BAIR eval default)',
                       'global_batch': world * B, 'batch_per_gpu': B, 'sampling_steps': S_steps,
                       'rounds': rounds, 'parallelism': f'clip-shard x{world} (+RCCL all-gather)',
                       'workspace_gb': round(h.workspace_bytes() / 2 ** 30, 2)},
            'roofline': {'bound': 'mfma', 'kernel': kname, 'achieved': round(achieved, 2), 'peak': round(peak, 1),
                         'unit': 'TFLOP/s', 'frac': round(achieved / peak, 4), 'traffic': traffic},
        }
        if not args.no_cpu_baseline and world == 1:
            result['cpu_baseline'] = cpu_baseline(pkg, fd, rounds, 1000, args.cpu_steps)
        print(json.dumps(result))
    if world > 1:
        torch.distributed.destroy_process_group()
    return result


if __name__ == '__main__':
    main()
