"""ExtDM sampling throughput on MI355X: predicted frames/sec/node.

Workload (BASELINE.json configs[1]): BAIR 64x64 ch3, 2 -> 28 (tc = 2, tp = 14
per autoregressive round x 2 rounds), DDPM 1000 steps, u12 Unet3D (dim 64,
dim_mults 1,2,4,4), random-init weights, synthetic inputs resident in HBM.

One bench "step" = one full 2 -> 28 sample of the per-GPU clip batch:
  for each of the 2 rounds: the DDPM-1000 reverse loop (one captured hipGraph
  step replayed 1000x: Unet3D forward + fused threshold/posterior/noise step)
  and the LFAE flow-warp decode of the round's tc + tp frames;
then (N > 1) an RCCL all-gather of the predicted frames to every rank.
The LFAE encoder is not in this build yet: round 1 uses
synthetic flow / bottleneck conditioning and round 2 conditions on round 1's
last predicted flows (+ zero occlusion channel, the BAIR eval default).

Clip batches are sharded over ranks (weak scaling, one process per GPU);
noise is a counter-based Philox stream keyed by the global sample index, so a
clip's result does not depend on the shard it lands on.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
PKG = '140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd'
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense fp32 matrix peak


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=1)
    ap.add_argument('--warmup', type=int, default=0)
    ap.add_argument('--batch', type=int, default=32, help='clips per GPU')
    ap.add_argument('--sampling-steps', type=int, default=1000)
    ap.add_argument('--rounds', type=int, default=2)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-steps', type=int, default=4)
    return ap.parse_args()


def cpu_baseline(ucfg, rounds, steps_per_round, n_steps):
    """The oracle (PyTorch-CPU restatement of the reference) timed on this box's
    host cores: B = 1, n_steps DDPM steps (Unet forward + p_sample update) and
    one round's decode, extrapolated to frames/s for the same 2 -> 28 workload."""
    from oracle import extdm_oracle as O
    import importlib
    pkg = importlib.import_module(PKG)
    torch.manual_seed(0)
    sd = pkg.weights.synth_state_dict(pkg.spec.unet_spec(ucfg), seed=1234)
    sch = O.schedule(1000)
    L, fs = ucfg.latent, ucfg.fea_size
    x = torch.randn(1, 3, ucfg.tp, L, L)
    cond = torch.rand(1, 3, ucfg.tc, L, L) * 2 - 1
    fea = torch.randn(1, 256, ucfg.tc + ucfg.tp, fs, fs)
    with torch.no_grad():
        t = torch.full((1,), 999, dtype=torch.long)
        O.ddpm_step(sch, x, O.unet_forward(sd, ucfg.as_dict(), x, t, cond, fea), t, torch.randn_like(x))  # warm
        t0 = time.perf_counter()
        for k in range(n_steps):
            t = torch.full((1,), 998 - k, dtype=torch.long)
            x = O.ddpm_step(sch, x, O.unet_forward(sd, ucfg.as_dict(), x, t, cond, fea), t, torch.randn_like(x))
        t_step = (time.perf_counter() - t0) / n_steps
        src = torch.rand(1, 3, 64, 64)
        flow = torch.rand(1, 32, 32, 2) * 2 - 1
        t0 = time.perf_counter()
        for _ in range(ucfg.tc + ucfg.tp):
            O.deform(src, flow)
        t_dec = time.perf_counter() - t0
    total = rounds * (steps_per_round * t_step + t_dec)
    return {'value': rounds * ucfg.tp / total, 'unit': 'frames/s', 'cores': torch.get_num_threads(),
            'kind': 'port',
            'sample': f'oracle B=1: {n_steps} DDPM steps ({t_step:.3f} s/step) + one round decode '
                      f'({t_dec:.4f} s), extrapolated to {rounds} rounds x {steps_per_round} steps'}


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
    ucfg = pkg.spec.UnetConfig()  # BAIR u12
    B = args.batch
    S = args.sampling_steps
    tc, tp, L, fs = ucfg.tc, ucfg.tp, ucfg.latent, ucfg.fea_size

    h = pkg._lib.Handle(ucfg, 1000, B, local)
    sd = pkg.weights.synth_state_dict(pkg.spec.unet_spec(ucfg), seed=1234)
    sd.update(pkg.schedule_buffers(1000))
    h.load_state(sd)
    h.finalize()
    gen = pkg.Generator()

    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x_cond0 = torch.cat([torch.rand(B, 2, tc, L, L, device=dev, generator=g) * 2 - 1,
                         torch.zeros(B, 1, tc, L, L, device=dev)], dim=1).contiguous()
    fea = torch.randn(B, 256, tc + tp, fs, fs, device=dev, generator=g).contiguous()
    ref_img = torch.rand(B, 3, 64, 64, device=dev, generator=g).contiguous()
    out_vid = torch.empty(B, 3, args.rounds * tp, 64, 64, device=dev)
    times = list(range(S - 1, -1, -1)) if S == 1000 else [int(round(999 * (1 - k / max(S - 1, 1)))) for k in range(S)]

    def one_step(step_idx):
        x_cond = x_cond0
        for r in range(args.rounds):
            pred = torch.empty(B, 3, tp, L, L, device=dev)
            h.sample(pkg._lib.SAMPLER_DDPM, times, None, 0., x_cond, fea, pred, seed=1234 + step_idx,
                     sample_base=rank * B, round_idx=r)
            flows = torch.cat([x_cond[:, :2], pred[:, :2]], dim=2).contiguous()
            frames = gen.decode_frames(ref_img, flows)  # (B, 3, tc + tp, 64, 64)
            out_vid[:, :, r * tp:(r + 1) * tp] = frames[:, :, tc:]
            x_cond = torch.cat([pred[:, :2, -tc:], torch.zeros(B, 1, tc, L, L, device=dev)], dim=1).contiguous()
        if world > 1:
            allv = torch.empty((world,) + tuple(out_vid.shape), device=dev)
            torch.distributed.all_gather_into_tensor(allv, out_vid)
        return out_vid

    # prime: load every kernel and capture / replay the step graph once (2 denoising steps, untimed)
    prime = torch.empty(B, 3, tp, L, L, device=dev)
    h.sample(pkg._lib.SAMPLER_DDPM, times[:2], None, 0., x_cond0, fea, prime, seed=1, sample_base=rank * B)
    gen.decode_frames(ref_img, torch.cat([x_cond0[:, :2], prime[:, :2]], dim=2).contiguous())
    for w in range(args.warmup):
        one_step(-1 - w)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        one_step(k)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([el], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        el = float(tt.item())
    frames = world * B * args.rounds * tp * args.steps
    value = frames / el

    result = None
    if rank == 0:
        assert torch.isfinite(out_vid).all()
        ms_layer, flops = h.bench_layer(B, 0, 20)
        achieved = flops / (ms_layer * 1e-3) / 1e12
        traffic = None
        pmc = os.path.join(REPO, 'profiles', 'pmc_init_conv.json')
        if os.path.exists(pmc):
            try:
                j = json.load(open(pmc))
                if int(j.get('batch', -1)) == B:
                    traffic = j.get('hbm_bytes_per_launch')
            except Exception:
                traffic = None
        meta = json.load(open(os.path.join(REPO, 'BASELINE.json')))
        result = {
            'metric': meta['metric'], 'value': round(value, 4), 'unit': 'frames/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(el / args.steps * 1e3, 2),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'fp32',
            'data': 'synthetic (seeded random-init weights, synthetic conditioning; no dataset/checkpoint offline)',
            'config': {'workload': f'BAIR 64x64 ch3 2->{args.rounds * tp} (tc={tc}, tp={tp} x {args.rounds} rounds), '
                                   f'DDPM {S} steps, u12 Unet3D dim 64 mults (1,2,4,4)',
                       'global_batch': world * B, 'batch_per_gpu': B, 'sampling_steps': S,
                       'rounds': args.rounds, 'parallelism': f'clip-shard x{world} (+RCCL all-gather)',
                       'workspace_gb': round(h.workspace_bytes() / 2 ** 30, 2)},
            'roofline': {'bound': 'mfma', 'kernel': 'conv_halo_kernel<7,64,1> (init_conv 512->64, 1x7x7)',
                         'achieved': round(achieved, 2), 'peak': FP32_MFMA_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                         'frac': round(achieved / FP32_MFMA_PEAK_TFLOPS, 4), 'traffic': traffic},
        }
        if not args.no_cpu_baseline and world == 1:
            result['cpu_baseline'] = cpu_baseline(ucfg, args.rounds, 1000, args.cpu_steps)
        print(json.dumps(result))
    if world > 1:
        torch.distributed.destroy_process_group()
    return result


if __name__ == '__main__':
    main()
