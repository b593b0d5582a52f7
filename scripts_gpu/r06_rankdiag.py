"""Round-6 diagnosis of test_gpu_bench_ranks (one rank at B = 4 vs two ranks at B = 2 differ):
in ONE process, the bench workload at batch 4 and two batch-2 workloads (rank slices 0:2, 2:4),
compared stage by stage — encoder outputs, one Unet forward on identical inputs, one sampling
call, the decode — plus a repeat of the batch-4 generation (run-to-run determinism).
Prints the first stage that differs, max |diff| and which clips."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402


def md(a, b):
    return float((a.float() - b.float()).abs().max())


def report(name, full, parts):
    cat = torch.cat(parts, 0)
    d = md(full, cat)
    per = [md(full[i], cat[i]) for i in range(full.shape[0])]
    print(f'{name:34s} max|diff| {d:.3e}  per clip {["%.1e" % p for p in per]}  equal={torch.equal(full, cat)}',
          flush=True)
    return d


def main():
    dev = torch.device('cuda:0')
    torch.cuda.set_device(dev)
    steps = int(os.environ.get('DIAG_STEPS', '4'))
    a4 = bench.parse(['--batch', '4', '--sampling-steps', str(steps)])
    a2 = bench.parse(['--batch', '2', '--sampling-steps', str(steps)])
    w4 = bench.NativeWorkload(a4, dev, 1, 0)
    w2 = [bench.NativeWorkload(a2, dev, 2, r) for r in range(2)]
    for w in [w4] + w2:
        w.prime(1)
    pkg = w4.pkg
    print('clips equal:', torch.equal(w4.clips, torch.cat([w.clips for w in w2])), flush=True)
    # weights equal?
    sd4 = w4.fd.state_dict()
    for r, w in enumerate(w2):
        sd = w.fd.state_dict()
        bad = [k for k in sd4 if not torch.equal(sd4[k].cpu(), sd[k].cpu())]
        print(f'rank {r} state_dict keys differing: {len(bad)} {bad[:5]}', flush=True)

    # 1. encoder
    e4 = w4.fd.encode(w4.clips)
    e2 = [w.fd.encode(w.clips) for w in w2]
    report('encode x_cond', e4[1], [e[1] for e in e2])
    report('encode fea', e4[2], [e[2] for e in e2])
    for k in e4[0]:
        report(f'encode ret[{k}]', e4[0][k], [e[0][k] for e in e2])
    # 2. one Unet forward on identical inputs (the batch-4 encoder's x_cond / fea)
    x_cond, fea = e4[1], e4[2]
    h4 = w4.fd.diffusion._native(4, dev, fea.shape[-1])
    h2 = [w.fd.diffusion._native(2, dev, fea.shape[-1]) for w in w2]
    g = torch.Generator().manual_seed(5)
    x = torch.randn((4, 3, w4.tp) + tuple(x_cond.shape[3:]), generator=g).to(dev)
    for tv in (999, 500, 3):
        t = torch.full((4,), tv, dtype=torch.long, device=dev)
        eps4 = torch.empty_like(x)
        h4.unet_forward(x, t, x_cond, fea, eps4)
        parts = []
        for r in range(2):
            sl = slice(2 * r, 2 * r + 2)
            e = torch.empty_like(x[sl])
            h2[r].unet_forward(x[sl].contiguous(), t[sl].contiguous(), x_cond[sl].contiguous(), fea[sl].contiguous(), e)
            parts.append(e)
        torch.cuda.synchronize()
        report(f'unet eps t={tv}', eps4, parts)
        eps4b = torch.empty_like(x)
        h4.unet_forward(x, t, x_cond, fea, eps4b)
        torch.cuda.synchronize()
        print(f'   unet repeat equal: {torch.equal(eps4, eps4b)}', flush=True)
    # 3. one sampling call (graph path), same inputs, Philox noise keyed by global index
    T = w4.fd.diffusion.num_timesteps
    times = list(range(T - 1, T - 1 - steps, -1))
    o4 = torch.empty_like(x)
    h4.sample(pkg._lib.SAMPLER_DDPM, times, None, 0., x_cond, fea, o4, seed=77, sample_base=0)
    parts = []
    for r in range(2):
        sl = slice(2 * r, 2 * r + 2)
        o = torch.empty_like(x[sl])
        h2[r].sample(pkg._lib.SAMPLER_DDPM, times, None, 0., x_cond[sl].contiguous(), fea[sl].contiguous(), o,
                     seed=77, sample_base=2 * r)
        parts.append(o)
    torch.cuda.synchronize()
    report(f'sample DDPM {steps} steps', o4, parts)
    o4b = torch.empty_like(x)
    h4.sample(pkg._lib.SAMPLER_DDPM, times, None, 0., x_cond, fea, o4b, seed=77, sample_base=0)
    torch.cuda.synchronize()
    print(f'   sample repeat equal: {torch.equal(o4, o4b)}', flush=True)
    # 4. decode of identical predictions
    d4 = w4.fd.decode(e4[0], o4, e4[3])['sample_out_vid']
    d2 = [w.fd.decode(e[0], o4[2 * r:2 * r + 2].contiguous(), e[3])['sample_out_vid'] for r, (w, e) in enumerate(zip(w2, e2))]
    report('decode', d4, d2)
    # 5. whole generations as the bench runs them
    g4 = pkg.autoregressive_sample(w4.fd, w4.clips, a4.total_pred, seed=1234, sample_base=0)
    g4b = pkg.autoregressive_sample(w4.fd, w4.clips, a4.total_pred, seed=1234, sample_base=0)
    g2 = [pkg.autoregressive_sample(w.fd, w.clips, a2.total_pred, seed=1234, sample_base=w.start) for w in w2]
    torch.cuda.synchronize()
    print(f'generation repeat equal: {torch.equal(g4, g4b)} max|diff| {md(g4, g4b):.3e}', flush=True)
    report('generation', g4, g2)


if __name__ == '__main__':
    main()
