"""Round-6 diagnosis: run-to-run determinism of each native stage under GPU contention.
Builds the bench's BAIR workload (batch --batch, DDPM steps --steps), takes reference outputs of
the encoder, one Unet forward at three t, one sampling call and the decode, then repeats each
stage --iters times and counts the repeats that are not bitwise equal to the reference (with
where the first mismatch lies). Run two copies at once on one GPU (the condition under which
tests/test_gpu_bench_ranks.py diverged); optional --hog runs large torch copies on a side stream
of this process between stages' launches."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402


def where(a, b):
    d = (a - b).abs()
    idx = torch.nonzero(d.reshape(d.shape[0], d.shape[1], d.shape[2], -1) > 0)
    if idx.numel() == 0:
        return 'equal'
    fr = sorted(set(idx[:, 2].tolist()))
    ch = sorted(set(idx[:, 1].tolist()))
    bs = sorted(set(idx[:, 0].tolist()))
    return f'max {float(d.max()):.3e} n={idx.shape[0]} clips {bs} ch {ch[:8]} frames {fr[:16]}'


def barrier(a):
    import glob
    if not a.sync:
        return
    open(f'{a.sync}.{a.tag}', 'w').close()
    t0 = time.time()
    while len(glob.glob(a.sync + '.*')) < a.peers and time.time() - t0 < 120:
        time.sleep(0.05)


def keep_going(a, it, t0):
    return time.time() - t0 < a.seconds if a.seconds else it < a.iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=4)
    ap.add_argument('--steps', type=int, default=4)
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--seconds', type=float, default=0, help='loop for this long instead of --iters')
    ap.add_argument('--sync', default='', help='start barrier: touch <sync>.<tag>, wait for --peers files')
    ap.add_argument('--peers', type=int, default=1)
    ap.add_argument('--tag', default='p')
    ap.add_argument('--stages', default='unet,sample,decode,encode')
    ap.add_argument('--eager', action='store_true', help='sample without the captured graph')
    ap.add_argument('--nch', type=int, default=1,
                    help='thresholds per (step, clip): 11 with the EXTDM_SAMPLER_DEBUG library (one per chunk)')
    a = ap.parse_args()
    dev = torch.device('cuda:0')
    torch.cuda.set_device(dev)
    args = bench.parse(['--batch', str(a.batch), '--sampling-steps', str(a.steps)])
    w = bench.NativeWorkload(args, dev, 1, 0)
    w.prime(1)
    pkg, fd, B = w.pkg, w.fd, a.batch
    ret, x_cond, fea, ref = fd.encode(w.clips)
    h = fd.diffusion._native(B, dev, fea.shape[-1])
    g = torch.Generator().manual_seed(5)
    x = torch.randn((B, 3, w.tp) + tuple(x_cond.shape[3:]), generator=g).to(dev)
    T = fd.diffusion.num_timesteps
    times = list(range(T - 1, T - 1 - a.steps, -1))
    stages = a.stages.split(',')

    def run_unet(tv):
        e = torch.empty_like(x)
        h.unet_forward(x, torch.full((B,), tv, dtype=torch.long, device=dev), x_cond, fea, e)
        return e

    rec = torch.full((a.steps * B * a.nch,), -1., device=dev)
    thr = []

    def run_sample():
        o = torch.empty_like(x)
        rec.fill_(-1.)
        h.record_thresholds(rec)
        h.sample(pkg._lib.SAMPLER_DDPM, times, None, 0., x_cond, fea, o, seed=77, sample_base=0,
                 use_graph=not a.eager)
        h.record_thresholds(None)
        thr.append(rec.view(a.steps, B, a.nch).cpu())
        return o

    def run_decode(o):
        return fd.decode(ret, o, ref)['sample_out_vid']

    refs = {}
    for tv in (999, 500, 3):
        refs[f'unet{tv}'] = run_unet(tv)
    refs['sample'] = run_sample()
    refs['decode'] = run_decode(refs['sample'])
    refs['encode'] = fd.encode(w.clips)[2]
    torch.cuda.synchronize()
    bad = {k: 0 for k in refs}
    first = {}
    barrier(a)
    t0 = time.time()
    it = -1
    while keep_going(a, it + 1, t0):
        it += 1
        cur = {}
        if 'unet' in stages:
            for tv in (999, 500, 3):
                cur[f'unet{tv}'] = run_unet(tv)
        if 'sample' in stages:
            cur['sample'] = run_sample()
        if 'decode' in stages:
            cur['decode'] = run_decode(refs['sample'])
        if 'encode' in stages:
            cur['encode'] = fd.encode(w.clips)[2]
        torch.cuda.synchronize()
        for k, v in cur.items():
            if not torch.equal(v, refs[k]):
                bad[k] += 1
                if k not in first:
                    first[k] = (it, where(v, refs[k]))
                if k == 'sample':
                    r0, r1 = thr[0], thr[-1]
                    spread = (r1 - r1[..., :1]).abs().amax(-1)  # chunks disagreeing within a (step, clip)
                    dif = torch.nonzero(r1 != r0).tolist()
                    print(f'[{a.tag}] iter {it} chunk spread per (step, clip) {spread.tolist()}; '
                          f'(step, clip, chunk) differing from ref: {dif[:12]}; {where(v, refs[k])}', flush=True)
        if it % 5 == 4:
            print(f'[{a.tag}] iter {it + 1} {time.time() - t0:.0f}s mismatches {bad}', flush=True)
    print(f'[{a.tag}] DONE mismatches {bad} in {it + 1} iterations, {time.time() - t0:.1f}s', flush=True)
    for k, (it, s) in first.items():
        print(f'[{a.tag}]   {k}: first at iter {it}: {s}', flush=True)


if __name__ == '__main__':
    main()
