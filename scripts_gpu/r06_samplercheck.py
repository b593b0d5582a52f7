"""Round-6 diagnosis: the sampler step alone (extdm_sampler_step on fixed x / eps / noise),
repeated; every repeat must be bitwise equal to the first. Run beside another GPU process."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from tests.sampler_run import bair_handle  # noqa: E402


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
    ap.add_argument('--iters', type=int, default=400)
    ap.add_argument('--seconds', type=float, default=0, help='loop for this long instead of --iters')
    ap.add_argument('--sync', default='', help='start barrier: touch <sync>.<tag>, wait for --peers files')
    ap.add_argument('--peers', type=int, default=1)
    ap.add_argument('--tag', default='s')
    a = ap.parse_args()
    dev = torch.device('cuda:0')
    B = a.batch
    h = bair_handle(B)
    n = 3 * 14 * 32 * 32
    g = torch.Generator().manual_seed(3)
    x0 = torch.randn(B, n, generator=g).to(dev)
    eps = (torch.randn(B, n, generator=g) * 0.999).to(dev)
    noise = torch.randn(1, B, n, generator=g).to(dev)
    th = torch.zeros(B, device=dev)
    ref = None
    bad = 0
    barrier(a)
    t0 = time.time()
    it = -1
    while keep_going(a, it + 1, t0):
        it += 1
        x = x0.clone()
        h.sampler_step(0, 700 - (it % 3), 0, 0., x, eps, noise, th)
        torch.cuda.synchronize()
        if it < 3:
            ref = ref or {}
            ref[it] = (x.clone(), th.clone())
            continue
        rx, rt = ref[it % 3]
        if not torch.equal(x, rx):
            bad += 1
            d = (x - rx).abs()
            idx = torch.nonzero(d > 0)
            print(f'[{a.tag}] iter {it}: {idx.shape[0]} elements differ, max {float(d.max()):.3e}, '
                  f'thresh equal {torch.equal(th, rt)}, first idx {idx[:6].tolist()}', flush=True)
    print(f'[{a.tag}] DONE {bad} of {it - 2} repeats differ ({time.time() - t0:.1f}s)', flush=True)


if __name__ == '__main__':
    main()
