"""Helper process of tests/test_gpu_sampler.py (not a test module): one of two GPU processes
started together (a file barrier), each repeating a native call on fixed inputs for --seconds and
counting the repeats that are not bitwise equal to the first:
  --mode step    extdm_sampler_step alone (full BAIR sample size, B = 4, injected noise)
  --mode sample  whole captured-graph sampling calls (DDPM, 4 steps, Philox noise)
Prints one JSON line {"mode", "repeats", "mismatches", "first"}. Two processes on one GPU are the
condition under which hipcc's SLP-packed form of the sampler update went wrong."""
import argparse
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def main():
    import torch
    from tests.golden_inputs import CONFIGS, unet_inputs
    from tests.sampler_run import bair_handle
    ap = argparse.ArgumentParser()
    ap.add_argument('--mode', choices=['step', 'sample'], required=True)
    ap.add_argument('--seconds', type=float, default=8.0)
    ap.add_argument('--sync', required=True)
    ap.add_argument('--peers', type=int, default=2)
    a = ap.parse_args()
    dev = torch.device('cuda:0')
    cfg = CONFIGS['bair']
    B = 4 if a.mode == 'step' else 2
    h = bair_handle(B)
    n = 3 * cfg.tp * cfg.latent * cfg.latent
    g = torch.Generator().manual_seed(3)
    if a.mode == 'step':
        x0 = torch.randn(B, n, generator=g).to(dev)
        eps = (torch.randn(B, n, generator=g) * 0.999).to(dev)
        noise = torch.randn(1, B, n, generator=g).to(dev)
        th = torch.zeros(B, device=dev)

        def run(k):
            x = x0.clone()
            h.sampler_step(0, 700 - k % 3, 0, 0., x, eps, noise, th)
            return x
    else:
        _, _, cond, fea = unet_inputs(cfg, B=B, seed=11)
        cd, fd = cond.to(dev), fea.to(dev)

        def run(k):
            o = torch.empty((B, 3, cfg.tp, cfg.latent, cfg.latent), device=dev)
            h.sample(0, [999 - k % 3, 990, 980, 970], None, 0., cd, fd, o, seed=5, use_graph=True)
            return o
    refs = {}
    for k in range(3):
        refs[k] = run(k).clone()
    torch.cuda.synchronize()
    open(f'{a.sync}.{a.mode}', 'w').close()
    t0 = time.time()
    while len(glob.glob(a.sync + '.*')) < a.peers and time.time() - t0 < 120:
        time.sleep(0.05)
    t0 = time.time()
    k = bad = 0
    first = None
    while time.time() - t0 < a.seconds:
        v = run(k)
        torch.cuda.synchronize()
        if not torch.equal(v, refs[k % 3]):
            bad += 1
            if first is None:
                d = (v - refs[k % 3]).abs()
                first = {'repeat': k, 'n': int((d > 0).sum()), 'max': float(d.max())}
        k += 1
    print(json.dumps({'mode': a.mode, 'repeats': k, 'mismatches': bad, 'first': first}), flush=True)


if __name__ == '__main__':
    main()
