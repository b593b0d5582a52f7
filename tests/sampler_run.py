"""Helper process of tests/test_gpu_sampler.py (not a test module): one captured-graph DDPM chain
at the metric's sample size (full BAIR u12, n = 43 008) with the per-step thresholds recorded
(extdm_record_thresholds), saved to --out. Run in its own process so that the sampler form can be
chosen by EXTDM_SAMPLER_1WG, which the library reads once per process."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def bair_handle(B):
    import importlib
    from tests.golden_inputs import CONFIGS, PKG, make_sd
    pkg = importlib.import_module(PKG)
    h = pkg._lib.Handle(CONFIGS['bair'], 1000, B, 0)
    sd = make_sd(CONFIGS['bair'])
    sd.update(pkg.schedule_buffers(1000))
    h.load_state(sd)
    h.finalize()
    return h


def graph_chain(h, B, times, cond, fea, xT, noise, dev):
    """(out, thresholds [S][B]) of one extdm_sample call on the graph path."""
    import torch
    S = len(times)
    rec = torch.full((S * B,), -1., device=dev)
    h.record_thresholds(rec)
    out = torch.empty(xT.shape, device=dev)
    try:
        h.sample(0, times, None, 0., cond.to(dev), fea.to(dev), out, x_T=xT.to(dev),
                 noise=None if noise is None else noise.to(dev).contiguous(), use_graph=True)
        torch.cuda.synchronize()
    finally:
        h.record_thresholds(None)
    return out.cpu(), rec.cpu().view(S, B)


def main():
    import torch
    from tests.golden_inputs import BAIR_CHAIN, CONFIGS, bair_chain_noise, unet_inputs
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', required=True)
    a = ap.parse_args()
    cfg, B, times = CONFIGS['bair'], BAIR_CHAIN['B'], BAIR_CHAIN['times']
    _, _, cond, fea = unet_inputs(cfg, B=B, seed=BAIR_CHAIN['seed'])
    xT, noise = bair_chain_noise(cfg, B, len(times), BAIR_CHAIN['noise_seed'])
    dev = torch.device('cuda:0')
    out, rec = graph_chain(bair_handle(B), B, times, cond, fea, xT, noise, dev)
    torch.save({'out': out, 'thresh': rec}, a.out)


if __name__ == '__main__':
    main()
