"""Round-6: why the oracle's B = 4 step cost 9.7x its B = 1 step on the GPU box.
Times one oracle Unet forward (BAIR, the bench's cpu_baseline leg) at B = 1 / 2 / 4 and several
thread counts, and reads the cgroup's CPU throttling counters (cpu.stat) around each point."""
import importlib
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from oracle import extdm_oracle as O  # noqa: E402


def cpu_stat():
    try:
        d = dict(l.split() for l in open('/sys/fs/cgroup/cpu.stat'))
        return {k: int(v) for k, v in d.items()}
    except OSError:
        return {}


def main():
    pkg = importlib.import_module(bench.PKG)
    wrapper, arch = pkg.configs.dm_arch('bair')
    fd = pkg.FlowDiffusion(config=pkg.configs.dm_config('bair'), is_train=False, Unet3D_architecture=arch,
                           wrapper=wrapper, timesteps=1000)
    u = fd.unet.ucfg
    usd = {k: v.detach().cpu() for k, v in fd.unet.state_dict().items()}
    g = torch.Generator().manual_seed(0)
    x_cond = torch.randn(1, 3, u.tc, u.latent, u.latent, generator=g)
    fea = torch.randn(1, 256, u.tc + u.tp, u.latent // 2, u.latent // 2, generator=g)
    x = torch.randn(1, 3, u.tp, u.latent, u.latent, generator=g)
    print('visible', len(os.sched_getaffinity(0)), 'cgroup cpus', bench.cgroup_cpus(), flush=True)
    for nth in [int(v) for v in os.environ.get('THREADS', '16,12,8').split(',')]:
        torch.set_num_threads(nth)
        for B in (1, 2, 4):
            xc, fb, xb = (v.expand(B, *v.shape[1:]).contiguous() for v in (x_cond, fea, x))
            t = torch.full((B,), 500, dtype=torch.long)
            with torch.no_grad():
                O.unet_forward(usd, u.as_dict(), xb, t, xc, fb)
                s0, w0, c0 = cpu_stat(), time.perf_counter(), time.process_time()
                for _ in range(3):
                    O.unet_forward(usd, u.as_dict(), xb, t, xc, fb)
                w = (time.perf_counter() - w0) / 3
                c = (time.process_time() - c0) / 3
            s1 = cpu_stat()
            thr = {k: s1.get(k, 0) - s0.get(k, 0) for k in ('nr_periods', 'nr_throttled', 'throttled_usec')}
            print(f'threads {nth:3d} B {B}: {w:.3f} s per forward ({w / B:.3f} per clip), cpu {c:.2f} s '
                  f'({c / w:.1f} cores busy), cgroup {thr}', flush=True)


if __name__ == '__main__':
    main()
