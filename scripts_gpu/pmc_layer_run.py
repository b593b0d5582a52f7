"""One bench layer of a BASELINE workload's denoiser in isolation for the PMC passes (rocprofv3 --pmc
FETCH_SIZE / WRITE_SIZE): `iters` launches exactly as the forward issues them (extdm_bench_layer).
Prints `KERNEL:<template>` (the attention layers' launched template, else the bench.py LAYERS name).
Usage: pmc_layer_run.py CONFIG LAYER [ITERS]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import cfg_handle  # noqa: E402

cfg_name, layer = sys.argv[1], int(sys.argv[2])
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
h, B, prec = cfg_handle.make(cfg_name)
ms, flops = h.bench_layer(B, layer, iters)
k = h.bench_layer_kernel(layer) or next((e[2] for e in cfg_handle.bench.NativeWorkload.LAYERS if e[0] == layer), '') or ''
print(f'layer {layer} B={B} {prec}: {ms:.3f} ms/launch, {flops / ms / 1e9:.1f} TFLOP/s')
print(f'KERNEL:{k}')
print(f'WIDE:{int(cfg_handle.bench.NativeWorkload.wide_reads(layer, k))}')
print(f'PREC:{prec} B:{B}')
