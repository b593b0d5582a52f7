"""Library fp16 GEMM rates (torch.matmul -> hipBLASLt) at the MotionAdaptor Tmodulator shapes,
for the f16x3 K-concatenated formulation: D (BP x M) = [Xh | Xl'] (BP x 2K) . [Wh ; Wd] (2K x M)
plus Xh (BP x K) . Wl (K x M)."""
import torch
import time

torch.backends.cuda.matmul.allow_fp16_reduced_precision_reduction = False
shapes = [('downs.2.4 / mid (L2, 8x8)', 64 * 64, 3584, 3584), ('downs.3.4 (L3, 4x4)', 64 * 16, 3584, 3584),
          ('ups.2.4 (L1, 16x16)', 64 * 256, 896, 896), ('ups.3.4 (L0, 32x32)', 64 * 1024, 896, 896)]
for name, BP, M, K in shapes:
    a2 = torch.randn(BP, 2 * K, device='cuda', dtype=torch.float16)
    b2 = torch.randn(2 * K, M, device='cuda', dtype=torch.float16)
    b1 = torch.randn(K, M, device='cuda', dtype=torch.float16)
    d = torch.empty(BP, M, device='cuda', dtype=torch.float32)
    def run():
        torch.matmul(a2, b2, out=None)
        torch.addmm(d, a2[:, :K].float() if False else a2[:, :K], b1) if False else None
    # fp16 in, fp32 out: use torch._scaled_mm? plain matmul returns fp16; time fp16-out GEMMs as a proxy
    for _ in range(3):
        torch.matmul(a2, b2); torch.matmul(a2[:, :K], b1)
    torch.cuda.synchronize()
    n = 20
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        torch.matmul(a2, b2)
    e1.record(); torch.cuda.synchronize()
    t2 = e0.elapsed_time(e1) / n
    e0.record()
    for _ in range(n):
        torch.matmul(a2[:, :K], b1)
    e1.record(); torch.cuda.synchronize()
    t1 = e0.elapsed_time(e1) / n
    fl = 2.0 * BP * M * K
    print(f'{name}: 2K GEMM {t2*1e3:.1f} us ({2*fl/t2/1e9:.0f} TF/s), K GEMM {t1*1e3:.1f} us ({fl/t1/1e9:.0f} TF/s); '
          f'f16x3 total {(t1+t2)*1e3:.1f} us = {fl/(t1+t2)/1e9:.0f} alg TF/s')
