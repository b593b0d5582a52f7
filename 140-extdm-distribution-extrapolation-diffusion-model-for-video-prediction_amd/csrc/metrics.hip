// Evaluation metrics of scripts/DM/valid.py:226-243 on the device (all HBM-light,
// fp64 arithmetic like the reference's numpy float64):
//   PSNR per frame   metrics/calculate_psnr.py:6-15   20 log10(1 / sqrt(mse)), 100 if mse < 1e-10
//   SSIM per frame   metrics/calculate_ssim.py:6-41   11x11 Gaussian (sigma 1.5) window, 'valid'
//                    region (the [5:-5, 5:-5] crop of cv2.filter2D), C1 = 0.01^2, C2 = 0.03^2,
//                    mean over the map, then over the 3 channels (or the single channel)
// Frames are addressed as [N][T][C][H][W] through strides, so channel-first [B][C][T][H][W]
// sample tensors need no transpose. Per-(frame, channel, strip) partial sums are reduced in
// a fixed order by a second kernel: results are deterministic.
#include <cmath>
#include <stdexcept>

#include <mutex>
#include <stdexcept>
#include <string>

#include "kernels.h"

namespace extdm {

namespace {

constexpr int SSIM_K = 11, SSIM_R = 5;  // window, radius
constexpr int STRIP = 16;               // output rows per SSIM workgroup

__device__ __forceinline__ double block_sum_d(double v, double* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += sh[i];
  return s;
}

// one workgroup per frame: sum of squared differences over C x H x W in double
__global__ __launch_bounds__(256) void psnr_kernel(const float* __restrict__ a, const float* __restrict__ b, int T,
                                                   int C, int H, int W, long sN, long sT, long sC,
                                                   double* __restrict__ psnr) {
  __shared__ double sh[4];
  const int f = blockIdx.x, n = f / T, t = f - n * T;
  const long base = (long)n * sN + (long)t * sT;
  const int HW = H * W;
  double s = 0.0;
  for (int c = 0; c < C; ++c) {
    const float* pa = a + base + (long)c * sC;
    const float* pb = b + base + (long)c * sC;
    for (int i = threadIdx.x; i < HW; i += 256) {
      const double d = (double)pa[i] - (double)pb[i];
      s += d * d;
    }
  }
  s = block_sum_d(s, sh);
  if (threadIdx.x == 0) {
    const double mse = s / ((double)C * HW);
    psnr[f] = mse < 1e-10 ? 100.0 : 20.0 * log10(1.0 / sqrt(mse));
  }
}

// one workgroup per (frame, channel, strip of STRIP output rows of the valid region):
// the strip's STRIP + 10 input rows of both images staged in LDS, one output pixel per
// thread-iteration with the five windowed sums in double, the strip's ssim_map sum out
__global__ __launch_bounds__(256) void ssim_kernel(const float* __restrict__ a, const float* __restrict__ b, int T,
                                                   int C, int H, int W, long sN, long sT, long sC, int nstrip,
                                                   double* __restrict__ part) {
  extern __shared__ float sm[];  // [2][STRIP + 10][W]
  __shared__ double sh[4];
  __shared__ double gw[SSIM_K];
  const int f = blockIdx.x, c = blockIdx.y, strip = blockIdx.z;
  const int n = f / T, t = f - n * T;
  const long base = (long)n * sN + (long)t * sT + (long)c * sC;
  const int Ho = H - 2 * SSIM_R, Wo = W - 2 * SSIM_R;
  const int y0 = strip * STRIP;
  const int rows = min(STRIP, Ho - y0);
  const int rin = rows + 2 * SSIM_R;
  if (threadIdx.x == 0) {
    // cv2.getGaussianKernel(11, 1.5): exp(-x^2 / (2 sigma^2)), x = i - 5, normalised
    double g[SSIM_K], sum = 0.0;
    for (int i = 0; i < SSIM_K; ++i) {
      const double x = i - SSIM_R;
      g[i] = exp((-0.5 / (1.5 * 1.5)) * x * x);
      sum += g[i];
    }
    for (int i = 0; i < SSIM_K; ++i) gw[i] = g[i] * (1.0 / sum);
  }
  float* A = sm;
  float* Bs = sm + (STRIP + 2 * SSIM_R) * W;
  for (int i = threadIdx.x; i < rin * W; i += 256) {
    const int r = i / W, x = i - r * W;
    A[i] = a[base + (long)(y0 + r) * W + x];
    Bs[i] = b[base + (long)(y0 + r) * W + x];
  }
  __syncthreads();
  const double C1 = 0.01 * 0.01, C2 = 0.03 * 0.03;
  double acc = 0.0;
  for (int o = threadIdx.x; o < rows * Wo; o += 256) {
    const int y = o / Wo, x = o - y * Wo;
    double m1 = 0.0, m2 = 0.0, s11 = 0.0, s22 = 0.0, s12 = 0.0;
    for (int i = 0; i < SSIM_K; ++i) {
      const float* ra = A + (y + i) * W + x;
      const float* rb = Bs + (y + i) * W + x;
#pragma unroll
      for (int j = 0; j < SSIM_K; ++j) {
        const double w = gw[i] * gw[j];
        const double va = ra[j], vb = rb[j];
        m1 += w * va;
        m2 += w * vb;
        s11 += w * (va * va);
        s22 += w * (vb * vb);
        s12 += w * (va * vb);
      }
    }
    const double mu1_sq = m1 * m1, mu2_sq = m2 * m2, mu1_mu2 = m1 * m2;
    const double sig1 = s11 - mu1_sq, sig2 = s22 - mu2_sq, sig12 = s12 - mu1_mu2;
    acc += ((2 * mu1_mu2 + C1) * (2 * sig12 + C2)) / ((mu1_sq + mu2_sq + C1) * (sig1 + sig2 + C2));
  }
  acc = block_sum_d(acc, sh);
  if (threadIdx.x == 0) part[((long)f * C + c) * nstrip + strip] = acc;
}

// per frame: each channel's map mean, then the mean over channels (calculate_ssim.py:33-38)
__global__ void ssim_finalize_kernel(const double* __restrict__ part, int nframes, int C, int nstrip, double npix,
                                     double* __restrict__ ssim) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nframes) return;
  double tot = 0.0;
  for (int c = 0; c < C; ++c) {
    double s = 0.0;
    for (int k = 0; k < nstrip; ++k) s += part[((long)f * C + c) * nstrip + k];
    tot += s / npix;
  }
  ssim[f] = tot / C;
}

}  // namespace

size_t frame_metrics_workspace(int nframes, int C, int H) {
  const int nstrip = (H - 2 * SSIM_R + STRIP - 1) / STRIP;
  return (size_t)nframes * C * nstrip * sizeof(double);
}

void frame_metrics(hipStream_t s, const float* a, const float* b, int N, int T, int C, int H, int W, long sN, long sT,
                   long sC, double* psnr, double* ssim, double* work) {
  if (N < 1 || T < 1 || (C != 1 && C != 3))
    throw std::invalid_argument("frame_metrics: frames must have 1 or 3 channels (calculate_ssim.py:33-41)");
  if (H <= 2 * SSIM_R || W <= 2 * SSIM_R) throw std::invalid_argument("frame_metrics: frames smaller than 11x11");
  const int nf = N * T;
  const int nstrip = (H - 2 * SSIM_R + STRIP - 1) / STRIP;
  const size_t lds = (size_t)(STRIP + 2 * SSIM_R) * W * 2 * sizeof(float);
  // the device's per-workgroup LDS less the kernel's static __shared__, read once per device
  // (160 KiB on gfx950: dynamic strips up to ~150 KiB, rows up to ~1900 px)
  struct Dev { std::once_flag once; size_t max_dyn = 0; hipError_t err = hipSuccess; };
  static Dev devs[64];
  int dev = 0;
  (void)hipGetDevice(&dev);
  Dev& dv = devs[dev & 63];
  std::call_once(dv.once, [&] {
    int smem = 0;
    hipFuncAttributes fa{};
    (void)hipDeviceGetAttribute(&smem, hipDeviceAttributeMaxSharedMemoryPerBlock, dev);
    (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&ssim_kernel));
    dv.max_dyn = smem > (int)fa.sharedSizeBytes ? (size_t)smem - fa.sharedSizeBytes : 0;
    dv.err = hipFuncSetAttribute(reinterpret_cast<const void*>(&ssim_kernel),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)dv.max_dyn);
  });
  if (dv.err != hipSuccess) throw std::runtime_error("frame_metrics: cannot raise the SSIM kernel's LDS limit");
  if (lds > dv.max_dyn)
    throw std::invalid_argument("frame_metrics: rows wider than the device's LDS strip (W = " + std::to_string(W) + ")");
  hipLaunchKernelGGL(psnr_kernel, dim3(nf), dim3(256), 0, s, a, b, T, C, H, W, sN, sT, sC, psnr);
  hipLaunchKernelGGL(ssim_kernel, dim3(nf, C, nstrip), dim3(256), lds, s, a, b, T, C, H, W, sN, sT, sC, nstrip, work);
  const double npix = (double)(H - 2 * SSIM_R) * (W - 2 * SSIM_R);
  hipLaunchKernelGGL(ssim_finalize_kernel, dim3((nf + 255) / 256), dim3(256), 0, s, work, nf, C, nstrip, npix, ssim);
}

}  // namespace extdm
