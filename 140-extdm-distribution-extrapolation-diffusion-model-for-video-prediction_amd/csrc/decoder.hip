// LFAE flow-warp decoder kernels (Generator.forward_with_flow, generator.py:63-93,
// 152-206; util.py:69-149). The convolutions run on the conv kernels (halo /
// nearest-x2 im2col) with BatchNorm(eval)+ReLU folded into their epilogues; the
// kernels here are the memory-bound rest:
//   warp_blend: deform_input (flow bilinear-resized to the feature size,
//               grid_sample align_corners=True, zero padding) fused with
//               apply_optical's occlusion blend  skip*occ + prev*(1-occ)
//   affine_relu: BatchNorm(eval) + ReLU before a ResBlock2d conv
//   avgpool2:   AvgPool2d(2)
#include "kernels.h"

namespace extdm {

namespace {

// torch upsample_bilinear2d, align_corners=False, scale = in/out
__device__ __forceinline__ void lin_idx(int o, int in, int out, int& i0, int& i1, float& l0, float& l1) {
  const float scale = (float)in / (float)out;
  float src = scale * ((float)o + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = src - (float)i0;
  l0 = 1.f - l1;
}

__device__ __forceinline__ float bilerp(const float* p, int w, int y0, int y1, int x0, int x1, float ly0, float ly1,
                                        float lx0, float lx1) {
  return ly0 * (lx0 * p[y0 * w + x0] + lx1 * p[y0 * w + x1]) + ly1 * (lx0 * p[y1 * w + x0] + lx1 * p[y1 * w + x1]);
}

// One thread per output pixel of frame n = (b, t); loops over channels.
//   src: [B][C][S][S] (clip-indexed), flow: [B][2][T][fh][fw], occ: [B][1][T][fh][fw] or null,
//   prev: [N][C][S][S] or null, out: [N][C][S][S] with N = B*T.
__global__ __launch_bounds__(256) void warp_blend_kernel(float* out, long osn, long osc, const float* src, int C,
                                                         int S, const float* flow, const float* occ, int T, int fh,
                                                         int fw, const float* prev) {
  const int pix = blockIdx.x * 256 + threadIdx.x;
  const int n = blockIdx.y;
  if (pix >= S * S) return;
  const int b = n / T, t = n % T;
  const int y = pix / S, xq = pix % S;
  const float* fx = flow + (((long)b * 2 + 0) * T + t) * fh * fw;
  const float* fy = flow + (((long)b * 2 + 1) * T + t) * fh * fw;
  float gx, gy, ov = 1.f;
  if (S == fh && S == fw) {
    gx = fx[y * fw + xq];
    gy = fy[y * fw + xq];
    if (occ) ov = occ[((long)b * T + t) * fh * fw + y * fw + xq];
  } else {
    int y0, y1, x0, x1;
    float ly0, ly1, lx0, lx1;
    lin_idx(y, fh, S, y0, y1, ly0, ly1);
    lin_idx(xq, fw, S, x0, x1, lx0, lx1);
    gx = bilerp(fx, fw, y0, y1, x0, x1, ly0, ly1, lx0, lx1);
    gy = bilerp(fy, fw, y0, y1, x0, x1, ly0, ly1, lx0, lx1);
    if (occ) ov = bilerp(occ + ((long)b * T + t) * fh * fw, fw, y0, y1, x0, x1, ly0, ly1, lx0, lx1);
  }
  const float sf = (float)(S - 1) / 2.0f;
  const float ix = (gx + 1.f) * sf, iy = (gy + 1.f) * sf;
  const float ixw = floorf(ix), iyn = floorf(iy);
  const float w = ix - ixw, e = 1.f - w;
  const float nn = iy - iyn, ss = 1.f - nn;
  const int xw = (int)ixw, yn = (int)iyn;
  const float nw = ss * e, ne = ss * w, sw = nn * e, se = nn * w;
  const bool vxw = xw >= 0 && xw < S, vxe = xw + 1 >= 0 && xw + 1 < S;
  const bool vyn = yn >= 0 && yn < S, vys = yn + 1 >= 0 && yn + 1 < S;
  // the four corners' in-plane offsets (a missing corner reads offset 0 and is zeroed): the
  // loads of 8 channels are issued unconditionally before any arithmetic (one channel at a
  // time left each gather's latency exposed: 8.3 ms for 2 x 2.1 GB at 256 x 256, C = 64)
  const bool ok[4] = {vxw && vyn, vxe && vyn, vxw && vys, vxe && vys};
  const int o4[4] = {ok[0] ? yn * S + xw : 0, ok[1] ? yn * S + xw + 1 : 0, ok[2] ? (yn + 1) * S + xw : 0,
                     ok[3] ? (yn + 1) * S + xw + 1 : 0};
  const long plane = (long)S * S;
  const float* sb = src + (long)b * C * plane;
  for (int c0 = 0; c0 < C; c0 += 8) {
    float g[8][4], pv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = c0 + u;
      if (c >= C) break;  // uniform
      const float* p = sb + (long)c * plane;
#pragma unroll
      for (int k = 0; k < 4; ++k) g[u][k] = p[o4[k]];
      pv[u] = (occ && prev) ? prev[(long)n * osn + (long)c * osc + pix] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = c0 + u;
      if (c >= C) break;
      const float vnw = ok[0] ? g[u][0] : 0.f, vne = ok[1] ? g[u][1] : 0.f;
      const float vsw = ok[2] ? g[u][2] : 0.f, vse = ok[3] ? g[u][3] : 0.f;
      float v = vnw * nw + vne * ne + vsw * sw + vse * se;
      if (occ) {
        if (prev) v = v * ov + pv[u] * (1.f - ov);
        else v = v * ov;
      }
      out[(long)n * osn + (long)c * osc + pix] = v;
    }
  }
}

__global__ __launch_bounds__(256) void affine_relu_kernel(float* out, const float* in, const float* a,
                                                          const float* bsh, int C, int HW, long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int c = (int)((i / HW) % C);
  const float v = in[i] * a[c] + bsh[c];
  out[i] = v > 0.f ? v : 0.f;
}

__global__ __launch_bounds__(256) void avgpool2_kernel(float* out, const float* in, int Ho, int Wo, long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % Wo);
  const long r = i / Wo;
  const int y = (int)(r % Ho);
  const long pc = r / Ho;  // plane
  const float* p = in + pc * (long)(4 * Ho * Wo) + (long)(2 * y) * (2 * Wo) + 2 * x;
  out[i] = (p[0] + p[1] + p[2 * Wo] + p[2 * Wo + 1]) / 4.f;
}

}  // namespace

void warp_blend(hipStream_t s, float* out, const float* src, int N, int C, int S, const float* flow,
                const float* occ, int T, int fh, int fw, const float* prev) {
  hipLaunchKernelGGL(warp_blend_kernel, dim3((S * S + 255) / 256, N), dim3(256), 0, s, out, (long)C * S * S,
                     (long)S * S, src, C, S, flow, occ, T, fh, fw, prev);
}

void affine_relu(hipStream_t s, float* out, const float* in, const float* a, const float* b, int N, int C, int HW) {
  const long total = (long)N * C * HW;
  hipLaunchKernelGGL(affine_relu_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, out, in, a, b, C,
                     HW, total);
}

void avgpool2(hipStream_t s, float* out, const float* in, int planes, int Ho, int Wo) {
  const long total = (long)planes * Ho * Wo;
  hipLaunchKernelGGL(avgpool2_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, out, in, Ho, Wo,
                     total);
}

}  // namespace extdm
