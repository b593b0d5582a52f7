// Normalisation and layout kernels of the sampling path (all HBM-bound):
//   GroupNorm(8) + FiLM + SiLU (+ residual)      Block / ResnetBlock, u12:162-203
//   channel LayerNorm (gamma only, biased var)     LayerNorm/PreNorm,  u12:138-158
//   fused temporal-attention prologue              u12:306-327, 915
//   maxpool (1,2,2), bilinear resize, strided copy u12:811, 1035-1037
//   MotionAdaptor statistics / normalisation       u12:670-691
// Reductions accumulate in double so the fp32 outputs track the reference's
// fp32 reductions to rounding.
#include "kernels.h"
#include <stdexcept>

namespace extdm {

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Block-wide sum of two doubles (blockDim = 256).
__device__ __forceinline__ void block_sum2(double& a, double& b, double* sh) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) { sh[w] = a; sh[4 + w] = b; }
  __syncthreads();
  a = sh[0] + sh[1] + sh[2] + sh[3];
  b = sh[4] + sh[5] + sh[6] + sh[7];
}

struct V5 {
  const float* p; long sb, sc, st; int C, T, HW;
};

__device__ __forceinline__ long off5(long sb, long sc, long st, int b, int c, int t, int hw) {
  return (long)b * sb + (long)c * sc + (long)t * st + hw;
}

// ---------------- GroupNorm ----------------
__global__ __launch_bounds__(256) void gn_stats_kernel(const float* __restrict__ x, long sb, long sc, int Cg,
                                                       int G, long L, int split, double* partials) {
  const int bg = blockIdx.y;
  const int b = bg / G, g = bg % G;
  const float* base = x + (long)b * sb + (long)g * Cg * sc;
  const long chunk = (L + split - 1) / split;
  const long e0 = blockIdx.x * chunk;
  const long e1 = e0 + chunk < L ? e0 + chunk : L;
  double s = 0.0, ss = 0.0;
  for (long e = e0 + threadIdx.x; e < e1; e += 256) {
    const double v = base[e];
    s += v;
    ss += v * v;
  }
  __shared__ double sh[8];
  block_sum2(s, ss, sh);
  if (threadIdx.x == 0) {
    partials[((long)bg * split + blockIdx.x) * 2] = s;
    partials[((long)bg * split + blockIdx.x) * 2 + 1] = ss;
  }
}

// Vectorised statistics: float4 loads, four of them in flight per thread before any
// accumulation (one 4-B load per thread per iteration left HBM latency exposed: 0.5 TB/s).
// Requires a 16-B aligned, contiguous group and L % 4 == 0; `chunk` is a multiple of 4096.
__global__ __launch_bounds__(256) void gn_stats4_kernel(const float* __restrict__ x, long sb, long sc, int Cg,
                                                        int G, long L, int split, long chunk, double* partials) {
  const int bg = blockIdx.y;
  const int b = bg / G, g = bg % G;
  const float4* base = reinterpret_cast<const float4*>(x + (long)b * sb + (long)g * Cg * sc);
  const long i0 = blockIdx.x * chunk / 4;
  const long i1 = (blockIdx.x * chunk + chunk < L ? blockIdx.x * chunk + chunk : L) / 4;
  double s = 0.0, ss = 0.0;
  long i = i0 + threadIdx.x;
  for (; i + 768 < i1; i += 1024) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = base[i + u * 256];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double a = v[u].x, bb = v[u].y, c = v[u].z, d = v[u].w;
      s += a; ss += a * a;
      s += bb; ss += bb * bb;
      s += c; ss += c * c;
      s += d; ss += d * d;
    }
  }
  for (; i < i1; i += 256) {
    const float4 v = base[i];
    const double a = v.x, bb = v.y, c = v.z, d = v.w;
    s += a; ss += a * a;
    s += bb; ss += bb * bb;
    s += c; ss += c * c;
    s += d; ss += d * d;
  }
  __shared__ double sh[8];
  block_sum2(s, ss, sh);
  if (threadIdx.x == 0) {
    partials[((long)bg * split + blockIdx.x) * 2] = s;
    partials[((long)bg * split + blockIdx.x) * 2 + 1] = ss;
  }
}

__global__ __launch_bounds__(256) void gn_apply_kernel(const float* __restrict__ x, long sb, long sc,
                                                       float* out, long osb, long osc, long ost, int C, int Cg,
                                                       int G, int T, int HW, const float2* __restrict__ gst,
                                                       const float* gamma, const float* beta, const float* film,
                                                       int film_row, int film_nt, const int* t_batch,
                                                       const float* res, long rsb, long rsc, long rst,
                                                       int split2) {
  const int bg = blockIdx.y;
  const int b = bg / G, g = bg % G;
  const float mean = gst[bg].x, rstd = gst[bg].y;
  const long L = (long)Cg * T * HW;
  const long chunk = (L + split2 - 1) / split2;
  const long e0 = blockIdx.x * chunk;
  const long e1 = e0 + chunk < L ? e0 + chunk : L;
  const float* base = x + (long)b * sb + (long)g * Cg * sc;
  int tb = film ? t_batch[b] : 0;
  for (long e = e0 + threadIdx.x; e < e1; e += 256) {
    const int cl = (int)(e / ((long)T * HW));
    const int rem = (int)(e - (long)cl * T * HW);
    const int t = rem / HW, hw = rem - t * HW;
    const int c = g * Cg + cl;
    const float sc_ = rstd * gamma[c];
    const float bi = beta[c] - mean * sc_;
    float v = base[(long)cl * sc + (long)t * HW + hw] * sc_ + bi;
    if (film) {
      const float scale = film[(long)(film_row + c) * film_nt + tb];
      const float shift = film[(long)(film_row + C + c) * film_nt + tb];
      v = v * (scale + 1.f) + shift;
    }
    v = v / (1.f + expf(-v));
    if (res) v += res[off5(rsb, rsc, rst, b, c, t, hw)];
    out[off5(osb, osc, ost, b, c, t, hw)] = v;
  }
}

// gn_apply_kernel on 4 pixels per thread with 32-bit indexing within one (b, g): the
// host checks HW % 4 == 0 and 16-byte aligned rows of x, out and res.
__global__ __launch_bounds__(256) void gn_apply4_kernel(const float* __restrict__ x, long sb, long sc,
                                                        float* out, long osb, long osc, long ost, int C, int Cg,
                                                        int G, int T, int HW, const float2* __restrict__ gst,
                                                        const float* gamma, const float* beta, const float* film,
                                                        int film_row, int film_nt, const int* t_batch,
                                                        const float* res, long rsb, long rsc, long rst,
                                                        int split2) {
  const int bg = blockIdx.y;
  const int b = bg / G, g = bg % G;
  const float mean = gst[bg].x, rstd = gst[bg].y;
  const int HW4 = HW >> 2, THW4 = T * HW4;
  const int L4 = Cg * THW4;
  const int chunk = (L4 + split2 - 1) / split2;
  const int e0 = blockIdx.x * chunk;
  const int e1 = e0 + chunk < L4 ? e0 + chunk : L4;
  const float* base = x + (long)b * sb + (long)g * Cg * sc;
  const int tb = film ? t_batch[b] : 0;
  // Four float4 per thread per iteration: all loads issued before any math.
  for (int e = e0 + threadIdx.x; e < e1; e += 1024) {
    float4 xv[4], rv[4];
    int cc[4], tt[4], hh[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int eu = e + u * 256 < e1 ? e + u * 256 : e;
      const int cl = eu / THW4;
      const int rem = eu - cl * THW4;
      tt[u] = rem / HW4;
      hh[u] = (rem - tt[u] * HW4) * 4;
      cc[u] = g * Cg + cl;
      xv[u] = *reinterpret_cast<const float4*>(base + (long)cl * sc + (long)tt[u] * HW + hh[u]);
      rv[u] = res ? *reinterpret_cast<const float4*>(res + off5(rsb, rsc, rst, b, cc[u], tt[u], hh[u]))
                  : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (e + u * 256 >= e1) break;
      const int c = cc[u];
      const float sc_ = rstd * gamma[c];
      const float bi = beta[c] - mean * sc_;
      float fsc = 1.f, fsh = 0.f;
      if (film) {
        fsc = film[(long)(film_row + c) * film_nt + tb] + 1.f;
        fsh = film[(long)(film_row + C + c) * film_nt + tb];
      }
      float v[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
      const float r[4] = {rv[u].x, rv[u].y, rv[u].z, rv[u].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float w = v[k] * sc_ + bi;
        if (film) w = w * fsc + fsh;
        w = w / (1.f + expf(-w));
        v[k] = w + r[k];
      }
      *reinterpret_cast<float4*>(out + off5(osb, osc, ost, b, c, tt[u], hh[u])) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

// gn_apply4_kernel for large planes: one (b, c) channel per grid.y, so the channel's
// scale / shift / FiLM are block constants and the element index needs no division
// (frames contiguous in x, out and res: st == H*W). Same arithmetic per element.
__global__ __launch_bounds__(256) void gn_apply_plane_kernel(const float* __restrict__ x, long sb, long sc,
                                                             float* out, long osb, long osc, int C, int Cg, int G,
                                                             int THW4, const float2* __restrict__ gst,
                                                             const float* gamma, const float* beta,
                                                             const float* film, int film_row, int film_nt,
                                                             const int* t_batch, const float* res, long rsb,
                                                             long rsc, int per) {
  const int bc = blockIdx.y;
  const int b = bc / C, c = bc - b * C;
  const int bg = b * G + c / Cg;
  const float mean = gst[bg].x, rstd = gst[bg].y;
  const float sc_ = rstd * gamma[c];
  const float bi = beta[c] - mean * sc_;
  float fsc = 1.f, fsh = 0.f;
  if (film) {
    const int tb = t_batch[b];
    fsc = film[(long)(film_row + c) * film_nt + tb] + 1.f;
    fsh = film[(long)(film_row + C + c) * film_nt + tb];
  }
  const float4* xp = reinterpret_cast<const float4*>(x + (long)b * sb + (long)c * sc);
  float4* op = reinterpret_cast<float4*>(out + (long)b * osb + (long)c * osc);
  const float4* rp = res ? reinterpret_cast<const float4*>(res + (long)b * rsb + (long)c * rsc) : nullptr;
  const int i0 = blockIdx.x * per;
  const int i1 = i0 + per < THW4 ? i0 + per : THW4;
  for (int i = i0 + threadIdx.x; i < i1; i += 1024) {
    float4 xv[4], rv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int iu = i + u * 256 < i1 ? i + u * 256 : i;
      xv[u] = xp[iu];
      rv[u] = rp ? rp[iu] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (i + u * 256 >= i1) break;
      float v[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
      const float r[4] = {rv[u].x, rv[u].y, rv[u].z, rv[u].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float w = v[k] * sc_ + bi;
        if (film) w = w * fsc + fsh;
        w = w / (1.f + expf(-w));
        v[k] = w + r[k];
      }
      op[i + u * 256] = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

// (mean, rstd) per (b, group) from the statistics partials: one wave per (b, group),
// lane i holds slot i, a fixed xor tree in double (deterministic). Computed once here
// rather than by every workgroup of the apply kernels (a serial 64-load chain each).
__global__ __launch_bounds__(64) void gn_finalize_kernel(const double* __restrict__ partials, int split, double n,
                                                         float2* __restrict__ gst) {
  const int bg = blockIdx.x, l = threadIdx.x;
  double s = l < split ? partials[((long)bg * split + l) * 2] : 0.0;
  double ss = l < split ? partials[((long)bg * split + l) * 2 + 1] : 0.0;
  s = wave_sum(s);
  ss = wave_sum(ss);
  if (l == 0) {
    const double mean = s / n;
    double var = ss / n - mean * mean;
    if (var < 0) var = 0;
    gst[bg] = make_float2((float)mean, 1.0f / sqrtf((float)var + 1e-5f));
  }
}

// (scale, shift) per (b, c) of a GroupNorm without FiLM: the per-element arithmetic of
// gn_apply_plane_kernel is then w = v * scale + shift
__global__ __launch_bounds__(256) void gn_affine_kernel(const float2* __restrict__ gst, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, int C, int Cg, int G,
                                                        float2* __restrict__ tab) {
  const int b = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += 256) {
    const float2 mr = gst[b * G + c / Cg];
    const float sc_ = mr.y * gamma[c];
    tab[(long)b * C + c] = make_float2(sc_, beta[c] - mr.x * sc_);
  }
}

// GroupNorm + FiLM + SiLU written as the pre-split f16x3 operand of the next 3x3 conv
// (X3Op, kernels.h): one (sample b, 16-channel group cg) per grid.(y, z), one padded
// position of the sample's T frames per thread (small planes share a workgroup); the
// zero ring is written too. Same per-element arithmetic as gn_apply_plane_kernel, then
// hi = fp16(w), lo = fp16(w - hi) of the opaque w.
__global__ __launch_bounds__(256) void gn_apply_x3op_kernel(const float* __restrict__ x, long sb, long sc, long st,
                                                            _Float16* __restrict__ op, long cg_stride, long hl_stride,
                                                            int C, int Cg, int G, int T, int H, int W, int pad,
                                                            const float2* __restrict__ gst, const float* gamma,
                                                            const float* beta, const float* film, int film_row,
                                                            int film_nt, const int* t_batch, int* range_flag) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  const int b = blockIdx.y, cg = blockIdx.z;
  __shared__ float csc[16], cbi[16], cfs[16], cfh[16];
  if (threadIdx.x < 16) {
    const int c = cg * 16 + threadIdx.x;
    const int bg = b * G + c / Cg;
    const float mean = gst[bg].x, rstd = gst[bg].y;
    const float sc_ = rstd * gamma[c];
    csc[threadIdx.x] = sc_;
    cbi[threadIdx.x] = beta[c] - mean * sc_;
    float fsc = 1.f, fsh = 0.f;
    if (film) {
      const int tb = t_batch[b];
      fsc = film[(long)(film_row + c) * film_nt + tb] + 1.f;
      fsh = film[(long)(film_row + C + c) * film_nt + tb];
    }
    cfs[threadIdx.x] = fsc;
    cfh[threadIdx.x] = fsh;
  }
  __syncthreads();
  const int Hp = H + 2 * pad, Wp = W + 2 * pad;
  const int n = T * Hp * Wp;  // (frame, padded position) of sample b
  const long c8s = hl_stride >> 1;  // planes (hl, c8): one 16-B record per position
  _Float16* const ob = op + (long)cg * cg_stride + (long)b * n * 8;
  const float* const xb = x + (long)b * sb + (long)(cg * 16) * sc;
  // PPT positions per thread, 256 apart (coalesced), all loads issued first (PPT = 4
  // measured 14 % slower than 1 over a DDIM-20 run at B = 64)
  constexpr int PPT = 1;
  float v[PPT][16];
  bool in[PPT];
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const int tpos = (blockIdx.x * PPT + u) * 256 + threadIdx.x;
    const int tp = tpos < n ? tpos : 0;
    const int t = tp / (Hp * Wp), pos = tp - t * (Hp * Wp);
    const int yy = pos / Wp, xx = pos - yy * Wp;
    const int iy = yy - pad, ix = xx - pad;
    in[u] = iy >= 0 && iy < H && ix >= 0 && ix < W;
    const float* xp = xb + (long)t * st + (in[u] ? iy * W + ix : 0);
#pragma unroll
    for (int e = 0; e < 16; ++e) v[u][e] = xp[(long)e * sc];
  }
  int bad = 0;
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const int tpos = (blockIdx.x * PPT + u) * 256 + threadIdx.x;
    h8 hi[2], lo[2];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      float w = v[u][e] * csc[e] + cbi[e];
      if (film) w = w * cfs[e] + cfh[e];
      w = w / (1.f + expf(-w));
      w = split_src(in[u] ? w : 0.f);
      bad |= fabsf(w) >= 65504.f;
      const _Float16 a = (_Float16)w;
      hi[e >> 3][e & 7] = a;
      lo[e >> 3][e & 7] = (_Float16)((w - (float)a) * X3_LO_UP);  // scaled lo (split2s, kernels.h)
    }
    if (tpos < n) {
      _Float16* d = ob + (long)tpos * 8;
      *reinterpret_cast<h8*>(d) = hi[0];
      *reinterpret_cast<h8*>(d + c8s) = hi[1];
      *reinterpret_cast<h8*>(d + hl_stride) = lo[0];
      *reinterpret_cast<h8*>(d + hl_stride + c8s) = lo[1];
    }
  }
  if (bad) atomicOr(range_flag, 1);
}

// ---------------- channel LayerNorm ----------------
__device__ __forceinline__ float ld2(const float* p0, long b0, long c0s, int C0, const float* p1, long b1,
                                     long c1s, int c) {
  return c < C0 ? p0[b0 + (long)c * c0s] : p1[b1 + (long)(c - C0) * c1s];
}

// The same LayerNorm on float4 pixel quads (H*W % 4 == 0, 16-B aligned rows): a block is 32
// quads x 8 channel groups, a half-wave reads 512 contiguous bytes per channel, and the
// channel loop keeps four loads in flight. Per pixel the same summation order as
// channel_ln_kernel (each group's channels in sequence, then the groups in order).
__global__ __launch_bounds__(256) void channel_ln4_kernel(float* out, long osb, long osc, long ost,
                                                          const float* p0, long sb0, long sc0, long st0, int C0,
                                                          const float* p1, long sb1, long sc1, long st1, int C,
                                                          int T, int HW, int B, const float* gamma) {
  __shared__ double red[8][32][4], red2[8][32][4];
  __shared__ float stat[2][32][4];
  const int q = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const long nq = (long)B * T * HW / 4;
  const long idx = (long)blockIdx.x * 32 + q;
  const bool ok = idx < nq;
  const long pix = (ok ? idx : 0) * 4;
  const int hw = (int)(pix % HW);
  const int t = (int)((pix / HW) % T);
  const int b = (int)(pix / ((long)HW * T));
  const long b0 = (long)b * sb0 + (long)t * st0 + hw;
  const long b1 = (long)b * sb1 + (long)t * st1 + hw;
  auto ld4 = [&](int c) __attribute__((always_inline)) {
    return c < C0 ? *reinterpret_cast<const float4*>(p0 + b0 + (long)c * sc0)
                  : *reinterpret_cast<const float4*>(p1 + b1 + (long)(c - C0) * sc1);
  };
  double s[4] = {0.0, 0.0, 0.0, 0.0}, ss[4] = {0.0, 0.0, 0.0, 0.0};
  if (ok) {
#pragma unroll 4
    for (int c = grp; c < C; c += 8) {
      const float4 v = ld4(c);
      const double d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) { s[k] += d[k]; ss[k] += d[k] * d[k]; }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) { red[grp][q][k] = s[k]; red2[grp][q][k] = ss[k]; }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int qq = threadIdx.x >> 2, k = threadIdx.x & 3;
    double tt = 0.0, t2 = 0.0;
    for (int i = 0; i < 8; ++i) { tt += red[i][qq][k]; t2 += red2[i][qq][k]; }
    const double mean = tt / C;
    double var = t2 / C - mean * mean;
    if (var < 0) var = 0;
    stat[0][qq][k] = (float)mean;
    stat[1][qq][k] = sqrtf((float)var + 1e-5f);
  }
  __syncthreads();
  if (!ok) return;
  float m[4], den[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) { m[k] = stat[0][q][k]; den[k] = stat[1][q][k]; }
  const long ob = (long)b * osb + (long)t * ost + hw;
#pragma unroll 4
  for (int c = grp; c < C; c += 8) {
    const float4 v = ld4(c);
    const float g = gamma[c];
    float4 o;
    o.x = (v.x - m[0]) / den[0] * g;
    o.y = (v.y - m[1]) / den[1] * g;
    o.z = (v.z - m[2]) / den[2] * g;
    o.w = (v.w - m[3]) / den[3] * g;
    *reinterpret_cast<float4*>(out + ob + (long)c * osc) = o;
  }
}

// 32 pixels per block, 8 channel groups per pixel (thread = (pixel, group)), so a
// LayerNorm over hundreds of channels at few pixels still fills the machine.
__global__ __launch_bounds__(256) void channel_ln_kernel(float* out, long osb, long osc, long ost,
                                                         const float* p0, long sb0, long sc0, long st0, int C0,
                                                         const float* p1, long sb1, long sc1, long st1, int C,
                                                         int T, int HW, int B, const float* gamma) {
  __shared__ double red[8][33], red2[8][33];
  __shared__ float stat[2][32];
  const int px = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const long idx = (long)blockIdx.x * 32 + px;
  const long npix = (long)B * T * HW;
  const bool ok = idx < npix;
  const long id2 = ok ? idx : 0;
  const int hw = (int)(id2 % HW);
  const int t = (int)((id2 / HW) % T);
  const int b = (int)(id2 / ((long)HW * T));
  const long b0 = (long)b * sb0 + (long)t * st0 + hw;
  const long b1 = (long)b * sb1 + (long)t * st1 + hw;
  // one pass: sum and sum of squares in double (E[x^2] - mean^2 in double keeps the
  // fp32 result of the two-pass form; a second read pass cost a quarter of the traffic)
  double s = 0.0, ss = 0.0;
  if (ok)
    for (int c = grp; c < C; c += 8) {
      const double v = ld2(p0, b0, sc0, C0, p1, b1, sc1, c);
      s += v;
      ss += v * v;
    }
  red[grp][px] = s;
  red2[grp][px] = ss;
  __syncthreads();
  if (threadIdx.x < 32) {
    double tt = 0.0, t2 = 0.0;
    for (int i = 0; i < 8; ++i) { tt += red[i][threadIdx.x]; t2 += red2[i][threadIdx.x]; }
    const double mean = tt / C;
    double var = t2 / C - mean * mean;
    if (var < 0) var = 0;
    stat[0][threadIdx.x] = (float)mean;
    stat[1][threadIdx.x] = sqrtf((float)var + 1e-5f);
  }
  __syncthreads();
  if (!ok) return;
  const float m = stat[0][px], den = stat[1][px];
  const long ob = (long)b * osb + (long)t * ost + hw;
  for (int c = grp; c < C; c += 8) {
    const float x = ld2(p0, b0, sc0, C0, p1, b1, sc1, c);
    out[ob + (long)c * osc] = (x - m) / den * gamma[c];
  }
}

__global__ __launch_bounds__(256) void temporal_prologue_kernel(const float* x, long sb, long sc, long st, int C,
                                                                int T, int HW, int B, const float* gamma,
                                                                const float* lw, const float* lb, float* z,
                                                                long zsb, long zsc, long zst, float* r, long rsb,
                                                                long rsc, long rst) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long npix = (long)B * T * HW;
  if (idx >= npix) return;
  const int hw = (int)(idx % HW);
  const int t = (int)((idx / HW) % T);
  const int b = (int)(idx / ((long)HW * T));
  const float* xp = x + (long)b * sb + (long)t * st + hw;
  double s = 0.0;
  for (int c = 0; c < C; ++c) s += xp[(long)c * sc];
  const float m = (float)(s / C);
  double v2 = 0.0;
  for (int c = 0; c < C; ++c) {
    const double d = (double)xp[(long)c * sc] - (double)(s / C);
    v2 += d * d;
  }
  const float den = sqrtf((float)(v2 / C) + 1e-5f);
  // y = chanLN(x) * gamma ; moments of y
  double sy = 0.0;
  for (int c = 0; c < C; ++c) sy += (double)((xp[(long)c * sc] - m) / den * gamma[c]);
  const double my = sy / C;
  double vy = 0.0;
  for (int c = 0; c < C; ++c) {
    const double d = (double)((xp[(long)c * sc] - m) / den * gamma[c]) - my;
    vy += d * d;
  }
  const float m2 = (float)my;
  const float rstd2 = 1.0f / sqrtf((float)(vy / C) + 1e-5f);
  float* zp = z + (long)b * zsb + (long)t * zst + hw;
  float* rp = r + (long)b * rsb + (long)t * rst + hw;
  for (int c = 0; c < C; ++c) {
    const float xv = xp[(long)c * sc];
    const float y = (xv - m) / den * gamma[c];
    zp[(long)c * zsc] = (y - m2) * rstd2 * lw[c] + lb[c];
    rp[(long)c * rsc] = xv + y;
  }
}

// The same prologue with a pixel's channels split over G thread groups (PX pixels per workgroup;
// each pass's per-group double partials summed in group order): for the deep levels, where one
// thread per pixel left a launch with a few workgroups walking every channel five times
// (Cityscapes: 448 pixels, two workgroups, 212 us per launch).
template <int PX, int G>
__global__ __launch_bounds__(PX * G) void temporal_prologue_grp_kernel(const float* x, long sb, long sc, long st, int C,
                                                                       int T, int HW, int B, const float* gamma,
                                                                       const float* lw, const float* lb, float* z,
                                                                       long zsb, long zsc, long zst, float* r, long rsb,
                                                                       long rsc, long rst) {
  __shared__ double red[G][PX];
  const int px = threadIdx.x % PX, grp = threadIdx.x / PX;
  const long idx = (long)blockIdx.x * PX + px;
  const long npix = (long)B * T * HW;
  const bool ok = idx < npix;
  const long id2 = ok ? idx : 0;
  const int hw = (int)(id2 % HW);
  const int t = (int)((id2 / HW) % T);
  const int b = (int)(id2 / ((long)HW * T));
  const float* xp = x + (long)b * sb + (long)t * st + hw;
  // the pixel's total of the groups' partials, in group order (every thread of the pixel)
  auto total = [&](double v) {
    red[grp][px] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < G; ++i) s += red[i][px];
    __syncthreads();
    return s;
  };
  double s = 0.0;
  if (ok)
    for (int c = grp; c < C; c += G) s += xp[(long)c * sc];
  const double mean = total(s) / C;
  const float m = (float)mean;
  double v2 = 0.0;
  if (ok)
    for (int c = grp; c < C; c += G) {
      const double d = (double)xp[(long)c * sc] - mean;
      v2 += d * d;
    }
  const float den = sqrtf((float)(total(v2) / C) + 1e-5f);
  // y = chanLN(x) * gamma ; moments of y
  double sy = 0.0;
  if (ok)
    for (int c = grp; c < C; c += G) sy += (double)((xp[(long)c * sc] - m) / den * gamma[c]);
  const double my = total(sy) / C;
  double vy = 0.0;
  if (ok)
    for (int c = grp; c < C; c += G) {
      const double d = (double)((xp[(long)c * sc] - m) / den * gamma[c]) - my;
      vy += d * d;
    }
  const float rstd2 = 1.0f / sqrtf((float)(total(vy) / C) + 1e-5f);
  if (!ok) return;
  const float m2 = (float)my;
  float* zp = z + (long)b * zsb + (long)t * zst + hw;
  float* rp = r + (long)b * rsb + (long)t * rst + hw;
  for (int c = grp; c < C; c += G) {
    const float xv = xp[(long)c * sc];
    const float y = (xv - m) / den * gamma[c];
    zp[(long)c * zsc] = (y - m2) * rstd2 * lw[c] + lb[c];
    rp[(long)c * rsc] = xv + y;
  }
}

// ---------------- layout / resampling ----------------
__global__ __launch_bounds__(256) void copy_kernel(float* d, long dsb, long dsc, long dst_, const float* s,
                                                   long ssb, long ssc, long sst, int C, int T, int HW, long total) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int hw = (int)(idx % HW);
  long r = idx / HW;
  const int t = (int)(r % T); r /= T;
  const int c = (int)(r % C);
  const int b = (int)(r / C);
  d[off5(dsb, dsc, dst_, b, c, t, hw)] = s[off5(ssb, ssc, sst, b, c, t, hw)];
}

__global__ __launch_bounds__(256) void maxpool_kernel(float* d, long dsb, long dsc, long dst_, const float* s,
                                                      long ssb, long ssc, long sst, int C, int T, int Ho, int Wo,
                                                      int Wi, long total) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int x = (int)(idx % Wo);
  long r = idx / Wo;
  const int y = (int)(r % Ho); r /= Ho;
  const int t = (int)(r % T); r /= T;
  const int c = (int)(r % C);
  const int b = (int)(r / C);
  const float* p = s + off5(ssb, ssc, sst, b, c, t, 0) + (long)(2 * y) * Wi + 2 * x;
  const float v = fmaxf(fmaxf(p[0], p[1]), fmaxf(p[Wi], p[Wi + 1]));
  d[off5(dsb, dsc, dst_, b, c, t, y * Wo + x)] = v;
}

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

__global__ __launch_bounds__(256) void bilinear_kernel(float* d, long dsb, long dsc, long dst_, const float* a,
                                                       long asb, long asc, long ast, const float* bb, long bsb,
                                                       long bsc, long bst, int tsplit, int C, int T, int Ho,
                                                       int Wo, int Hi, int Wi, long total) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int x = (int)(idx % Wo);
  long r = idx / Wo;
  const int y = (int)(r % Ho); r /= Ho;
  const int t = (int)(r % T); r /= T;
  const int c = (int)(r % C);
  const int b = (int)(r / C);
  const float* p = t < tsplit ? a + off5(asb, asc, ast, b, c, t, 0) : bb + off5(bsb, bsc, bst, b, c, t - tsplit, 0);
  int y0, y1, x0, x1;
  float ly0, ly1, lx0, lx1;
  lin_idx(y, Hi, Ho, y0, y1, ly0, ly1);
  lin_idx(x, Wi, Wo, x0, x1, lx0, lx1);
  const float v = ly0 * (lx0 * p[y0 * Wi + x0] + lx1 * p[y0 * Wi + x1]) +
                  ly1 * (lx0 * p[y1 * Wi + x0] + lx1 * p[y1 * Wi + x1]);
  d[off5(dsb, dsc, dst_, b, c, t, y * Wo + x)] = v;
}

// Four consecutive output pixels per thread, one (b, c) per grid.z and one frame per
// grid.y: 32-bit index math only (the flat-index kernel's 64-bit div/mod chain ran at
// ~1.3 TB/s). Requires Wo % 4 == 0; float4 stores when the destination rows are aligned.
__global__ __launch_bounds__(256) void bilinear4_kernel(float* d, long dsb, long dsc, long dst_, const float* a,
                                                        long asb, long asc, long ast, const float* bb, long bsb,
                                                        long bsc, long bst, int tsplit, int C, int Ho, int Wo,
                                                        int Hi, int Wi, int vec) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (4 * q >= Ho * Wo) return;
  const int t = blockIdx.y;
  const int b = blockIdx.z / C, c = blockIdx.z % C;
  const int y = 4 * q / Wo, x = 4 * q - y * Wo;
  const float* p = t < tsplit ? a + off5(asb, asc, ast, b, c, t, 0) : bb + off5(bsb, bsc, bst, b, c, t - tsplit, 0);
  int y0, y1;
  float ly0, ly1;
  lin_idx(y, Hi, Ho, y0, y1, ly0, ly1);
  const float* r0 = p + y0 * Wi;
  const float* r1 = p + y1 * Wi;
  float v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int x0, x1;
    float lx0, lx1;
    lin_idx(x + k, Wi, Wo, x0, x1, lx0, lx1);
    v[k] = ly0 * (lx0 * r0[x0] + lx1 * r0[x1]) + ly1 * (lx0 * r1[x0] + lx1 * r1[x1]);
  }
  float* o = d + off5(dsb, dsc, dst_, b, c, t, y * Wo + x);
  if (vec) {
    *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = v[k];
  }
}

// Small input planes (Hi*Wi <= 1024): BPLS (b, c) planes of one frame per block are
// staged into LDS with coalesced loads, the 2-D interpolation gathers from LDS and each
// thread stores float4 runs. Same lin_idx weights and expression as bilinear_kernel.
constexpr int BPLS = 8;
__global__ __launch_bounds__(256) void bilinear_lds_kernel(float* d, long dsb, long dsc, long dst_, const float* a,
                                                           long asb, long asc, long ast, const float* bb, long bsb,
                                                           long bsc, long bst, int tsplit, int C, int nbc, int Ho,
                                                           int Wo, int Hi, int Wi, int vec) {
  __shared__ float pl[BPLS * 1024];
  const int t = blockIdx.y;
  const int bc0 = blockIdx.x * BPLS;
  const int np = nbc - bc0 < BPLS ? nbc - bc0 : BPLS;
  const int HWi = Hi * Wi;
  for (int k = threadIdx.x; k < np * HWi; k += 256) {
    const int j = k / HWi, e = k - j * HWi;
    const int bc = bc0 + j;
    const int b = bc / C, c = bc - b * C;
    const float* p = t < tsplit ? a + off5(asb, asc, ast, b, c, t, 0) : bb + off5(bsb, bsc, bst, b, c, t - tsplit, 0);
    pl[j * HWi + e] = p[e];
  }
  __syncthreads();
  const int n4 = Ho * Wo / 4;
  for (int k = threadIdx.x; k < np * n4; k += 256) {
    const int j = k / n4, q = k - j * n4;
    const int bc = bc0 + j;
    const int b = bc / C, c = bc - b * C;
    const int y = 4 * q / Wo, x = 4 * q - y * Wo;
    int y0, y1;
    float ly0, ly1;
    lin_idx(y, Hi, Ho, y0, y1, ly0, ly1);
    const float* r0 = pl + j * HWi + y0 * Wi;
    const float* r1 = pl + j * HWi + y1 * Wi;
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      int x0, x1;
      float lx0, lx1;
      lin_idx(x + u, Wi, Wo, x0, x1, lx0, lx1);
      v[u] = ly0 * (lx0 * r0[x0] + lx1 * r0[x1]) + ly1 * (lx0 * r1[x0] + lx1 * r1[x1]);
    }
    float* o = d + off5(dsb, dsc, dst_, b, c, t, y * Wo + x);
    if (vec) {
      *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) o[u] = v[u];
    }
  }
}

// ---------------- MotionAdaptor ----------------
__global__ __launch_bounds__(256) void adaptor_stats_kernel(const float* x, long sb, long sc, long st, int C, int T,
                                                            int HW, float* mean_out, float* std_out) {
  const int bc = blockIdx.x;
  const int b = bc / C, c = bc % C;
  const float* p = x + (long)b * sb + (long)c * sc;
  const int n = T * HW;
  double s = 0.0, dummy = 0.0;
  // (t, hw) of element e tracked incrementally (no division per element); same order
  const int t0 = threadIdx.x / HW, hw0 = threadIdx.x - t0 * HW;
  const int dt = 256 / HW, dhw = 256 - dt * HW;
  {
    int t = t0, hw = hw0;
    for (int e = threadIdx.x; e < n; e += 256) {
      s += p[(long)t * st + hw];
      t += dt; hw += dhw;
      if (hw >= HW) { hw -= HW; ++t; }
    }
  }
  __shared__ double sh[8];
  block_sum2(s, dummy, sh);
  const double mean = s / n;
  double v2 = 0.0;
  dummy = 0.0;
  {
    int t = t0, hw = hw0;
    for (int e = threadIdx.x; e < n; e += 256) {
      const double d = p[(long)t * st + hw] - mean;
      v2 += d * d;
      t += dt; hw += dhw;
      if (hw >= HW) { hw -= HW; ++t; }
    }
  }
  __syncthreads();
  block_sum2(v2, dummy, sh);
  if (threadIdx.x == 0) {
    mean_out[bc] = (float)mean;
    std_out[bc] = sqrtf((float)(v2 / (n - 1)) + 1e-5f);
  }
}

// one (b, c) per grid.y, 32-bit (t, hw) within it (the flat 64-bit div/mod chain dominated)
__global__ __launch_bounds__(256) void adaptor_norm_kernel(float* d, long dsb, long dsc, long dst_, const float* s,
                                                           long ssb, long ssc, long sst, int C, int T, int HW,
                                                           const float* mean, const float* std_) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= T * HW) return;
  const int bc = blockIdx.y;
  const int b = bc / C, c = bc - b * C;
  const int t = e / HW, hw = e - t * HW;
  d[off5(dsb, dsc, dst_, b, c, t, hw)] = (s[off5(ssb, ssc, sst, b, c, t, hw)] - mean[bc]) / std_[bc];
}

// zero the first and last frame of every clip of a frame-major buffer (the 3x3x3 extrapolator's
// temporal zero padding): grid.y = 2 B rows of `len` floats, float4 stores
__global__ __launch_bounds__(256) void zero_pad_frames_kernel(float* p, long sb, long last, long len4) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= len4) return;
  const int r = blockIdx.y;
  float4* row = reinterpret_cast<float4*>(p + (long)(r >> 1) * sb + (r & 1) * last);
  row[e] = make_float4(0.f, 0.f, 0.f, 0.f);
}

inline unsigned nblk(long n) { return (unsigned)((n + 255) / 256); }

}  // namespace

namespace {

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// (sum, sumsq) partials per (b, group) unless the producer wrote them; returns the slots
int gn_statistics(hipStream_t s, const View& x, int groups, double* partials, int given_split) {
  // the statistics kernels read each (b, group) as Cg*T*H*W contiguous floats
  if (x.st != x.HW() || x.sc != (long)x.T * x.HW() || x.C % groups != 0)
    throw std::invalid_argument("groupnorm_silu: input must be [B][C][T][H][W] with contiguous (C, T, H, W) "
                                "per sample and C divisible by the group count");
  if (given_split > 0) return given_split;  // the producing conv's epilogue wrote the partials
  const int Cg = x.C / groups;
  const long L = (long)Cg * x.T * x.HW();
  int split = (int)((L + 32767) / 32768);
  if (split < 1) split = 1;
  if (split > 64) split = 64;
  if (L % 4 == 0 && al16(x.p) && x.sb % 4 == 0 && x.sc % 4 == 0) {
    // ~8 float4 loads per thread per block, at most 64 blocks per group (partials size)
    long chunk = (L + 63) / 64;
    if (chunk < 8192) chunk = 8192;
    chunk = (chunk + 4095) / 4096 * 4096;
    split = (int)((L + chunk - 1) / chunk);
    hipLaunchKernelGGL(gn_stats4_kernel, dim3(split, x.B * groups), dim3(256), 0, s, x.p, x.sb, x.sc, Cg, groups,
                       L, split, chunk, partials);
  } else {
    hipLaunchKernelGGL(gn_stats_kernel, dim3(split, x.B * groups), dim3(256), 0, s, x.p, x.sb, x.sc, Cg, groups, L,
                       split, partials);
  }
  return split;
}

// statistics (or the producer's partials) -> (mean, rstd) per (b, group), stored after
// the partial slots of the runtime's buffer ([B][groups][64][2] doubles, then gst)
const float2* gn_mean_rstd(hipStream_t s, const View& x, int groups, double* partials, int given_split) {
  const int split = gn_statistics(s, x, groups, partials, given_split);
  if (split > 64) throw std::invalid_argument("groupnorm: more than 64 statistics slots");
  float2* gst = reinterpret_cast<float2*>(partials + (size_t)x.B * groups * 64 * 2);
  const double n = (double)(x.C / groups) * x.T * x.HW();
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(x.B * groups), dim3(64), 0, s, partials, split, n, gst);
  return gst;
}

}  // namespace

const float2* groupnorm_affine(hipStream_t s, const View& x, int groups, const float* gamma, const float* beta,
                               double* partials, int given_split) {
  const float2* gst = gn_mean_rstd(s, x, groups, partials, given_split);
  float2* tab = reinterpret_cast<float2*>(partials + (size_t)x.B * groups * 64 * 2 + (size_t)x.B * groups);
  hipLaunchKernelGGL(gn_affine_kernel, dim3(x.B), dim3(256), 0, s, gst, gamma, beta, x.C, x.C / groups, groups, tab);
  return tab;
}

void groupnorm_silu(hipStream_t s, const View& x, const View& out, int groups, const float* gamma,
                    const float* beta, const float* film, int film_row, int film_nt, const int* t_batch,
                    const View* res, double* partials, int given_split) {
  const float2* gst = gn_mean_rstd(s, x, groups, partials, given_split);
  const int Cg = x.C / groups;
  const long L = (long)Cg * x.T * x.HW();
  const bool vec4 = x.HW() % 4 == 0 && L / 4 < (1L << 31) && al16(x.p) && al16(out.p) && x.sb % 4 == 0 &&
                    x.sc % 4 == 0 && out.sb % 4 == 0 && out.sc % 4 == 0 && out.st % 4 == 0 &&
                    (!res || (al16(res->p) && res->sb % 4 == 0 && res->sc % 4 == 0 && res->st % 4 == 0));
  const int HW = x.HW();
  if (vec4 && (long)x.T * HW / 4 >= 1024 && x.st == HW && out.st == HW && (!res || res->st == HW) &&
      (long)x.B * x.C < 65536) {
    const int THW4 = x.T * HW / 4;
    const int per = 2048;  // float4 per block: eight per thread
    hipLaunchKernelGGL(gn_apply_plane_kernel, dim3((THW4 + per - 1) / per, x.B * x.C), dim3(256), 0, s, x.p, x.sb,
                       x.sc, out.p, out.sb, out.sc, x.C, Cg, groups, THW4, gst, gamma, beta, film,
                       film_row, film_nt, t_batch, res ? res->p : nullptr, res ? res->sb : 0, res ? res->sc : 0, per);
    return;
  }
  if (vec4) {
    int split4 = (int)((L / 4 + 2047) / 2048);
    if (split4 < 1) split4 = 1;
    hipLaunchKernelGGL(gn_apply4_kernel, dim3(split4, x.B * groups), dim3(256), 0, s, x.p, x.sb, x.sc, out.p, out.sb,
                       out.sc, out.st, x.C, Cg, groups, x.T, x.HW(), gst, gamma, beta, film, film_row,
                       film_nt, t_batch, res ? res->p : nullptr, res ? res->sb : 0, res ? res->sc : 0,
                       res ? res->st : 0, split4);
    return;
  }
  int split2 = (int)((L + 8191) / 8192);
  if (split2 < 1) split2 = 1;
  hipLaunchKernelGGL(gn_apply_kernel, dim3(split2, x.B * groups), dim3(256), 0, s, x.p, x.sb, x.sc, out.p, out.sb,
                     out.sc, out.st, x.C, Cg, groups, x.T, x.HW(), gst, gamma, beta, film, film_row,
                     film_nt, t_batch, res ? res->p : nullptr, res ? res->sb : 0, res ? res->sc : 0,
                     res ? res->st : 0, split2);
}

void groupnorm_silu_x3op(hipStream_t s, const View& x, const X3Op& out, int groups, const float* gamma,
                         const float* beta, const float* film, int film_row, int film_nt, const int* t_batch,
                         double* partials, int given_split) {
  if (x.C % 16 != 0 || out.C != x.C || out.B != x.B || out.T != x.T || out.H != x.H || out.W != x.W)
    throw std::invalid_argument("groupnorm_silu_x3op: operand geometry does not match the input");
  const float2* gst = gn_mean_rstd(s, x, groups, partials, given_split);
  const int Hp = x.H + 2 * out.pad, Wp = x.W + 2 * out.pad;
  // [hl][c8][cg][P][Hp*Wp][8] halves
  const long cg_stride = (long)x.B * x.T * Hp * Wp * 8, hl_stride = (long)(x.C / 16) * cg_stride * 2;
  hipLaunchKernelGGL(gn_apply_x3op_kernel, dim3((x.T * Hp * Wp + 255) / 256, x.B, x.C / 16), dim3(256), 0, s, x.p,
                     x.sb, x.sc, x.st, out.p, cg_stride, hl_stride, x.C, x.C / groups, groups, x.T, x.H, x.W, out.pad,
                     gst, gamma, beta, film, film_row, film_nt, t_batch, x3_range_ptr());
}

void channel_ln(hipStream_t s, const View& out, const View& in0, const View* in1, const float* gamma) {
  const View& i1 = in1 ? *in1 : in0;
  const long npix = (long)out.B * out.T * out.HW();
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  auto m4 = [](const View& v) { return v.sb % 4 == 0 && v.sc % 4 == 0 && v.st % 4 == 0; };
  if (out.HW() % 4 == 0 && a16(out.p) && a16(in0.p) && a16(i1.p) && m4(out) && m4(in0) && m4(i1)) {
    hipLaunchKernelGGL(channel_ln4_kernel, dim3((unsigned)((npix / 4 + 31) / 32)), dim3(256), 0, s, out.p, out.sb, out.sc,
                       out.st, in0.p, in0.sb, in0.sc, in0.st, in0.C, i1.p, i1.sb, i1.sc, i1.st, out.C, out.T, out.HW(),
                       out.B, gamma);
    return;
  }
  hipLaunchKernelGGL(channel_ln_kernel, dim3((unsigned)((npix + 31) / 32)), dim3(256), 0, s, out.p, out.sb, out.sc, out.st, in0.p,
                     in0.sb, in0.sc, in0.st, in0.C, i1.p, i1.sb, i1.sc, i1.st, out.C, out.T, out.HW(), out.B, gamma);
}

void temporal_prologue(hipStream_t s, const View& x, const float* gamma, const float* lw, const float* lb,
                       const View& z, const View& r) {
  const long npix = (long)x.B * x.T * x.HW();
  // one thread per pixel where that fills the chip (256-wide coalesced channel planes), else the
  // channels split over 16 groups of 16 pixels
  if (npix >= 256L * 1024) {
    hipLaunchKernelGGL(temporal_prologue_kernel, dim3(nblk(npix)), dim3(256), 0, s, x.p, x.sb, x.sc, x.st, x.C, x.T,
                       x.HW(), x.B, gamma, lw, lb, z.p, z.sb, z.sc, z.st, r.p, r.sb, r.sc, r.st);
  } else {
    hipLaunchKernelGGL((temporal_prologue_grp_kernel<16, 16>), dim3((unsigned)((npix + 15) / 16)), dim3(256), 0, s, x.p,
                       x.sb, x.sc, x.st, x.C, x.T, x.HW(), x.B, gamma, lw, lb, z.p, z.sb, z.sc, z.st, r.p, r.sb, r.sc,
                       r.st);
  }
}

void copy_view(hipStream_t s, const View& d, const View& src) {
  const long total = d.numel();
  hipLaunchKernelGGL(copy_kernel, dim3(nblk(total)), dim3(256), 0, s, d.p, d.sb, d.sc, d.st, src.p, src.sb, src.sc,
                     src.st, d.C, d.T, d.HW(), total);
}

void maxpool_hw2(hipStream_t s, const View& d, const View& src) {
  const long total = d.numel();
  hipLaunchKernelGGL(maxpool_kernel, dim3(nblk(total)), dim3(256), 0, s, d.p, d.sb, d.sc, d.st, src.p, src.sb,
                     src.sc, src.st, d.C, d.T, d.H, d.W, src.W, total);
}

void bilinear_frames(hipStream_t s, const View& d, const View& a, const View& b, int t_split) {
  const long total = d.numel();
  if (d.W % 4 == 0 && a.H * a.W <= 1024 && d.T < 65536 && a.H == b.H && a.W == b.W) {
    const int vec = ((uintptr_t)d.p & 15) == 0 && d.sb % 4 == 0 && d.sc % 4 == 0 && d.st % 4 == 0;
    const int nbc = d.B * d.C;
    hipLaunchKernelGGL(bilinear_lds_kernel, dim3((nbc + BPLS - 1) / BPLS, d.T), dim3(256), 0, s, d.p, d.sb, d.sc,
                       d.st, a.p, a.sb, a.sc, a.st, b.p, b.sb, b.sc, b.st, t_split, d.C, nbc, d.H, d.W, a.H, a.W,
                       vec);
    return;
  }
  if (d.W % 4 == 0 && (long)d.B * d.C < 65536 && d.T < 65536) {
    const int vec = ((uintptr_t)d.p & 15) == 0 && d.sb % 4 == 0 && d.sc % 4 == 0 && d.st % 4 == 0;
    const int n4 = d.H * d.W / 4;
    hipLaunchKernelGGL(bilinear4_kernel, dim3((n4 + 255) / 256, d.T, d.B * d.C), dim3(256), 0, s, d.p, d.sb, d.sc,
                       d.st, a.p, a.sb, a.sc, a.st, b.p, b.sb, b.sc, b.st, t_split, d.C, d.H, d.W, a.H, a.W, vec);
    return;
  }
  hipLaunchKernelGGL(bilinear_kernel, dim3(nblk(total)), dim3(256), 0, s, d.p, d.sb, d.sc, d.st, a.p, a.sb, a.sc,
                     a.st, b.p, b.sb, b.sc, b.st, t_split, d.C, d.T, d.H, d.W, a.H, a.W, total);
}

void adaptor_stats(hipStream_t s, const View& x, float* mean, float* std_, double* /*partials*/) {
  hipLaunchKernelGGL(adaptor_stats_kernel, dim3(x.B * x.C), dim3(256), 0, s, x.p, x.sb, x.sc, x.st, x.C, x.T, x.HW(),
                     mean, std_);
}

void adaptor_normalize(hipStream_t s, const View& d, const View& src, const float* mean, const float* std_) {
  const int bstep = 65535 / d.C;  // grid.y limit
  for (int b0 = 0; b0 < d.B; b0 += bstep) {
    const int nb = d.B - b0 < bstep ? d.B - b0 : bstep;
    hipLaunchKernelGGL(adaptor_norm_kernel, dim3(nblk((long)d.T * d.HW()), nb * d.C), dim3(256), 0, s,
                       d.p + (long)b0 * d.sb, d.sb, d.sc, d.st, src.p + (long)b0 * src.sb, src.sb, src.sc, src.st,
                       d.C, d.T, d.HW(), mean + (long)b0 * d.C, std_ + (long)b0 * d.C);
  }
}

void zero_pad_frames(hipStream_t s, const View& x) {
  // frame-major: frame t of clip b is st contiguous floats at b * sb + t * st
  if (!(x.st == (long)x.C * x.HW() && x.sc == x.HW() && x.st % 4 == 0 && x.sb % 4 == 0 &&
        ((uintptr_t)x.p & 15) == 0 && x.B <= 32767 && x.T >= 2))
    throw std::invalid_argument("zero_pad_frames: needs a frame-major buffer of 16-byte aligned frames");
  hipLaunchKernelGGL(zero_pad_frames_kernel, dim3(nblk(x.st / 4), 2 * x.B), dim3(256), 0, s, x.p, x.sb,
                     (long)(x.T - 1) * x.st, x.st / 4);
}

}  // namespace extdm
