// Attention kernels on fp32 MFMA (v_mfma_f32_32x32x2_f32), one wave per head.
//
// window_attention: shifted 3-D window self-attention (WindowAttention3D +
//   STWAttentionLayer, u12:408-559) or temporal attention per pixel
//   (Attention, u12:252-302). A window / pixel has N <= 32 tokens, so one
//   32x32 MFMA tile holds the whole score matrix:
//     S^T = K Q^T   (lane = query i, 16 key rows j in registers; the other 16
//                    in lane i^32)  -> +bias, shift mask, softmax in registers
//     O^T = V^T P^T (P^T is the accumulator of the first product, used as the
//                    B operand with the k order permuted to the register order;
//                    V^T comes from an LDS transpose of the V tile)
//   The cyclic shift, zero padding and window partition/reverse are index maps:
//   tokens are gathered from and scattered back to their original positions.
// cross_attention: TrajWarp multi-head cross-attention (u12:719-773),
//   flash-style over 32-key chunks with an online softmax (the reference
//   materialises the 8x3584x512 map; its outputs are the same up to rounding).
#include "kernels.h"

namespace extdm {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int region_label(int c, int P, int w, int s) {
  // compute_mask's slice sweep (u12:376-389): [:-w] -> 0, [-w:-s] -> 1, [-s:] -> 2,
  // where a zero shift makes the last slice cover the whole axis.
  if (s == 0) return 2;
  if (c >= P - s) return 2;
  if (c >= P - w) return 1;
  return 0;
}

__global__ __launch_bounds__(256) void window_attn_kernel(const float* __restrict__ qkv, long qsb, long qsc,
                                                          float* __restrict__ o, long osb, long osc, AttnGeom g,
                                                          int heads, const float* __restrict__ bias_dense,
                                                          const float* __restrict__ rcos,
                                                          const float* __restrict__ rsin, float q_scale,
                                                          long plane /* T stride = H*W */) {
  __shared__ float Vs[4][32][33];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int tok = lane & 31;
  const int h = lane >> 5;

  int b, N;
  long pos;
  bool valid;
  int lab = 0;
  if (g.mode == 0) {
    const int nWd = g.Dp / g.ws0, nWh = g.Hp / g.ws1, nWw = g.Wp / g.ws2;
    int r = blockIdx.x;
    const int ww = r % nWw; r /= nWw;
    const int wh = r % nWh; r /= nWh;
    const int wd = r % nWd;
    b = r / nWd;
    N = g.ws0 * g.ws1 * g.ws2;
    const int td = tok / (g.ws1 * g.ws2), th = (tok / g.ws2) % g.ws1, tw = tok % g.ws2;
    const int cd = wd * g.ws0 + td, ch = wh * g.ws1 + th, cw = ww * g.ws2 + tw;
    const int od = (cd + g.ss0) % g.Dp, oh = (ch + g.ss1) % g.Hp, ow = (cw + g.ss2) % g.Wp;
    valid = tok < N && od < g.D && oh < g.H && ow < g.W;
    pos = (long)od * plane + (long)oh * g.W + ow;
    lab = region_label(cd, g.Dp, g.ws0, g.ss0) * 9 + region_label(ch, g.Hp, g.ws1, g.ss1) * 3 +
          region_label(cw, g.Wp, g.ws2, g.ss2);
  } else {
    const int HW = g.H * g.W;
    b = blockIdx.x / HW;
    const int hw = blockIdx.x % HW;
    N = g.D;
    valid = tok < N;
    pos = (long)tok * plane + hw;
  }
  const bool shifted = g.mode == 0 && (g.ss0 | g.ss1 | g.ss2);
  const int hid = heads * 32;
  const float* qb = qkv + (long)b * qsb;

  for (int hd = wave; hd < heads; hd += 4) {
    float q[16], k[16], v[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int d = 2 * s + h;
      q[s] = valid ? qb[(long)(hd * 32 + d) * qsc + pos] : 0.f;
      k[s] = valid ? qb[(long)(hid + hd * 32 + d) * qsc + pos] : 0.f;
      v[s] = valid ? qb[(long)(2 * hid + hd * 32 + d) * qsc + pos] : 0.f;
    }
    // scale, then rotary (interleaved pairs; partner element lives in lane ^ 32)
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      q[s] *= q_scale;
      const float qp = __shfl_xor(q[s], 32);
      const float kp = __shfl_xor(k[s], 32);
      const float c = rcos[tok * 16 + s], sn = rsin[tok * 16 + s];
      if (h == 0) {
        q[s] = q[s] * c + (-qp) * sn;
        k[s] = k[s] * c + (-kp) * sn;
      } else {
        q[s] = q[s] * c + qp * sn;
        k[s] = k[s] * c + kp * sn;
      }
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) Vs[wave][tok][2 * s + h] = v[s];

    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(k[s], q[s], acc, 0, 0, 0);

    // acc[r] = S[i = tok][j = (r&3) + 8(r>>2) + 4h]
    const float* bd = bias_dense + (long)hd * 1024 + tok * 32;
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = (r & 3) + 8 * (r >> 2) + 4 * h;
      float sv = acc[r] + bd[j];
      if (shifted) {
        const int lj = __shfl(lab, j);
        if (lj != lab) sv += -100.f;
      }
      if (j >= N) sv = -INFINITY;
      acc[r] = sv;
      mx = fmaxf(mx, sv);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc[r] = expf(acc[r] - mx);
      sum += acc[r];
    }
    sum += __shfl_xor(sum, 32);
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = acc[r] / sum;

    __syncthreads();  // Vs visible
    f32x16 out;
#pragma unroll
    for (int r = 0; r < 16; ++r) out[r] = 0.f;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int j = (s & 3) + 8 * (s >> 2) + 4 * h;
      out = __builtin_amdgcn_mfma_f32_32x32x2f32(Vs[wave][j][tok], acc[s], out, 0, 0, 0);
    }
    // out[r] = O[i = tok][dd = (r&3) + 8(r>>2) + 4h]
    if (valid) {
      float* ob = o + (long)b * osb + pos;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int dd = (r & 3) + 8 * (r >> 2) + 4 * h;
        ob[(long)(hd * 32 + dd) * osc] = out[r];
      }
    }
    __syncthreads();  // Vs reuse
  }
}

__global__ __launch_bounds__(256) void cross_attn_kernel(const float* __restrict__ Q, const float* __restrict__ K,
                                                         const float* __restrict__ V, float* __restrict__ O, int C,
                                                         int heads, int NQ, int NK) {
  __shared__ float Vs[4][32][33];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int tok = lane & 31;
  const int h = lane >> 5;
  const int nqt = (NQ + 31) / 32;
  const int b = blockIdx.x / nqt;
  const int i0 = (blockIdx.x % nqt) * 32;
  const bool qvalid = i0 + tok < NQ;
  const float* qb = Q + (long)b * C * NQ;
  const float* kb = K + (long)b * C * NK;
  const float* vb = V + (long)b * C * NK;
  const float inv = 5.656854249492381f;  // sqrt(32): scores / sqrt(dk)
  for (int hd = wave; hd < heads; hd += 4) {
    float q[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) q[s] = qvalid ? qb[(long)(hd * 32 + 2 * s + h) * NQ + i0 + tok] : 0.f;
    f32x16 out;
#pragma unroll
    for (int r = 0; r < 16; ++r) out[r] = 0.f;
    float m = -INFINITY, l = 0.f;
    for (int j0 = 0; j0 < NK; j0 += 32) {
      const bool kvalid = j0 + tok < NK;
      float k[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const long off = (long)(hd * 32 + 2 * s + h) * NK + j0 + tok;
        k[s] = kvalid ? kb[off] : 0.f;
        Vs[wave][tok][2 * s + h] = kvalid ? vb[off] : 0.f;
      }
      f32x16 sc;
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[r] = 0.f;
#pragma unroll
      for (int s = 0; s < 16; ++s) sc = __builtin_amdgcn_mfma_f32_32x32x2f32(k[s], q[s], sc, 0, 0, 0);
      float cm = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = j0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        float sv = sc[r] / inv;
        if (j >= NK) sv = -INFINITY;
        sc[r] = sv;
        cm = fmaxf(cm, sv);
      }
      cm = fmaxf(cm, __shfl_xor(cm, 32));
      const float mn = fmaxf(m, cm);
      const float alpha = expf(m - mn);
      float ps = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sc[r] = expf(sc[r] - mn);
        ps += sc[r];
      }
      ps += __shfl_xor(ps, 32);
      l = l * alpha + ps;
      m = mn;
#pragma unroll
      for (int r = 0; r < 16; ++r) out[r] *= alpha;
      __syncthreads();
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int j = (s & 3) + 8 * (s >> 2) + 4 * h;
        out = __builtin_amdgcn_mfma_f32_32x32x2f32(Vs[wave][j][tok], sc[s], out, 0, 0, 0);
      }
      __syncthreads();
    }
    if (qvalid) {
      float* ob = O + (long)b * C * NQ + i0 + tok;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int dd = (r & 3) + 8 * (r >> 2) + 4 * h;
        ob[(long)(hd * 32 + dd) * NQ] = out[r] / l;
      }
    }
  }
}

}  // namespace

void window_attention(hipStream_t s, const View& qkv, const View& o, const AttnGeom& g, int heads,
                      const float* bias_dense, const float* rope_cos, const float* rope_sin, float q_scale) {
  unsigned nblocks;
  if (g.mode == 0) nblocks = (unsigned)(qkv.B * (g.Dp / g.ws0) * (g.Hp / g.ws1) * (g.Wp / g.ws2));
  else nblocks = (unsigned)(qkv.B * g.H * g.W);
  note_kernel("window_attn_kernel");
  hipLaunchKernelGGL(window_attn_kernel, dim3(nblocks), dim3(256), 0, s, qkv.p, qkv.sb, qkv.sc, o.p, o.sb, o.sc, g,
                     heads, bias_dense, rope_cos, rope_sin, q_scale, qkv.st);
}

void cross_attention(hipStream_t s, const float* q, const float* k, const float* v, float* o, int B, int C,
                     int heads, int NQ, int NK) {
  const unsigned nblocks = (unsigned)(B * ((NQ + 31) / 32));
  hipLaunchKernelGGL(cross_attn_kernel, dim3(nblocks), dim3(256), 0, s, q, k, v, o, C, heads, NQ, NK);
}

}  // namespace extdm
