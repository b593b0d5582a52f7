// Fused Residual(PreNorm(STWAttentionLayer)) — one workgroup per 3-D window
// (u12:138-158 LayerNorm, 408-559 WindowAttention3D / STWAttentionLayer, 961-963):
//
//   x[:, window] += proj( attn( qkv( LN(x[:, window]) ) ) )
//
// 1. the window's C x 32 tokens are gathered from their (shifted, padded)
//    positions, layer-normalised over C (biased var, gamma) and kept in LDS;
// 2. each wave takes heads w and w+4: q/k/v (3 x 32x32 MFMA tiles, K = C) come
//    out with lane = token and rows = head dims, which is already the operand
//    layout of S^T = K Q^T (the contraction over head dims is taken in the
//    accumulator's register order, so no data moves); RoPE pairs (d, d+1) sit in
//    adjacent registers; bias / shift mask / softmax in registers; O^T = V^T P^T
//    with V transposed once through LDS; O goes to LDS;
// 3. proj (C x 256) + bias + residual, written back to the original positions.
// The qkv tensor (768 channels) never touches HBM.
// Weights are pre-packed so each MFMA's A fragment is one contiguous 256-B wave load:
//   qkv:  [head][s][which q|k|v][lane] = W[which*256 + head*32 + (lane&31)][2s + (lane>>5)]
//   proj: [tile][s][lane]              = W[tile*32 + (lane&31)][2s + (lane>>5)]
#include "kernels.h"

namespace extdm {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int region_label(int c, int P, int w, int s) {
  if (s == 0) return 2;
  if (c >= P - s) return 2;
  if (c >= P - w) return 1;
  return 0;
}

__device__ __forceinline__ int dof(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

template <int C>
__global__ __launch_bounds__(256) void stw_fused_kernel(float* __restrict__ x, long sb, long sc, long st,
                                                        AttnGeom g, const float* __restrict__ gamma,
                                                        const float* __restrict__ wqkv, const float* __restrict__ wp,
                                                        const float* __restrict__ bp,
                                                        const float* __restrict__ bias_dense,
                                                        const float* __restrict__ rcos,
                                                        const float* __restrict__ rsin, float q_scale) {
  constexpr int HEADS = 8;
  __shared__ float Xn[C][32];
  __shared__ float Ob[HEADS * 32][32];
  __shared__ float Vt[4][32][33];
  __shared__ float red[8][32];
  __shared__ float stat[2][32];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, lc = lane & 31;

  // ---- window geometry (same index maps as window_attn_kernel) ----
  const int nWd = g.Dp / g.ws0, nWh = g.Hp / g.ws1, nWw = g.Wp / g.ws2;
  int rb = blockIdx.x;
  const int ww = rb % nWw; rb /= nWw;
  const int wh = rb % nWh; rb /= nWh;
  const int wd = rb % nWd;
  const int b = rb / nWd;
  const int N = g.ws0 * g.ws1 * g.ws2;
  float* xb = x + (long)b * sb;

  auto token = [&](int tk, long& pos, bool& valid, int& lab) {
    const int td = tk / (g.ws1 * g.ws2), th = (tk / g.ws2) % g.ws1, tw = tk % g.ws2;
    const int cd = wd * g.ws0 + td, ch = wh * g.ws1 + th, cw = ww * g.ws2 + tw;
    const int od = (cd + g.ss0) % g.Dp, oh = (ch + g.ss1) % g.Hp, ow = (cw + g.ss2) % g.Wp;
    valid = tk < N && od < g.D && oh < g.H && ow < g.W;
    pos = (long)od * st + (long)oh * g.W + ow;
    lab = region_label(cd, g.Dp, g.ws0, g.ss0) * 9 + region_label(ch, g.Hp, g.ws1, g.ss1) * 3 +
          region_label(cw, g.Wp, g.ws2, g.ss2);
  };

  // ---- 1. LayerNorm of the window's tokens into LDS ----
  {
    const int tk = tid & 31, grp = tid >> 5;  // 8 channel groups
    long pos; bool valid; int lab;
    token(tk, pos, valid, lab);
    float s = 0.f;
    if (valid)
      for (int c = grp; c < C; c += 8) s += xb[(long)c * sc + pos];
    red[grp][tk] = s;
    __syncthreads();
    if (tid < 32) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) t += red[i][tid];
      stat[0][tid] = t / C;
    }
    __syncthreads();
    const float mean = stat[0][tk];
    float v = 0.f;
    if (valid)
      for (int c = grp; c < C; c += 8) {
        const float d = xb[(long)c * sc + pos] - mean;
        v += d * d;
      }
    red[grp][tk] = v;
    __syncthreads();
    if (tid < 32) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) t += red[i][tid];
      stat[1][tid] = sqrtf(t / C + 1e-5f);
    }
    __syncthreads();
    const float den = stat[1][tk];
    for (int c = grp; c < C; c += 8)
      Xn[c][tk] = valid ? (xb[(long)c * sc + pos] - mean) / den * gamma[c] : 0.f;
    __syncthreads();
  }

  long mypos; bool myvalid; int mylab;
  token(lc, mypos, myvalid, mylab);
  const bool shifted = (g.ss0 | g.ss1 | g.ss2) != 0;

  // ---- 2. per head: qkv, attention ----
  for (int hd = wave; hd < HEADS; hd += 4) {
    f32x16 q, k, v;
#pragma unroll
    for (int r = 0; r < 16; ++r) { q[r] = 0.f; k[r] = 0.f; v[r] = 0.f; }
    const float* wq = wqkv + (long)hd * (C / 2) * 3 * 64 + lane;
#pragma unroll 8
    for (int s = 0; s < C / 2; ++s) {
      const float xv = Xn[2 * s + h][lc];
      const float a0 = wq[(s * 3 + 0) * 64];
      const float a1 = wq[(s * 3 + 1) * 64];
      const float a2 = wq[(s * 3 + 2) * 64];
      q = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, xv, q, 0, 0, 0);
      k = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, xv, k, 0, 0, 0);
      v = __builtin_amdgcn_mfma_f32_32x32x2f32(a2, xv, v, 0, 0, 0);
    }
    // q[r] = Q[token lc][d(r,h)]: scale, then RoPE on (d, d+1) = registers (r, r+1)
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const int pi = dof(r, h) >> 1;
      const float c = rcos[lc * 16 + pi], sn = rsin[lc * 16 + pi];
      const float q0 = q[r] * q_scale, q1 = q[r + 1] * q_scale;
      q[r] = q0 * c + (-q1) * sn;
      q[r + 1] = q1 * c + q0 * sn;
      const float k0 = k[r], k1 = k[r + 1];
      k[r] = k0 * c + (-k1) * sn;
      k[r + 1] = k1 * c + k0 * sn;
    }
    // S^T = K Q^T, contraction over head dims in register order
    f32x16 sacc;
#pragma unroll
    for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
#pragma unroll
    for (int s = 0; s < 16; ++s) sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(k[s], q[s], sacc, 0, 0, 0);
    // sacc[r] = S[i = lc][j = d(r,h)]
    const float* bd = bias_dense + (long)hd * 1024 + lc * 32;
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = dof(r, h);
      float sv = sacc[r] + bd[j];
      if (shifted) {
        const int lj = __shfl(mylab, j);
        if (lj != mylab) sv += -100.f;
      }
      if (j >= N) sv = -INFINITY;
      sacc[r] = sv;
      mx = fmaxf(mx, sv);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sacc[r] = expf(sacc[r] - mx);
      sum += sacc[r];
    }
    sum += __shfl_xor(sum, 32);
#pragma unroll
    for (int r = 0; r < 16; ++r) sacc[r] = sacc[r] / sum;
    // V^T through LDS: Vt[token][d]
#pragma unroll
    for (int r = 0; r < 16; ++r) Vt[wave][lc][dof(r, h)] = v[r];
    __syncthreads();
    f32x16 o;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = 0.f;
#pragma unroll
    for (int s = 0; s < 16; ++s)
      o = __builtin_amdgcn_mfma_f32_32x32x2f32(Vt[wave][dof(s, h)][lc], sacc[s], o, 0, 0, 0);
    // o[r] = O[i = lc][dd = d(r,h)]
#pragma unroll
    for (int r = 0; r < 16; ++r) Ob[hd * 32 + dof(r, h)][lc] = o[r];
    __syncthreads();
  }

  // ---- 3. proj + bias + residual ----
  for (int tile = wave; tile < C / 32; tile += 4) {
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const float* wpt = wp + (long)tile * (HEADS * 16) * 64 + lane;
#pragma unroll 8
    for (int s = 0; s < HEADS * 16; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wpt[s * 64], Ob[2 * s + h][lc], acc, 0, 0, 0);
    if (myvalid) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = tile * 32 + dof(r, h);
        float* p = xb + (long)c * sc + mypos;
        *p = (acc[r] + bp[c]) + *p;
      }
    }
  }
}

}  // namespace

bool stw_fused(hipStream_t s, const View& x, const AttnGeom& g, int heads, const float* gamma, const float* wqkv,
               const float* wp, const float* bp, const float* bias_dense, const float* rcos, const float* rsin,
               float q_scale) {
  if (heads != 8) return false;
  const unsigned nblocks = (unsigned)(x.B * (g.Dp / g.ws0) * (g.Hp / g.ws1) * (g.Wp / g.ws2));
#define L(CC)                                                                                                   \
  hipLaunchKernelGGL(stw_fused_kernel<CC>, dim3(nblocks), dim3(256), 0, s, x.p, x.sb, x.sc, x.st, g, gamma, wqkv, \
                     wp, bp, bias_dense, rcos, rsin, q_scale)
  if (x.C == 64) L(64);
  else if (x.C == 128) L(128);
  else if (x.C == 256) L(256);
  else return false;
#undef L
  return true;
}

}  // namespace extdm
