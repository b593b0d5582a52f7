// Fused attention layers — one workgroup per 32-token group, qkv never in HBM.
//
// MODE 0: Residual(PreNorm(STWAttentionLayer)) — the group is one 3-D window
//   (u12:138-158 LayerNorm, 408-559 WindowAttention3D / STWAttentionLayer, 961-963):
//     x[:, window] += proj( attn( qkv( chanLN(x[:, window]) ) ) ) + proj.bias
// MODE 1: init_temporal_attn = Residual(PreNorm(chanLN, AttentionLayer)) — the group
//   is the T frames of 32/T pixels (T <= 16: two pixels, cross-pixel scores masked)
//   (u12:236-327, 903-915):
//     y = chanLN(x)*g; z = LayerNorm(y)*w+b; out = x + y + to_out(attn(qkv(z)))
//
// 1. the group's C x 32 tokens are gathered from their positions (shift / padding /
//    pixel maps), normalised over C and kept in LDS;
// 2. each wave takes heads w and w+4: q/k/v (3 x 32x32 MFMA tiles, K = C) come out
//    with lane = token and rows = head dims, which is already the operand layout of
//    S^T = K Q^T (the contraction over head dims runs in the accumulator's register
//    order, so no data moves); RoPE pairs (d, d+1) sit in adjacent registers;
//    bias / mask / softmax in registers; O^T = V^T P^T with V transposed once
//    through LDS; O goes to LDS;
// 3. the output projection + residual, written back to the original positions.
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

struct Tok {
  long pos;
  bool valid;  // a real (unpadded) position: read / written
  bool exists; // a token of the group (participates as a key)
  int lab;     // shift-mask region label (MODE 0) / pixel index (MODE 1)
  int rpos;    // rotary / relative-bias position
};

template <int MODE>
__device__ __forceinline__ Tok token_of(int tk, const AttnGeom& g, long st, int blk_rem) {
  Tok o;
  if (MODE == 0) {
    const int nWh = g.Hp / g.ws1, nWw = g.Wp / g.ws2;
    int rb = blk_rem;
    const int ww = rb % nWw; rb /= nWw;
    const int wh = rb % nWh; rb /= nWh;
    const int wd = rb;
    const int N = g.ws0 * g.ws1 * g.ws2;
    const int td = tk / (g.ws1 * g.ws2), th = (tk / g.ws2) % g.ws1, tw = tk % g.ws2;
    const int cd = wd * g.ws0 + td, ch = wh * g.ws1 + th, cw = ww * g.ws2 + tw;
    const int od = (cd + g.ss0) % g.Dp, oh = (ch + g.ss1) % g.Hp, ow = (cw + g.ss2) % g.Wp;
    o.exists = tk < N;
    o.valid = o.exists && od < g.D && oh < g.H && ow < g.W;
    o.pos = (long)od * st + (long)oh * g.W + ow;
    o.lab = region_label(cd, g.Dp, g.ws0, g.ss0) * 9 + region_label(ch, g.Hp, g.ws1, g.ss1) * 3 +
            region_label(cw, g.Wp, g.ws2, g.ss2);
    o.rpos = tk;
  } else {
    const int HW = g.H * g.W;
    const int per = g.D <= 16 ? 16 : 32;  // token slots per pixel
    const int p = tk / per, t = tk % per;
    const int hw = blk_rem * (32 / per) + p;
    o.exists = t < g.D && hw < HW;
    o.valid = o.exists;
    o.pos = (long)t * st + hw;
    o.lab = p;
    o.rpos = t;
  }
  return o;
}

template <int C, int MODE>
__global__ __launch_bounds__(256) void attn_fused_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                         long sb, long sc, long st, long osb, long osc, AttnGeom g,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ ln_w,
                                                         const float* __restrict__ ln_b,
                                                         const float* __restrict__ wqkv,
                                                         const float* __restrict__ wp,
                                                         const float* __restrict__ bp,
                                                         const float* __restrict__ bias_dense,
                                                         const float* __restrict__ rcos,
                                                         const float* __restrict__ rsin, float q_scale,
                                                         int groups_per_sample) {
  constexpr int HEADS = 8;
  __shared__ float Xn[C][32];
  __shared__ float Ob[HEADS * 32][32];
  __shared__ float Vt[4][32][33];
  __shared__ float red[8][32];
  __shared__ float stat[4][32];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, lc = lane & 31;
  const int b = blockIdx.x / groups_per_sample;
  const int grp_idx = blockIdx.x % groups_per_sample;
  const float* xb = x + (long)b * sb;
  float* ob = out + (long)b * osb;

  // ---- 1. normalisation of the group's tokens into LDS ----
  {
    const int tk = tid & 31, cg = tid >> 5;  // 8 channel groups
    const Tok T = token_of<MODE>(tk, g, st, grp_idx);
    auto reduce_to = [&](float v, int slot, bool is_mean, float mean_for_var) {
      red[cg][tk] = v;
      __syncthreads();
      if (tid < 32) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) t += red[i][tid];
        stat[slot][tid] = is_mean ? t / C : sqrtf(t / C + 1e-5f);
      }
      __syncthreads();
      (void)mean_for_var;
    };
    float s = 0.f;
    if (T.valid)
      for (int c = cg; c < C; c += 8) s += xb[(long)c * sc + T.pos];
    reduce_to(s, 0, true, 0.f);
    const float m1 = stat[0][tk];
    float v = 0.f;
    if (T.valid)
      for (int c = cg; c < C; c += 8) {
        const float d = xb[(long)c * sc + T.pos] - m1;
        v += d * d;
      }
    reduce_to(v, 1, false, m1);
    const float den1 = stat[1][tk];
    if (MODE == 0) {
      for (int c = cg; c < C; c += 8)
        Xn[c][tk] = T.valid ? (xb[(long)c * sc + T.pos] - m1) / den1 * gamma[c] : 0.f;
    } else {
      // second LayerNorm over y = chanLN(x) * gamma
      float s2 = 0.f;
      if (T.valid)
        for (int c = cg; c < C; c += 8) s2 += (xb[(long)c * sc + T.pos] - m1) / den1 * gamma[c];
      reduce_to(s2, 2, true, 0.f);
      const float m2 = stat[2][tk];
      float v2 = 0.f;
      if (T.valid)
        for (int c = cg; c < C; c += 8) {
          const float d = (xb[(long)c * sc + T.pos] - m1) / den1 * gamma[c] - m2;
          v2 += d * d;
        }
      reduce_to(v2, 3, false, m2);
      const float rstd2 = 1.0f / stat[3][tk];
      for (int c = cg; c < C; c += 8) {
        const float y = (xb[(long)c * sc + T.pos] - m1) / den1 * gamma[c];
        Xn[c][tk] = T.valid ? (y - m2) * rstd2 * ln_w[c] + ln_b[c] : 0.f;
      }
    }
    __syncthreads();
  }

  const Tok me = token_of<MODE>(lc, g, st, grp_idx);
  const bool masked = MODE == 1 || (g.ss0 | g.ss1 | g.ss2) != 0;

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
      const float c = rcos[me.rpos * 16 + pi], sn = rsin[me.rpos * 16 + pi];
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
    const float* bd = bias_dense + (long)hd * 1024 + me.rpos * 32;
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = dof(r, h);
      const int lj = __shfl(me.lab, j);
      const int pj = __shfl(me.rpos, j);
      const int ej = __shfl((int)me.exists, j);
      float sv = sacc[r] + bd[pj];
      if (MODE == 0) {
        if (masked && lj != me.lab) sv += -100.f;
      } else {
        if (lj != me.lab) sv = -INFINITY;  // another pixel's frames
      }
      if (!ej) sv = -INFINITY;
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

  // ---- 3. output projection + residual ----
  const float m1 = stat[0][lc], den1 = stat[1][lc];
  for (int tile = wave; tile < C / 32; tile += 4) {
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const float* wpt = wp + (long)tile * (HEADS * 16) * 64 + lane;
#pragma unroll 8
    for (int s = 0; s < HEADS * 16; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wpt[s * 64], Ob[2 * s + h][lc], acc, 0, 0, 0);
    if (me.valid) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = tile * 32 + dof(r, h);
        const float xv = xb[(long)c * sc + me.pos];
        float res;
        if (MODE == 0) res = (acc[r] + bp[c]) + xv;
        else res = acc[r] + (xv + (xv - m1) / den1 * gamma[c]);
        ob[(long)c * osc + me.pos] = res;
      }
    }
  }
}

template <int MODE>
bool launch_mode(hipStream_t s, const View& x, const View& out, const AttnGeom& g, const float* gamma,
                 const float* lw, const float* lb, const float* wqkv, const float* wp, const float* bp,
                 const float* bias_dense, const float* rcos, const float* rsin, float q_scale) {
  int groups;
  if (MODE == 0) groups = (g.Dp / g.ws0) * (g.Hp / g.ws1) * (g.Wp / g.ws2);
  else {
    if (g.D > 32) return false;
    const int ppb = g.D <= 16 ? 2 : 1;
    groups = (g.H * g.W + ppb - 1) / ppb;
  }
  const unsigned nblocks = (unsigned)(x.B * groups);
#define L(CC)                                                                                                    \
  hipLaunchKernelGGL((attn_fused_kernel<CC, MODE>), dim3(nblocks), dim3(256), 0, s, x.p, out.p, x.sb, x.sc, x.st, \
                     out.sb, out.sc, g, gamma, lw, lb, wqkv, wp, bp, bias_dense, rcos, rsin, q_scale, groups)
  if (x.C == 64) L(64);
  else if (x.C == 128) L(128);
  else if (x.C == 256) L(256);
  else return false;
#undef L
  return true;
}

}  // namespace

bool stw_fused(hipStream_t s, const View& x, const AttnGeom& g, int heads, const float* gamma, const float* wqkv,
               const float* wp, const float* bp, const float* bias_dense, const float* rcos, const float* rsin,
               float q_scale) {
  if (heads != 8) return false;
  return launch_mode<0>(s, x, x, g, gamma, nullptr, nullptr, wqkv, wp, bp, bias_dense, rcos, rsin, q_scale);
}

bool temporal_fused(hipStream_t s, const View& x, const View& out, const AttnGeom& g, int heads, const float* gamma,
                    const float* ln_w, const float* ln_b, const float* wqkv, const float* wout,
                    const float* bias_dense, const float* rcos, const float* rsin, float q_scale) {
  if (heads != 8 || out.sc != x.sc || out.st != x.st) return false;
  return launch_mode<1>(s, x, out, g, gamma, ln_w, ln_b, wqkv, wout, nullptr, bias_dense, rcos, rsin, q_scale);
}

}  // namespace extdm
