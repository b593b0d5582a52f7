// Fused attention layers — one workgroup per token group, qkv never in HBM.
//
// MODE 0: Residual(PreNorm(STWAttentionLayer)) — the group is one 3-D window of
//   NT = 32 (window 2x4x4) or 64 (4x4x4) tokens (u12:138-158, 408-559, 961-963):
//     x[:, window] += proj( attn( qkv( chanLN(x[:, window]) ) ) ) + proj.bias
// MODE 1: Residual(PreNorm(chanLN, AttentionLayer)) over frames — the group is the
//   T <= 32 frames of 32/T pixels (cross-pixel scores masked) (u12:236-327, 903-915):
//     y = chanLN(x)*g; z = LayerNorm(y)*w+b; out = x + y + to_out(attn(qkv(z)))
//
// 1. the group's C x NT tokens are gathered from their positions (shift / padding /
//    pixel maps), normalised over C and kept in LDS;
// 2. heads are processed in units of 32 qkv rows (one head of dim 32, or a pair of
//    heads of dim 16), one unit per wave per phase. q/k/v come out of the MFMA with
//    lane = token and rows = head dims, which is already the operand layout of
//    S^T = K Q^T (the contraction over head dims runs in the accumulator's register
//    order, so no data moves; a dim-16 head uses half the registers); RoPE pairs
//    (d, d+1) sit in adjacent registers; bias / mask / softmax in registers;
//    O^T = V^T P^T with V transposed once through LDS; the unit's O goes to LDS;
// 3. after each phase (4 units) the output projection accumulates in registers;
//    the last phase adds bias + residual and writes back to the original positions.
// Weights are pre-packed so each MFMA's A fragment is one contiguous 256-B wave load:
//   qkv:  [unit][s][which q|k|v][lane] = W[which*HID + unit*32 + (lane&31)][2s + (lane>>5)]
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
  int valid;   // a real (unpadded) position: read / written
  int exists;  // a token of the group (participates as a key)
  int lab;     // shift-mask region label (MODE 0) / pixel index (MODE 1)
  int rpos;    // rotary / relative-bias position
};

template <int MODE>
__device__ __forceinline__ Tok token_of(int tk, const AttnGeom& g, long st, int grp) {
  Tok o;
  if (MODE == 0) {
    const int nWh = g.Hp / g.ws1, nWw = g.Wp / g.ws2;
    int rb = grp;
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
    const int hw = grp * (32 / per) + p;
    o.exists = t < g.D && hw < HW;
    o.valid = o.exists;
    o.pos = (long)t * st + hw;
    o.lab = p;
    o.rpos = t;
  }
  return o;
}

// Softmax over the NT keys of query row (lane) given per-tile score registers.
template <int TT>
__device__ __forceinline__ void softmax_rows(f32x16 (&s)[TT]) {
  float mx = -INFINITY;
#pragma unroll
  for (int t = 0; t < TT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[t][r]);
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < TT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[t][r] = expf(s[t][r] - mx);
      sum += s[t][r];
    }
  sum += __shfl_xor(sum, 32);
#pragma unroll
  for (int t = 0; t < TT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) s[t][r] = s[t][r] / sum;
}

template <int C, int MODE, int TT, int DH>
__global__ __launch_bounds__(256) void attn_fused_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                         long sb, long sc, long st, long osb, long osc, AttnGeom g,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ ln_w,
                                                         const float* __restrict__ ln_b,
                                                         const float* __restrict__ wqkv,
                                                         const float* __restrict__ wp,
                                                         const float* __restrict__ bp,
                                                         const float* __restrict__ bias_dense, int bstride,
                                                         const float* __restrict__ rcos,
                                                         const float* __restrict__ rsin, float q_scale,
                                                         int groups_per_sample) {
  constexpr int HEADS = 8;
  constexpr int NT = 32 * TT;
  constexpr int HID = HEADS * DH;
  constexpr int UNITS = HID / 32;         // 32-row qkv units
  constexpr int PHASES = (UNITS + 3) / 4;
  constexpr int HPU = 32 / DH;            // heads per unit
  constexpr int RH = DH / 2;              // rotary pairs per head
  constexpr int CG = 256 / NT;            // channel groups in the LayerNorm pass
  constexpr int NTILES = (C / 32) * TT;   // proj output tiles
  constexpr int TPW = (NTILES + 3) / 4;   // proj tiles per wave
  __shared__ float Xn[C][NT];
  __shared__ float Ob[128][NT];
  __shared__ float Vt[4][NT][33];
  __shared__ float red[CG][NT];
  __shared__ float stat[4][NT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, lc = lane & 31;
  const int b = blockIdx.x / groups_per_sample;
  const int grp = blockIdx.x % groups_per_sample;
  const float* xb = x + (long)b * sb;
  float* ob = out + (long)b * osb;

  // ---- 1. normalisation of the group's tokens into LDS ----
  {
    const int tk = tid % NT, cg = tid / NT;
    const Tok T = token_of<MODE>(tk, g, st, grp);
    auto reduce_to = [&](float v, int slot, bool is_mean) {
      red[cg][tk] = v;
      __syncthreads();
      if (tid < NT) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < CG; ++i) t += red[i][tid];
        stat[slot][tid] = is_mean ? t / C : sqrtf(t / C + 1e-5f);
      }
      __syncthreads();
    };
    float s = 0.f;
    if (T.valid)
      for (int c = cg; c < C; c += CG) s += xb[(long)c * sc + T.pos];
    reduce_to(s, 0, true);
    const float m1 = stat[0][tk];
    float v = 0.f;
    if (T.valid)
      for (int c = cg; c < C; c += CG) {
        const float d = xb[(long)c * sc + T.pos] - m1;
        v += d * d;
      }
    reduce_to(v, 1, false);
    const float den1 = stat[1][tk];
    if (MODE == 0) {
      for (int c = cg; c < C; c += CG)
        Xn[c][tk] = T.valid ? (xb[(long)c * sc + T.pos] - m1) / den1 * gamma[c] : 0.f;
    } else {
      float s2 = 0.f;
      if (T.valid)
        for (int c = cg; c < C; c += CG) s2 += (xb[(long)c * sc + T.pos] - m1) / den1 * gamma[c];
      reduce_to(s2, 2, true);
      const float m2 = stat[2][tk];
      float v2 = 0.f;
      if (T.valid)
        for (int c = cg; c < C; c += CG) {
          const float d = (xb[(long)c * sc + T.pos] - m1) / den1 * gamma[c] - m2;
          v2 += d * d;
        }
      reduce_to(v2, 3, false);
      const float rstd2 = 1.0f / stat[3][tk];
      for (int c = cg; c < C; c += CG) {
        const float y = (xb[(long)c * sc + T.pos] - m1) / den1 * gamma[c];
        Xn[c][tk] = T.valid ? (y - m2) * rstd2 * ln_w[c] + ln_b[c] : 0.f;
      }
    }
    __syncthreads();
  }

  Tok me[TT];
#pragma unroll
  for (int t = 0; t < TT; ++t) me[t] = token_of<MODE>(t * 32 + lc, g, st, grp);
  const bool shifted = MODE == 0 && (g.ss0 | g.ss1 | g.ss2) != 0;

  f32x16 pacc[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) pacc[i][r] = 0.f;

  for (int ph = 0; ph < PHASES; ++ph) {
    const int unit = ph * 4 + wave;
    if (unit < UNITS) {
      // ---- 2a. q, k, v for this unit: TT token tiles x 32 rows ----
      f32x16 q[TT], k[TT], v[TT];
#pragma unroll
      for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) { q[t][r] = 0.f; k[t][r] = 0.f; v[t][r] = 0.f; }
      const float* wq = wqkv + (long)unit * (C / 2) * 3 * 64 + lane;
#pragma unroll 4
      for (int s = 0; s < C / 2; ++s) {
        const float a0 = wq[(s * 3 + 0) * 64];
        const float a1 = wq[(s * 3 + 1) * 64];
        const float a2 = wq[(s * 3 + 2) * 64];
#pragma unroll
        for (int t = 0; t < TT; ++t) {
          const float xv = Xn[2 * s + h][t * 32 + lc];
          q[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, xv, q[t], 0, 0, 0);
          k[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, xv, k[t], 0, 0, 0);
          v[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a2, xv, v[t], 0, 0, 0);
        }
      }
      // q[t][r] = Q[token t*32+lc][d(r,h)] : scale then RoPE on (d, d+1) = registers (r, r+1)
#pragma unroll
      for (int t = 0; t < TT; ++t) {
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const int pi = (dof(r, h) % DH) >> 1;
          const float c = rcos[me[t].rpos * RH + pi], sn = rsin[me[t].rpos * RH + pi];
          const float q0 = q[t][r] * q_scale, q1 = q[t][r + 1] * q_scale;
          q[t][r] = q0 * c + (-q1) * sn;
          q[t][r + 1] = q1 * c + q0 * sn;
          const float k0 = k[t][r], k1 = k[t][r + 1];
          k[t][r] = k0 * c + (-k1) * sn;
          k[t][r + 1] = k1 * c + k0 * sn;
        }
        // V^T through LDS: Vt[token][d]
#pragma unroll
        for (int r = 0; r < 16; ++r) Vt[wave][t * 32 + lc][dof(r, h)] = v[t][r];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // ---- 2b. attention per head of the unit, per query tile ----
#pragma unroll
      for (int ti = 0; ti < TT; ++ti) {
        f32x16 o;
#pragma unroll
        for (int r = 0; r < 16; ++r) o[r] = 0.f;
#pragma unroll
        for (int hh = 0; hh < HPU; ++hh) {
          const int head = unit * HPU + hh;
          constexpr int S0 = 0;
          const int s_lo = hh * (16 / HPU), s_hi = s_lo + 16 / HPU;
          f32x16 sc_[TT];
#pragma unroll
          for (int tj = 0; tj < TT; ++tj) {
#pragma unroll
            for (int r = 0; r < 16; ++r) sc_[tj][r] = 0.f;
#pragma unroll
            for (int s = S0; s < 16; ++s)
              if (s >= s_lo && s < s_hi)
                sc_[tj] = __builtin_amdgcn_mfma_f32_32x32x2f32(k[tj][s], q[ti][s], sc_[tj], 0, 0, 0);
          }
          // sc_[tj][r] = S[i = ti*32+lc][j = tj*32 + d(r,h)]
          const float* bd = bias_dense + ((long)head * bstride + me[ti].rpos) * bstride;
#pragma unroll
          for (int tj = 0; tj < TT; ++tj) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int jj = dof(r, h);
              const int lj = __shfl(me[tj].lab, jj);
              const int pj = __shfl(me[tj].rpos, jj);
              const int ej = __shfl(me[tj].exists, jj);
              float sv = sc_[tj][r] + bd[pj];
              if (MODE == 0) {
                if (shifted && lj != me[ti].lab) sv += -100.f;
              } else {
                if (lj != me[ti].lab) sv = -INFINITY;  // another pixel's frames
              }
              if (!ej) sv = -INFINITY;
              sc_[tj][r] = sv;
            }
          }
          softmax_rows<TT>(sc_);
          // O^T[dd][i] += V^T[dd][j] P^T[j][i], rows of other heads of the unit masked
#pragma unroll
          for (int tj = 0; tj < TT; ++tj) {
#pragma unroll
            for (int s = 0; s < 16; ++s) {
              const int jj = dof(s, h);
              float va = Vt[wave][tj * 32 + jj][lc];
              if (HPU > 1 && (lc / DH) != hh) va = 0.f;
              o = __builtin_amdgcn_mfma_f32_32x32x2f32(va, sc_[tj][s], o, 0, 0, 0);
            }
          }
        }
        // o[r] = O[i = ti*32+lc][dd = d(r,h)] of this unit
#pragma unroll
        for (int r = 0; r < 16; ++r) Ob[wave * 32 + dof(r, h)][ti * 32 + lc] = o[r];
      }
    }
    __syncthreads();
    // ---- 3. output projection over this phase's 128 rows of O ----
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int tile = wave + 4 * i;
      if (tile < NTILES) {
        const int mt = tile / TT, tt = tile % TT;
        const float* wpt = wp + ((long)mt * (HID / 2) + ph * 64) * 64 + lane;
        const int rows = (HID - ph * 128) < 128 ? (HID - ph * 128) : 128;
#pragma unroll 8
        for (int s = 0; s < 64; ++s)
          if (2 * s < rows)
            pacc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(wpt[s * 64], Ob[2 * s + h][tt * 32 + lc], pacc[i], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // ---- 4. bias + residual, write back ----
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int tile = wave + 4 * i;
    if (tile >= NTILES) continue;
    const int mt = tile / TT, tt = tile % TT;
    const Tok& T = me[tt];
    if (!T.valid) continue;
    const float m1 = stat[0][tt * 32 + lc], den1 = stat[1][tt * 32 + lc];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = mt * 32 + dof(r, h);
      const float xv = xb[(long)c * sc + T.pos];
      float res;
      if (MODE == 0) res = (pacc[i][r] + bp[c]) + xv;
      else res = pacc[i][r] + (xv + (xv - m1) / den1 * gamma[c]);
      ob[(long)c * osc + T.pos] = res;
    }
  }
}

template <int MODE, int TT, int DH>
bool launch_c(hipStream_t s, const View& x, const View& out, const AttnGeom& g, const float* gamma,
              const float* lw, const float* lb, const float* wqkv, const float* wp, const float* bp,
              const float* bias_dense, int bstride, const float* rcos, const float* rsin, float q_scale) {
  int groups;
  if (MODE == 0) groups = (g.Dp / g.ws0) * (g.Hp / g.ws1) * (g.Wp / g.ws2);
  else {
    if (g.D > 32) return false;
    const int ppb = g.D <= 16 ? 2 : 1;
    groups = (g.H * g.W + ppb - 1) / ppb;
  }
  const unsigned nblocks = (unsigned)(x.B * groups);
  note_kernel("attn_fused_kernel<%d, %d, %d, %d>", x.C, MODE, TT, DH);
#define L(CC)                                                                                                     \
  hipLaunchKernelGGL((attn_fused_kernel<CC, MODE, TT, DH>), dim3(nblocks), dim3(256), 0, s, x.p, out.p, x.sb, x.sc, \
                     x.st, out.sb, out.sc, g, gamma, lw, lb, wqkv, wp, bp, bias_dense, bstride, rcos, rsin, q_scale,  \
                     groups)
  if (x.C == 64) L(64);
  else if (x.C == 128) L(128);
  else if (x.C == 256) L(256);
  else return false;
#undef L
  return true;
}

}  // namespace

bool fused_attn_supported(int C, int ntok, int dim_head, int heads) {
  return heads == 8 && (C == 64 || C == 128 || C == 256) && (ntok <= 32 || ntok == 64) &&
         (dim_head == 32 || dim_head == 16);
}

bool stw_fused(hipStream_t s, const View& x, const AttnGeom& g, int heads, int dim_head, const float* gamma,
               const float* wqkv, const float* wp, const float* bp, const float* bias_dense, int bstride,
               const float* rcos, const float* rsin, float q_scale) {
  const int N = g.ws0 * g.ws1 * g.ws2;
  if (!fused_attn_supported(x.C, N, dim_head, heads)) return false;
  const bool big = N > 32;
  if (dim_head == 32) {
    return big ? launch_c<0, 2, 32>(s, x, x, g, gamma, nullptr, nullptr, wqkv, wp, bp, bias_dense, bstride, rcos, rsin,
                                    q_scale)
               : launch_c<0, 1, 32>(s, x, x, g, gamma, nullptr, nullptr, wqkv, wp, bp, bias_dense, bstride, rcos, rsin,
                                    q_scale);
  }
  return big ? launch_c<0, 2, 16>(s, x, x, g, gamma, nullptr, nullptr, wqkv, wp, bp, bias_dense, bstride, rcos, rsin,
                                  q_scale)
             : launch_c<0, 1, 16>(s, x, x, g, gamma, nullptr, nullptr, wqkv, wp, bp, bias_dense, bstride, rcos, rsin,
                                  q_scale);
}

bool temporal_fused(hipStream_t s, const View& x, const View& out, const AttnGeom& g, int heads, int dim_head,
                    const float* gamma, const float* ln_w, const float* ln_b, const float* wqkv, const float* wout,
                    const float* bias_dense, int bstride, const float* rcos, const float* rsin, float q_scale) {
  if (!fused_attn_supported(x.C, g.D, dim_head, heads) || g.D > 32) return false;
  if (out.sc != x.sc || out.st != x.st) return false;
  if (dim_head == 32)
    return launch_c<1, 1, 32>(s, x, out, g, gamma, ln_w, ln_b, wqkv, wout, nullptr, bias_dense, bstride, rcos, rsin,
                              q_scale);
  return launch_c<1, 1, 16>(s, x, out, g, gamma, ln_w, ln_b, wqkv, wout, nullptr, bias_dense, bstride, rcos, rsin,
                            q_scale);
}

}  // namespace extdm
