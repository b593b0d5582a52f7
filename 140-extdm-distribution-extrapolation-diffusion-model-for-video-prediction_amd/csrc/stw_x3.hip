// Fused attention layers on f16x3 MFMA (see conv_x3.hip for the split): one WAVE per
// token group of 32 tokens, every intermediate in registers.
//
// MODE 0: Residual(PreNorm(STWAttentionLayer)) over one 3-D window of <= 32 tokens
//   (u12:138-158, 408-559, 961-963):  x[:, win] += proj(attn(qkv(chanLN(x[:, win])))) + b
// MODE 1: Residual(PreNorm(chanLN, AttentionLayer)) over frames: 32 / T pixels' T <= 32
//   frames, cross-pixel scores masked (u12:236-327, 903-915):
//   y = chanLN(x)*g; z = LayerNorm(y)*w+b; out = x + y + to_out(attn(qkv(z)))
//
// Per wave (lane = (token lc, half h)):
//  1. the lane loads exactly the channels of its MFMA k-slices (16s + 8h + e) of its
//     token, normalises (mean / var reduced with the partner half) and keeps them as
//     fp16 hi/lo fragments: Xn never leaves registers;
//  2. per unit of 32 qkv rows (one dim-32 head or two dim-16 heads):
//       Q^T, K^T = Wq·Xn^T, Wk·Xn^T  (rows = head dims in registers, lane = token)
//       V       = Xn·Wv^T            (rows = tokens in registers, lane = head dim)
//     RoPE pairs are adjacent registers. S^T = K·Q^T, P^T = softmax, O^T = V^T·P^T and
//     the projection Y += Wp·O^T all take the previous accumulator as an MFMA operand
//     (registers 8s..8s+7 = k-step s, the same row permutation on both sides);
//  3. epilogue: Y + bias + residual to the token positions.
// The unit's packed weights (q, k, v, proj slices; hi/lo fp16, pre-scaled by a power
// of two per matrix) are shared by the block's waves through a double-buffered
// LDS-DMA ring, one barrier per unit.
#include <algorithm>
#include <cstdlib>

#include "kernels.h"

namespace extdm {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ int dof(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ int region_label(int c, int P, int w, int s) {
  if (s == 0) return 2;
  if (c >= P - s) return 2;
  if (c >= P - w) return 1;
  return 0;
}

struct Tok {
  long pos;
  int valid, exists, lab, rpos;
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
    const int per = g.D <= 16 ? 16 : 32;
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

// hi = fp16(v), lo = fp16(v - hi) of an opaque v (split_src, kernels.h): the
// probabilities and scaled q / k / v here are products, whose two fp16 roundings hipcc
// would otherwise lower differently (hi + lo off by an fp16 ulp in ~2^-13 of the values;
// it made the reciprocal-multiply softmax fail at 2.7e-4).
// CHECK: OR |v| >= 65504 (fp16 overflow of hi) into bad; the probabilities (in [0, 1])
// skip it. Compiler-visible split2c rather than the split2 asm (kernels.h): these splits
// read MFMA results and feed MFMAs, and only compiler-visible VALU gets its MFMA hazard
// waits (4 VALU per pair; the per-element cvt / cvt-back / sub / pack took 8).
template <bool CHECK = true>
__device__ __forceinline__ void split8(const float* v, h8& hi, h8& lo, int& bad) {
  float m = 0.f;
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    const float w0 = split_src(v[e]), w1 = split_src(v[e + 1]);
    if (CHECK) m = fmaxf(fmaxf(m, fabsf(w0)), fabsf(w1));
    f16x2_t ph, pl;
    split2c(w0, w1, ph, pl);
    hi[e] = ph.x; hi[e + 1] = ph.y;
    lo[e] = pl.x; lo[e + 1] = pl.y;
  }
  if (CHECK) bad |= m >= 65504.f;
}

__device__ __forceinline__ f32x16 mma3(const h8& ah, const h8& al, const h8& bh, const h8& bl, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
  return c;
}

// Packed unit slice (halves): [q: C/16 frags][k: C/16][v: C/16][proj: C/32 tiles x 2 k-steps],
// each frag = [hl][64 lanes][8].
template <int C>
struct UnitLayout {
  static constexpr int KS = C / 16;
  static constexpr int FRAG = 2 * 512;  // halves per frag (hi + lo)
  static constexpr int Q = 0, K = KS * FRAG, V = 2 * KS * FRAG, P = 3 * KS * FRAG;
  static constexpr int HALVES = 3 * KS * FRAG + (C / 32) * 2 * FRAG;
};

template <int C, int MODE, int DH, int NW>
// x and out alias for the in-place STW layers (MODE 0): no __restrict__ on them.
__global__ __launch_bounds__(NW * 64) void attn_x3_kernel(const float* x, float* out,
                                                          long sb, long sc, long st, long osb, long osc, AttnGeom g,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ ln_w,
                                                          const float* __restrict__ ln_b,
                                                          const _Float16* __restrict__ wpk,
                                                          const float* __restrict__ wsc,  // 2^-s: q, k, v, proj
                                                          const float* __restrict__ bp,
                                                          const float* __restrict__ bias_dense, int bstride,
                                                          const float* __restrict__ rcos,
                                                          const float* __restrict__ rsin, float q_scale,
                                                          int groups_per_sample, int total_groups,
                                                          int* __restrict__ range_flag, int dbg) {
  using UL = UnitLayout<C>;
  constexpr int KS = UL::KS;
  constexpr int UNITS = 8 * DH / 32;  // heads 8
  constexpr int HPU = 32 / DH;
  constexpr int RH = DH / 2;
  constexpr int CT = C / 32;
  extern __shared__ __attribute__((aligned(16))) _Float16 wsm[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, lc = lane & 31;
  const int gidx = blockIdx.x * NW + wave;
  const bool active = gidx < total_groups;
  const int b = active ? gidx / groups_per_sample : 0;
  const int grp = active ? gidx % groups_per_sample : 0;
  const float* xb = x + (long)b * sb;
  float* ob = out + (long)b * osb;
  // Global traffic through buffer descriptors: a lane's 32-bit byte offset carries its token
  // (and channel half), the channel row goes into the wave-uniform soffset, and an invalid
  // token's offset lies past the extent (loads return 0, stores are dropped): no 64-bit
  // address arithmetic and no divergent branch per element (the host checks the extents
  // fit 31 bits).
  constexpr int OOB = 0x40000000;
  const int x_bytes = (int)(((long)(C - 1) * sc + (long)g.D * st) * 4);
  const int o_bytes = (int)(((long)(C - 1) * osc + (long)g.D * st) * 4);
  const auto rs_x = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xb), 0, x_bytes, 0x00020000);
  const auto rs_o = __builtin_amdgcn_make_buffer_rsrc(ob, 0, o_bytes, 0x00020000);
  const auto rs_g = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(gamma), 0, C * 4, 0x00020000);
  const auto rs_lw = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(MODE == 1 ? ln_w : gamma), 0, C * 4, 0x00020000);
  const auto rs_lb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(MODE == 1 ? ln_b : gamma), 0, C * 4, 0x00020000);
  auto ldb = [](const __amdgpu_buffer_rsrc_t& r, int vo, int so) __attribute__((always_inline)) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
  };

  auto load_unit = [&](int u, _Float16* dst) {
    const _Float16* src = wpk + (long)u * UL::HALVES;
    if (dbg & 1) {
      for (int pc = wave; pc < UL::HALVES / 512; pc += NW)
        *reinterpret_cast<h8*>(dst + pc * 512 + lane * 8) = *reinterpret_cast<const h8*>(src + pc * 512 + lane * 8);
    } else {
      for (int pc = wave; pc < UL::HALVES / 512; pc += NW)
        __builtin_amdgcn_global_load_lds((const void*)(src + pc * 512 + lane * 8), (lds_ptr_t)(dst + pc * 512), 16, 0,
                                         0);
    }
    if (dbg & 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  };
  load_unit(0, wsm);

  // ---- 1. normalisation into register fragments ----
  const Tok me = token_of<MODE>(lc, g, st, grp);
  const bool tok_ok = active && me.valid;
  const int vpro = tok_ok ? (int)((8 * h * sc + me.pos) * 4) : OOB;  // channel 8h + (16k + e)
  int bad = 0;
  h8 xh[KS], xl[KS];
  float m1 = 0.f, den1 = 1.f, rden1 = 1.f;
  {
    float xv[KS][8];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = 16 * k + 8 * h + e;
        // dbg & 4 (timing only): no x loads
        xv[k][e] = (dbg & 4) ? (tok_ok ? (float)(c ^ lane) * 0.01f : 0.f)
                             : ldb(rs_x, vpro, (int)((16 * k + e) * sc * 4));
        s += xv[k][e];
      }
    s += __shfl_xor(s, 32);
    m1 = s / C;
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = xv[k][e] - m1; v += d * d; }
    v += __shfl_xor(v, 32);
    den1 = sqrtf(v / C + 1e-5f);
    // one reciprocal instead of a division per element (~10 VALU each, in the prologue and
    // MODE 1's epilogue): the product differs from the quotient by at most an ulp
    rden1 = 1.f / den1;
    if (MODE == 0) {
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int c = 16 * k + 8 * h + e;
          xv[k][e] = me.valid ? (xv[k][e] - m1) * rden1 * ldb(rs_g, 32 * h, (16 * k + e) * 4) : 0.f;
        }
    } else {
      float s2 = 0.f;
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int c = 16 * k + 8 * h + e;
          xv[k][e] = (xv[k][e] - m1) * rden1 * ldb(rs_g, 32 * h, (16 * k + e) * 4);
          s2 += xv[k][e];
        }
      s2 += __shfl_xor(s2, 32);
      const float m2 = s2 / C;
      float v2 = 0.f;
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) { const float d = xv[k][e] - m2; v2 += d * d; }
      v2 += __shfl_xor(v2, 32);
      const float rstd2 = 1.0f / sqrtf(v2 / C + 1e-5f);
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int c = 16 * k + 8 * h + e;
          xv[k][e] = me.valid ? (xv[k][e] - m2) * rstd2 * ldb(rs_lw, 32 * h, (16 * k + e) * 4) +
                                    ldb(rs_lb, 32 * h, (16 * k + e) * 4)
                              : 0.f;
        }
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) split8(xv[k], xh[k], xl[k], bad);
  }
  // key-side token descriptors for the 16 keys j = dof(r, h) this lane's scores hold
  const bool shifted = MODE == 0 && (g.ss0 | g.ss1 | g.ss2) != 0;
  const int desc = (me.lab & 0xFFFF) | (me.exists << 16);
  // The keys j = dof(r, h) of this lane's score registers do not depend on the unit:
  // their masks are computed once (bit r), and their positions are known in closed
  // form, so the bias loads carry no shuffle dependency and issue early.
  unsigned kmis = 0, kgone = 0;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int dj = __shfl(desc, dof(r, h));
    kmis |= (unsigned)((dj & 0xFFFF) != me.lab) << r;
    kgone |= (unsigned)(!((dj >> 16) & 1)) << r;
  }
  const int kper = g.D <= 16 ? 16 : 32;

  f32x16 pacc[CT];
#pragma unroll
  for (int i = 0; i < CT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) pacc[i][r] = 0.f;

  const float sq = wsc[0] * q_scale, sk = wsc[1], sv = wsc[2];
  // RoPE factors of this lane's (token, dim pair) registers, the same for every unit (with
  // the q / k scales folded in when FOLD)
  // folded at C = 64 only: at C = 128 (one wave per SIMD) the 16 extra live registers
  // cost 20 % (interleaved A/B)
  constexpr bool FOLD = C == 64;
  float rcq[8], rsq[8], rck[8], rsk[8];
#pragma unroll
  for (int r = 0; r < 16; r += 2) {
    const int pi = (dof(r, h) % DH) >> 1;
    const float c = rcos[me.rpos * RH + pi], sn = rsin[me.rpos * RH + pi];
    rcq[r >> 1] = FOLD ? c * sq : c; rsq[r >> 1] = FOLD ? sn * sq : sn;
    rck[r >> 1] = FOLD ? c * sk : c; rsk[r >> 1] = FOLD ? sn * sk : sn;
  }
  for (int u = 0; u < UNITS; ++u) {
    _Float16* W = wsm + (u & 1) * UL::HALVES;
    // unit u's slice has landed in every wave's pieces: LDS-DMA completion is tracked by
    // the issuing wave's vmcnt only, so each wave drains it before the barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // ... and slot (u+1)&1 is free
    if (u + 1 < UNITS) load_unit(u + 1, wsm + ((u + 1) & 1) * UL::HALVES);
    if (!active) continue;
    // ---- 2a. Q^T, K^T (rows = dims, lane = token), V (rows = tokens, lane = dim) ----
    f32x16 q, k, v;
#pragma unroll
    for (int r = 0; r < 16; ++r) { q[r] = 0.f; k[r] = 0.f; v[r] = 0.f; }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const _Float16* fq = W + UL::Q + s * UL::FRAG + lane * 8;
      const _Float16* fk = W + UL::K + s * UL::FRAG + lane * 8;
      const _Float16* fv = W + UL::V + s * UL::FRAG + lane * 8;
      const h8 qh = *reinterpret_cast<const h8*>(fq), ql = *reinterpret_cast<const h8*>(fq + 512);
      const h8 kh = *reinterpret_cast<const h8*>(fk), kl = *reinterpret_cast<const h8*>(fk + 512);
      const h8 vh = *reinterpret_cast<const h8*>(fv), vl = *reinterpret_cast<const h8*>(fv + 512);
      q = mma3(qh, ql, xh[s], xl[s], q);
      k = mma3(kh, kl, xh[s], xl[s], k);
      v = mma3(xh[s], xl[s], vh, vl, v);
    }
    // scale, RoPE on (d, d+1) = registers (r, r+1); d = dof(r, h) within the head
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      float q0 = q[r], q1 = q[r + 1], k0 = k[r], k1 = k[r + 1];
      if (!FOLD) {
        q0 *= sq; q1 *= sq; k0 *= sk; k1 *= sk;
      }
      // one fma per output (a mul + fma instead of two muls and an add: one rounding fewer)
      q[r] = fmaf(q0, rcq[r >> 1], -(q1 * rsq[r >> 1]));
      q[r + 1] = fmaf(q1, rcq[r >> 1], q0 * rsq[r >> 1]);
      k[r] = fmaf(k0, rck[r >> 1], -(k1 * rsk[r >> 1]));
      k[r + 1] = fmaf(k1, rck[r >> 1], k0 * rsk[r >> 1]);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] *= sv;
    h8 qf[2][2], kf[2][2], vf[2][2];  // [k-step][hi|lo]
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float tq[8], tk[8], tv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { tq[e] = q[8 * s + e]; tk[e] = k[8 * s + e]; tv[e] = v[8 * s + e]; }
      split8(tq, qf[s][0], qf[s][1], bad);
      split8(tk, kf[s][0], kf[s][1], bad);
      split8(tv, vf[s][0], vf[s][1], bad);
    }
    // ---- 2b. per head: S^T = K Q^T (rows = keys j, lane = query i), softmax, O^T += V^T P^T ----
    f32x16 o;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = 0.f;
#pragma unroll
    for (int hh = 0; hh < HPU; ++hh) {
      const int head = u * HPU + hh;
      f32x16 sc_;
#pragma unroll
      for (int r = 0; r < 16; ++r) sc_[r] = 0.f;
#pragma unroll
      for (int s = 0; s < 2; ++s)
        if (HPU == 1 || s == hh) sc_ = mma3(kf[s][0], kf[s][1], qf[s][0], qf[s][1], sc_);
      const float* bd = bias_dense + ((long)head * bstride + me.rpos) * bstride;
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = dof(r, h);
        float s_ = sc_[r] + bd[MODE == 0 ? j : j % kper];
        if (MODE == 0) {
          if (shifted && ((kmis >> r) & 1)) s_ += -100.f;
        } else {
          if ((kmis >> r) & 1) s_ = -INFINITY;
        }
        if ((kgone >> r) & 1) s_ = -INFINITY;
        sc_[r] = s_;
        mx = fmaxf(mx, s_);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      // exp(s - mx) as v_exp_f32 (2^x) of fma(s, log2 e, -mx log2 e): masked -inf -> 0
      const float mxl = mx * 1.44269504088896341f;
      float sum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sc_[r] = __builtin_amdgcn_exp2f(fmaf(sc_[r], 1.44269504088896341f, -mxl));
        sum += sc_[r];
      }
      sum += __shfl_xor(sum, 32);
      const float inv = 1.f / sum;
#pragma unroll
      for (int r = 0; r < 16; ++r) sc_[r] *= inv;
      // O^T[dd][i] = sum_j V^T[dd][j] P^T[j][i]; lanes of the unit's other head masked
      const bool mine = HPU == 1 || (lc / DH) == hh;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float tp[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) tp[e] = sc_[8 * s + e];
        h8 ph, pl;
        split8<false>(tp, ph, pl, bad);
        h8 ah = vf[s][0], al = vf[s][1];
        if (!mine) {
#pragma unroll
          for (int e = 0; e < 8; ++e) { ah[e] = (_Float16)0.f; al[e] = (_Float16)0.f; }
        }
        o = mma3(ah, al, ph, pl, o);
      }
    }
    // ---- 2c. projection: Y[c][i] += sum_dd Wp[c][u*32 + dd] O^T[dd][i] ----
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float to[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) to[e] = o[8 * s + e];
      h8 oh, ol;
      split8(to, oh, ol, bad);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const _Float16* fp = W + UL::P + (ct * 2 + s) * UL::FRAG + lane * 8;
        pacc[ct] = mma3(*reinterpret_cast<const h8*>(fp), *reinterpret_cast<const h8*>(fp + 512), oh, ol, pacc[ct]);
      }
    }
  }
  if (bad) atomicOr(range_flag, 2);
  // MODE 1 with 2-pixel groups: a lane's token is (pixel, frame), so a direct store touches
  // 16 frame planes per instruction, 8 bytes each, and every 64-B line is written by 8
  // waves. Instead the workgroup's 16 consecutive pixels x D frames x C channels go through
  // LDS ([c][t][16 px], rows padded for conflict-free lane writes) and leave as 64-B rows.
  const bool lds_epi = MODE == 1 && C == 64 && NW == 8 && g.D <= 16 && groups_per_sample % NW == 0 && (g.H * g.W) % 16 == 0 &&
                       (osc & 3) == 0 && (st & 3) == 0 && (((uintptr_t)out) & 15) == 0;
  if (MODE == 1 && lds_epi) {
    constexpr int RS = 20, CS = 16 * RS + 8;  // CS % 16 == 8: the two lane halves hit other banks
    float* T = reinterpret_cast<float*>(wsm);
    __syncthreads();  // every wave is done with the weight ring
    const int pl = wave * 2 + (lc >> 4), tt = lc & 15;
    const float spj = wsc[3];
    const int vex = (int)((4 * h * sc + me.pos) * 4);
    if (active) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int cu = ct * 32 + (r & 3) + 8 * (r >> 2);
          const float xv = ldb(rs_x, vex, (int)(cu * sc * 4));
          const float y = pacc[ct][r] * spj;
          const float res = y + (xv + (xv - m1) * rden1 * ldb(rs_g, 16 * h, cu * 4));
          T[(cu + 4 * h) * CS + tt * RS + pl] = res;
        }
    }
    __syncthreads();
    if (!active) return;
    const int hw0 = (blockIdx.x * NW) % groups_per_sample * 2;
    float* o0 = ob + hw0;
    for (int i = tid; i < C * g.D * 4; i += NW * 64) {
      const int q = i & 3, ctr = i >> 2;
      const int t = ctr % g.D, c = ctr / g.D;
      const float4 v = *reinterpret_cast<const float4*>(T + c * CS + t * RS + 4 * q);
      *reinterpret_cast<float4*>(o0 + (long)c * osc + (long)t * st + 4 * q) = v;
    }
    return;
  }
  if (!active || !me.valid) return;
  if (dbg & 8) {  // timing only: no epilogue loads / stores (one store keeps the work live)
    float acc = 0.f;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc += pacc[ct][r];
    if (acc == 12345.f) ob[me.pos] = acc;
    return;
  }

  // ---- 3. bias + residual, write back ----
  // row c = cu + 4h of register r: the lane offset carries 4h, the soffset cu
  const float spj = wsc[3];
  const int vex = (int)((4 * h * sc + me.pos) * 4), veo = (int)((4 * h * osc + me.pos) * 4);
  const auto rs_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(MODE == 0 ? bp : gamma), 0, C * 4, 0x00020000);
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int cu = ct * 32 + (r & 3) + 8 * (r >> 2);
      const float xv = ldb(rs_x, vex, (int)(cu * sc * 4));
      const float pb = ldb(rs_b, 16 * h, cu * 4);  // MODE 0: proj bias; MODE 1: gamma
      const float y = pacc[ct][r] * spj;
      float res;
      if (MODE == 0) res = (y + pb) + xv;
      else res = y + (xv + (xv - m1) * rden1 * pb);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(res), rs_o, veo, (int)(cu * osc * 4), 0);
    }
  }
}

template <int C, int MODE, int DH, int NW>
void launch_nw(hipStream_t s, const View& x, const View& out, const AttnGeom& g, int groups, const float* gamma,
               const float* lw, const float* lb, const void* wpk, const float* wsc, const float* bp,
               const float* bias_dense, int bstride, const float* rcos, const float* rsin, float q_scale) {
  static const int dbg = [] { const char* v = getenv("EXTDM_X3_DBG"); return v ? atoi(v) : 0; }();
  // MODE 1 at C = 64, 8 waves: the epilogue's [C][16 frames][16 px] staging tile (rows of
  // 20, channels of 328 floats) reuses the ring
  const size_t ring = (size_t)2 * UnitLayout<C>::HALVES * sizeof(_Float16);
  const size_t lds = (MODE == 1 && C == 64 && NW == 8) ? std::max(ring, (size_t)C * 328 * sizeof(float)) : ring;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_x3_kernel<C, MODE, DH, NW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const int total = x.B * groups;
  hipLaunchKernelGGL((attn_x3_kernel<C, MODE, DH, NW>), dim3((total + NW - 1) / NW), dim3(NW * 64), lds, s, x.p,
                     out.p, x.sb, x.sc, x.st, out.sb, out.sc, g, gamma, lw, lb,
                     reinterpret_cast<const _Float16*>(wpk), wsc, bp, bias_dense, bstride, rcos, rsin, q_scale, groups,
                     total, x3_range_ptr(), dbg);
}

template <int C, int MODE, int DH>
void launch(hipStream_t s, const View& x, const View& out, const AttnGeom& g, int groups, const float* gamma,
            const float* lw, const float* lb, const void* wpk, const float* wsc, const float* bp,
            const float* bias_dense, int bstride, const float* rcos, const float* rsin, float q_scale) {
  static const int nw = [] { const char* v = getenv("EXTDM_X3_ATTN_NW"); return v ? atoi(v) : 0; }();
  // C = 128 needs > 256 VGPRs: one wave per SIMD
  if (C == 64 && nw != 4)
    launch_nw<C, MODE, DH, 8>(s, x, out, g, groups, gamma, lw, lb, wpk, wsc, bp, bias_dense, bstride, rcos, rsin, q_scale);
  else
    launch_nw<C, MODE, DH, 4>(s, x, out, g, groups, gamma, lw, lb, wpk, wsc, bp, bias_dense, bstride, rcos, rsin, q_scale);
}

template <int MODE, int DH>
bool dispatch_c(hipStream_t s, const View& x, const View& out, const AttnGeom& g, int groups, const float* gamma,
                const float* lw, const float* lb, const void* wpk, const float* wsc, const float* bp,
                const float* bias_dense, int bstride, const float* rcos, const float* rsin, float q_scale) {
  if (x.C == 64) launch<64, MODE, DH>(s, x, out, g, groups, gamma, lw, lb, wpk, wsc, bp, bias_dense, bstride, rcos, rsin, q_scale);
  else if (x.C == 128) launch<128, MODE, DH>(s, x, out, g, groups, gamma, lw, lb, wpk, wsc, bp, bias_dense, bstride, rcos, rsin, q_scale);
  else return false;
  return true;
}

}  // namespace

int attn_x3_unit_halves(int C) {
  if (C == 64) return UnitLayout<64>::HALVES;
  if (C == 128) return UnitLayout<128>::HALVES;
  return 0;
}

bool attn_x3_supported(int C, int ntok, int dim_head, int heads) {
  return heads == 8 && (C == 64 || C == 128) && ntok <= 32 && (dim_head == 32 || dim_head == 16);
}

// the kernels address a sample of x / out with 31-bit byte offsets (buffer descriptors)
static bool extent_ok(const View& v, const AttnGeom& g) {
  return ((long)(v.C - 1) * v.sc + (long)g.D * v.st) * 4 < (1L << 30) && v.st == (long)v.H * v.W;
}

bool stw_x3(hipStream_t s, const View& x, const AttnGeom& g, int heads, int dim_head, const float* gamma,
            const void* wpk, const float* wsc, const float* bp, const float* bias_dense, int bstride,
            const float* rcos, const float* rsin, float q_scale) {
  const int N = g.ws0 * g.ws1 * g.ws2;
  if (!attn_x3_supported(x.C, N, dim_head, heads) || !extent_ok(x, g)) return false;
  const int groups = (g.Dp / g.ws0) * (g.Hp / g.ws1) * (g.Wp / g.ws2);
  if (dim_head == 32)
    return dispatch_c<0, 32>(s, x, x, g, groups, gamma, nullptr, nullptr, wpk, wsc, bp, bias_dense, bstride, rcos,
                             rsin, q_scale);
  return dispatch_c<0, 16>(s, x, x, g, groups, gamma, nullptr, nullptr, wpk, wsc, bp, bias_dense, bstride, rcos, rsin,
                           q_scale);
}

bool temporal_x3(hipStream_t s, const View& x, const View& out, const AttnGeom& g, int heads, int dim_head,
                 const float* gamma, const float* ln_w, const float* ln_b, const void* wpk, const float* wsc,
                 const float* bias_dense, int bstride, const float* rcos, const float* rsin, float q_scale) {
  if (!attn_x3_supported(x.C, g.D, dim_head, heads) || g.D > 32 || !extent_ok(x, g) || !extent_ok(out, g)) return false;
  if (out.sc != x.sc || out.st != x.st) return false;
  const int ppb = g.D <= 16 ? 2 : 1;
  const int groups = (g.H * g.W + ppb - 1) / ppb;
  if (dim_head == 32)
    return dispatch_c<1, 32>(s, x, out, g, groups, gamma, ln_w, ln_b, wpk, wsc, nullptr, bias_dense, bstride, rcos,
                             rsin, q_scale);
  return dispatch_c<1, 16>(s, x, out, g, groups, gamma, ln_w, ln_b, wpk, wsc, nullptr, bias_dense, bstride, rcos, rsin,
                           q_scale);
}

}  // namespace extdm
