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
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "attn_x3_ops.h"

namespace extdm {

namespace {

using namespace attn_ops;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

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
    const int per = temporal_slots(g);
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

// Packed unit slice (halves): [q: C/16 frags][k: C/16][v: C/16][proj: C/32 tiles x 2 k-steps],
// each frag = [hl][64 lanes][8].
template <int C>
struct UnitLayout {
  static constexpr int KS = C / 16;
  static constexpr int FRAG = 2 * 512;  // halves per frag (hi + lo)
  static constexpr int Q = 0, K = KS * FRAG, V = 2 * KS * FRAG, P = 3 * KS * FRAG;
  static constexpr int HALVES = 3 * KS * FRAG + (C / 32) * 2 * FRAG;
};

// mbias: [npat][8 heads][32 queries][32 keys] fp32, the relative-position bias with the
// masks folded in (build_mask_bias, runtime.cpp): -100 for a shifted window's region
// mismatch (u12:414-436), -inf for keys past the window's N tokens and for another
// pixel's frames (MODE 1). MODE 0 shifted layers carry 8 window classes (bit d: last
// window along a shifted dim, where the region labels differ), the rest one. A lane's 16
// score registers hold keys j = dof(r, h) = 8q + 4h + e (r = 4q + e): four 16-B rows of
// its query's table row, added to the QK^T accumulator in one v_add per score (masks need
// no further VALU). The table carries the scores' factor 2^(e_q + e_k) (wsc note).
template <int C, int MODE, int DH, int NW, bool TILE, bool BF>
// BF: the attention contractions (QK^T, PV) on bf16 MFMA (EXTDM_PRECISION_BF16_ATTN); qkv / proj stay f16x3.
// x and out alias for the in-place STW layers (MODE 0): no __restrict__ on them.
__global__ __launch_bounds__(NW * 64) void attn_x3_kernel(const float* x, float* out,
                                                          long sb, long sc, long st, long osb, long osc, AttnGeom g,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ ln_w,
                                                          const float* __restrict__ ln_b,
                                                          const _Float16* __restrict__ wpk,
                                                          const float* __restrict__ wsc,  // 2^-s: q, k, v, proj
                                                          const float* __restrict__ bp,
                                                          const float* __restrict__ mbias, int npat,
                                                          const float* __restrict__ rcos,
                                                          const float* __restrict__ rsin, float q_scale,
                                                          int groups_per_sample, int total_groups,
                                                          int* __restrict__ range_flag, int dbg,
                                                          long long* __restrict__ tstamp) {
  using UL = UnitLayout<C>;
  constexpr int KS = UL::KS;
  constexpr int UNITS = 8 * DH / 32;  // heads 8
  constexpr int HPU = 32 / DH;
  constexpr int RH = DH / 2;
  constexpr int CT = C / 32;
  extern __shared__ __attribute__((aligned(16))) _Float16 wsm[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // Global traffic through buffer descriptors: a lane's 32-bit byte offset carries its token
  // (and channel half), the channel row goes into the wave-uniform soffset, and an invalid
  // token's offset lies past the extent (loads return 0, stores are dropped): no 64-bit
  // address arithmetic and no divergent branch per element (the host checks the extents
  // fit 31 bits).
  constexpr int OOB = 0x40000000;
  const int x_bytes = (int)(((long)(C - 1) * sc + (long)g.D * st) * 4);
  const int o_bytes = (int)(((long)(C - 1) * osc + (long)g.D * st) * 4);
  const auto rs_g = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(gamma), 0, C * 4, 0x00020000);
  const auto rs_lw = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(MODE == 1 ? ln_w : gamma), 0, C * 4, 0x00020000);
  const auto rs_lb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(MODE == 1 ? ln_b : gamma), 0, C * 4, 0x00020000);
  const auto rs_mb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(mbias), 0, npat * 8 * 4096, 0x00020000);
  auto ldb = [](const __amdgpu_buffer_rsrc_t& r, int vo, int so) __attribute__((always_inline)) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
  };


  // Operand scales. An fp16 lo below 2^-14 is subnormal, so a split operand far below unit
  // scale loses bits (tests/test_gpu_precision.py activation-scale cases); here every split
  // operand is brought near unit scale by powers of two (exact): the normalised input by
  // 2^e_w, e_w from the wave's (tile paths: the workgroup's) largest |value| (prologue), and wsc (packed_attn_x3,
  // runtime.cpp) takes the MFMA results (weights pre-scaled per matrix) to q * q_scale *
  // 2^e_q, k * 2^e_k, v * 2^e_v once 2^-e_w is folded in, exponents estimated from the
  // weights and the norm's affine for an input of unit largest value;
  // the scores are then S * 2^(e_q + e_k) (the bias / mask table carries the same factor),
  // csm = log2(e) * 2^-(e_q + e_k) is the softmax's exp2 factor, P is split as 16 P (its lo
  // normal down to P ~ 2^-7) and spj undoes 2^(e_v + 4) with the projection's weight scale
  const float sq0 = wsc[0] * q_scale, sk0 = wsc[1], sv0 = wsc[2], csm = wsc[4];
  constexpr bool FOLD = C == 64;

  const int h = lane >> 5, lc = lane & 31;
  const int wg = blockIdx.x;
  const int gidx = wg * NW + wave;
  const bool active = gidx < total_groups;
  const int b = active ? gidx / groups_per_sample : 0;
  const int grp = active ? gidx % groups_per_sample : 0;
  const float* xb = x + (long)b * sb;
  float* ob = out + (long)b * osb;
  // diagnostic builds only (EXTDM_X3_DBG & 32): s_memtime stamps per wave into tstamp
  auto stamp = [&](int k) __attribute__((always_inline)) {
    if (tstamp != nullptr && lane == 0) tstamp[(long)gidx * 24 + k] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  const auto rs_x = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xb), 0, x_bytes, 0x00020000);
  const auto rs_o = __builtin_amdgcn_make_buffer_rsrc(ob, 0, o_bytes, 0x00020000);
  // a unit's weight slice by LDS-DMA, UL::HALVES / 512 pieces of 1 KiB spread over the
  // waves (a whole number each: static trip count)
  static_assert((UL::HALVES / 512) % NW == 0, "unit slice pieces per wave");
  auto load_unit = [&](int u, _Float16* dst) {
    const _Float16* src = wpk + (long)u * UL::HALVES;
#pragma unroll
    for (int i = 0; i < UL::HALVES / 512 / NW; ++i) {
      const int pc = wave + i * NW;
      __builtin_amdgcn_global_load_lds((const void*)(src + pc * 512 + lane * 8), (lds_ptr_t)(dst + pc * 512), 16, 0, 0);
    }
  };
  // PIPE: step j's slot = the q / k / v pieces of unit j and the proj pieces of unit j - 1
  // (pieces pc = wave + i * NW: the first 3 * KS pieces are q, k, v, the rest proj)
  constexpr bool PIPE = false;  // C == 64: measured 3-4 % slower than one unit per step (kept for A/B)
  auto load_step = [&](int j, _Float16* dst) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < UL::HALVES / 512 / NW; ++i) {
      const int pc = wave + i * NW;
      const bool is_qkv = pc < 3 * KS * 2;  // wave-uniform; static per (i, wave range)
      const int u = is_qkv ? j : j - 1;
      if (u < 0 || u >= UNITS) continue;
      __builtin_amdgcn_global_load_lds((const void*)(wpk + (long)u * UL::HALVES + pc * 512 + lane * 8),
                                       (lds_ptr_t)(dst + pc * 512), 16, 0, 0);
    }
  };
  if (PIPE) load_step(0, wsm);
  else load_unit(0, wsm);

  // ---- MODE 0 tile path (template TILE, host check attn_x3_tile_ok): the workgroup's 8 windows
  // are one row of 2x4x4 windows across W = 32 (no padding), so together they read
  // [C][2 frames x 4 rows][32] of x: 8 whole 128-B lines per channel. That tile is staged
  // into LDS by LDS-DMA (one 1-KiB instruction per channel), the lanes read their token's
  // channels from it, and the epilogue writes the layer output back into it and stores it
  // as whole lines — 8 coalesced instructions per wave each way instead of 32 per-lane dword
  // accesses that each touch 16 lines (the per-lane prologue / epilogue took ~30 % of the
  // kernel, s_memtime stamps). The residual is read from the tile, not from HBM again.
  // Layout [c][r = td*4 + th][32], the 16-B chunk q of row r stored at q ^ r: the 32 lanes of
  // a half-wave (8 rows x 4 columns of one channel) read 32 distinct banks ((a/4) mod 32 for
  // 4-B accesses; shifted windows straddle two chunks at complementary column offsets).
  static_assert(!TILE || (C == 64 && NW == 8), "tile path: C = 64, 8 waves");
  // T0: the MODE 0 tile above. T1: MODE 1 (temporal attention over PER = 16 frame slots, two
  // pixels per wave, or PER = 32, one pixel per wave; D <= PER frames): the workgroup's
  // 32 NW / PER consecutive pixels x PER frames x C, as [c][16-B chunk q][frame t][4 px] (one
  // 1-KiB LDS-DMA instruction per channel: lane l = (q = l / PER, t = l % PER) loads the 16 B of
  // pixels 4q .. 4q+3 of frame t; slots t >= D re-read frame D - 1 and are masked, never stored),
  // so the prologue reads x from LDS (2-way bank conflicts: frames t and t + 8 share banks), the
  // residual comes from the tile and the output leaves as 16-B row pieces; gamma and the inner
  // LayerNorm's w / b are in LDS too. (Round 5: PER = 32 and D < PER, for KTH's 30, SMMNIST's 20
  // and Cityscapes' 7 frames, whose per-lane loads touched one cache line per frame and channel.)
  // The per-lane path spent 31.7K of ~112K cycles per wave in the prologue (strided x loads and
  // per-element parameter loads) and 23.4K in the epilogue (s_memtime stamps, B = 64).
  constexpr bool T0 = TILE && MODE == 0, T1 = TILE && MODE == 1;
  float* const tileT = reinterpret_cast<float*>(wsm + 2 * UL::HALVES);
  // behind the tile: T0 gamma + proj bias, T1 gamma + LayerNorm w + b (192 floats)
  float* const parL = tileT + C * 256;
  const int PER = temporal_slots(g);                                       // T1: frame slots per pixel
  const int hw0 = T1 ? ((wg * NW) % groups_per_sample) * (32 / PER) : 0;  // T1: the workgroup's first pixel
  if (T1) {
    const int lt = lane % PER, lq = lane / PER;
    const long loff = (long)(lt < g.D ? lt : g.D - 1) * st + hw0 + 4 * lq;
#pragma unroll
    for (int i = 0; i < C / NW; ++i) {
      const int c = wave + i * NW;
      __builtin_amdgcn_global_load_lds((const void*)(xb + (long)c * sc + loff), (lds_ptr_t)(tileT + c * 256), 16, 0, 0);
    }
    if (wave == 0 && lane < 48)
      __builtin_amdgcn_global_load_lds((const void*)(lane < 16 ? gamma + 4 * lane
                                                     : (lane < 32 ? ln_w + 4 * (lane - 16) : ln_b + 4 * (lane - 32))),
                                       (lds_ptr_t)parL, 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // T1: this lane's (frame, pixel) in the tile: pixel pw of the workgroup, frame slot lc % PER
  const int t1pw = (32 / PER) * wave + lc / PER;
  const int t1idx = (t1pw >> 2) * (4 * PER) + (lc % PER) * 4 + (t1pw & 3);
  int trow[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // element offset of tile row r in a channel plane
  // rows of a padded frame (D odd, Dp = D + 1: frame D of the padded volume): loaded from frame D - 1
  // (any finite data: those tokens normalise to 0 like the reference's zero padding), never stored
  int rowpad = 0;
  if (T0) {
    const int grp0 = (wg * NW) % groups_per_sample;
    const int nWw = g.Wp / g.ws2, nWh = g.Hp / g.ws1;
    const int wh = (grp0 / nWw) % nWh, wd = grp0 / (nWw * nWh);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int fd = (wd * 2 + (r >> 2) + g.ss0) % g.Dp;
      rowpad |= (fd >= g.D ? 1 : 0) << r;
      trow[r] = (fd < g.D ? fd : g.D - 1) * (int)st + ((wh * 4 + (r & 3) + g.ss1) % g.Hp) * 32;
    }
    const int r = lane >> 3, q = (lane & 7) ^ r;
    int roff = trow[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) roff = r == i ? trow[i] : roff;
#pragma unroll
    for (int i = 0; i < C / NW; ++i) {
      const int c = wave + i * NW;
      __builtin_amdgcn_global_load_lds((const void*)(xb + (long)c * sc + roff + 4 * q), (lds_ptr_t)(tileT + c * 256),
                                       16, 0, 0);
    }
    // the norm's gamma and the projection bias behind the tile (lanes 0-15 / 16-31 of wave 0)
    if (wave == 0 && lane < 32)
      __builtin_amdgcn_global_load_lds((const void*)(lane < 16 ? gamma + 4 * lane : bp + 4 * (lane - 16)),
                                       (lds_ptr_t)(tileT + C * 256), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  stamp(20);
  // this lane's token in the tile (row lc >> 2, column 4 * window + tw + shift)
  const int tcol = (4 * wave + (lane & 3) + g.ss2) & 31;
  const int tidx = (lc >> 2) * 32 + (((tcol >> 2) ^ (lc >> 2)) << 2) + (tcol & 3);

  // window class of the bias / mask table (MODE 0 shifted layers): bit d for the last
  // window along a shifted dim d
  int pat = 0;
  if (T0 && npat > 1) {
    // the workgroup's row of windows: ww = wave, (wd, wh) of its first window
    const int grp0 = (wg * NW) % groups_per_sample;
    const int nWd = g.Dp / g.ws0, nWh = g.Hp / g.ws1;
    const int wh = (grp0 >> 3) % nWh, wd = (grp0 >> 3) / nWh;
    pat = (g.ss0 && wd == nWd - 1 ? 1 : 0) | (g.ss1 && wh == nWh - 1 ? 2 : 0) | (g.ss2 && wave == 7 ? 4 : 0);
  } else if (MODE == 0 && npat > 1) {
    const int nWd = g.Dp / g.ws0, nWh = g.Hp / g.ws1, nWw = g.Wp / g.ws2;
    const int ww = grp % nWw, wh = (grp / nWw) % nWh, wd = grp / (nWw * nWh);
    pat = (g.ss0 && wd == nWd - 1 ? 1 : 0) | (g.ss1 && wh == nWh - 1 ? 2 : 0) | (g.ss2 && ww == nWw - 1 ? 4 : 0);
  }
  // (wave-uniform: readfirstlane keeps the soffset in an SGPR — hipcc's divergence analysis
  // does not see through the window decomposition and would waterfall the loads)
  const int mb_lane = (lc * 32 + 4 * h) * 4, mb_wave = __builtin_amdgcn_readfirstlane(pat * 8 * 4096);

  // ---- 1. normalisation into register fragments ----
  Tok me;
  if (T0) {  // every token of a tile window exists; rows of a padded frame are not valid
    me.pos = 0; me.valid = ((rowpad >> (lc >> 2)) & 1) ? 0 : 1; me.exists = 1; me.lab = 0; me.rpos = lc;
  } else {
    me = token_of<MODE>(lc, g, st, grp);
  }
  const bool tok_ok = active && me.valid;
  const int vpro = tok_ok ? (int)((8 * h * sc + me.pos) * 4) : OOB;  // channel 8h + (16k + e)
  int bad = 0;
  h8 xh[KS], xl[KS];
  float m1 = 0.f, den1 = 1.f, rden1 = 1.f, gi = 1.f;
  // e_w reduction slots (NW floats) behind everything else the kernel keeps in LDS
  float* const redL = reinterpret_cast<float*>(wsm + 2 * UL::HALVES) + (TILE || PIPE ? C * 256 + 192 + 2048 : 0);
  {
    float xv[KS][8];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xv[k][e] = T0 ? tileT[(16 * k + 8 * h + e) * 256 + tidx]
                   : T1 ? tileT[(16 * k + 8 * h + e) * 256 + t1idx] : ldb(rs_x, vpro, (int)((16 * k + e) * sc * 4));
        s += xv[k][e];
      }
    s = xh_sum(s);
    m1 = s / C;
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = xv[k][e] - m1; v += d * d; }
    v = xh_sum(v);
    stamp(21);
    den1 = sqrtf(v / C + 1e-5f);
    // one reciprocal instead of a division per element (~10 VALU each, in the prologue and
    // MODE 1's epilogue): the product differs from the quotient by at most an ulp
    rden1 = 1.f / den1;
    // padded tokens (x loads 0 there) normalise to 0 through a 0 factor, not a select:
    // with a select hipcc sank each gamma load into a branch of its own, waited for it
    // there and so serialised 32 L2 round trips per wave
    const float vm = me.valid ? 1.f : 0.f;
    if (MODE == 0) {
      const float rv = rden1 * vm;
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          xv[k][e] = (xv[k][e] - m1) * rv * (T0 ? parL[16 * k + 8 * h + e] : ldb(rs_g, 32 * h, (16 * k + e) * 4));
    } else {
      float s2 = 0.f;
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          xv[k][e] = (xv[k][e] - m1) * rden1 * (T1 ? parL[16 * k + 8 * h + e] : ldb(rs_g, 32 * h, (16 * k + e) * 4));
          s2 += xv[k][e];
        }
      s2 = xh_sum(s2);
      const float m2 = s2 / C;
      float v2 = 0.f;
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) { const float d = xv[k][e] - m2; v2 += d * d; }
      v2 = xh_sum(v2);
      const float rstd2 = 1.0f / sqrtf(v2 / C + 1e-5f);
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          xv[k][e] = ((xv[k][e] - m2) * rstd2 * (T1 ? parL[64 + 16 * k + 8 * h + e] : ldb(rs_lw, 32 * h, (16 * k + e) * 4)) +
                      (T1 ? parL[128 + 16 * k + 8 * h + e] : ldb(rs_lb, 32 * h, (16 * k + e) * 4))) * vm;
    }
    // e_w: the largest |normalised value| to [2^8, 2^9) (a LayerNorm whose variance is below
    // its eps leaves the output far from unit scale, so this is data-dependent). On the tile
    // paths it is the workgroup's (wave 0 folds the q / k scales into the RoPE factors every
    // wave reads from LDS; a tile workgroup is one window row / pixel run of one sample); on the
    // per-lane path it is the wave's own: a wave owns one window or pixel set of one sample,
    // whereas that workgroup spans two samples when the groups per sample are not a multiple
    // of NW, and a sample's lo roundings must not depend on its batch neighbour (bitwise batch
    // independence). One barrier, which also retires every wave's tile reads before PIPE reuses
    // the tile.
    float am = 0.f;
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(xv[k][e]));
    am = xh_max(am);
#pragma unroll
    for (int off = 1; off < 32; off <<= 1) am = fmaxf(am, __shfl_xor(am, off));
    if (lane == 0) redL[wave] = am;
    __syncthreads();
    float wm = am;
    if (TILE || PIPE) {
      wm = redL[0];
#pragma unroll
      for (int i = 1; i < NW; ++i) wm = fmaxf(wm, redL[i]);
    }
    // largest at [2^8, 2^9): every value above 2^-11 of it keeps a normal lo
    int ew = wm > 0.f && wm < INFINITY ? 9 - __builtin_amdgcn_frexp_expf(wm) : 0;
    ew = ew < -100 ? -100 : (ew > 100 ? 100 : ew);
    const float gs = __builtin_amdgcn_ldexpf(1.f, ew);
    gi = __builtin_amdgcn_ldexpf(1.f, -ew);
#pragma unroll
    for (int k = 0; k < KS; ++k) {
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[k][e] *= gs;
      split8(xv[k], xh[k], xl[k], bad);
    }
  }
  const float sq = sq0 * gi, sk = sk0 * gi, sv = sv0 * gi;
  // PIPE: the normalised fragments go to LDS ([wave][k-step][hi|lo][lane][8], 8 KB per wave,
  // in the tile's place — every wave must be done reading the tile first) and are re-read
  // per unit: the 32 VGPRs they held are what the two units in flight need
  h8* const xfr = reinterpret_cast<h8*>(tileT) + wave * (KS * 2 * 64);
  if (PIPE) {
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      xfr[(2 * k) * 64 + lane] = xh[k];
      xfr[(2 * k + 1) * 64 + lane] = xl[k];
    }
  }
  stamp(22);

  f32x16 pacc[CT];
#pragma unroll
  for (int i = 0; i < CT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) pacc[i][r] = 0.f;

  // RoPE factors of this lane's (token, dim pair) registers, the same for every unit (with
  // the q / k scales folded in when FOLD); reloaded per group rather than kept live through
  // the prologue. Folded at C = 64 only: at C = 128 (one wave per SIMD) the 16 extra live
  // registers cost 20 % (interleaved A/B)
  float rcq[8], rsq[8], rck[8], rsk[8];
#pragma unroll
  for (int r = 0; r < 16; r += 2) {
    const int pi = (dof(r, h) % DH) >> 1;
    const float c = rcos[me.rpos * RH + pi], sn = rsin[me.rpos * RH + pi];
    rcq[r >> 1] = FOLD ? c * sq : c; rsq[r >> 1] = FOLD ? sn * sq : sn;
    rck[r >> 1] = FOLD ? c * sk : c; rsk[r >> 1] = FOLD ? sn * sk : sn;
  }
  // tile path: the factors (the same in every wave: token = lane) go to LDS as [8 float4][64
  // lanes] and are re-read per unit (8 conflict-free ds_read_b128) instead of holding 32
  // VGPRs through the unit loop
  float4* const ropeL = reinterpret_cast<float4*>(tileT + C * 256 + 192);
  if ((TILE || PIPE) && wave == 0) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      ropeL[(0 + j) * 64 + lane] = make_float4(rcq[4 * j], rcq[4 * j + 1], rcq[4 * j + 2], rcq[4 * j + 3]);
      ropeL[(2 + j) * 64 + lane] = make_float4(rsq[4 * j], rsq[4 * j + 1], rsq[4 * j + 2], rsq[4 * j + 3]);
      ropeL[(4 + j) * 64 + lane] = make_float4(rck[4 * j], rck[4 * j + 1], rck[4 * j + 2], rck[4 * j + 3]);
      ropeL[(6 + j) * 64 + lane] = make_float4(rsk[4 * j], rsk[4 * j + 1], rsk[4 * j + 2], rsk[4 * j + 3]);
    }
  }

  // ---- 2. per unit of 32 qkv rows ----
  // Q^T, K^T (rows = dims, lane = token) from the unit slice W
  auto qk_mfma = [&](const _Float16* W, f32x16& q, f32x16& k) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) { q[r] = 0.f; k[r] = 0.f; }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const _Float16* fq = W + UL::Q + s * UL::FRAG + lane * 8;
      const _Float16* fk = W + UL::K + s * UL::FRAG + lane * 8;
      q = mma3(*reinterpret_cast<const h8*>(fq), *reinterpret_cast<const h8*>(fq + 512), xh[s], xl[s], q);
      k = mma3(*reinterpret_cast<const h8*>(fk), *reinterpret_cast<const h8*>(fk + 512), xh[s], xl[s], k);
    }
  };
  // V (rows = tokens, lane = dim)
  auto v_mfma = [&](const _Float16* W, f32x16& v) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const _Float16* fv = W + UL::V + s * UL::FRAG + lane * 8;
      v = mma3(xh[s], xl[s], *reinterpret_cast<const h8*>(fv), *reinterpret_cast<const h8*>(fv + 512), v);
    }
  };
  // Q^T, K^T first, the next k-step's four fragments read from LDS while this step's six
  // MFMAs run (sched_barrier pins the order: left alone, hipcc issued each fragment pair
  // right before its MFMAs and waited for it, exposing the LDS latency 8x per unit)
  auto qkv_mfma = [&](const _Float16* W, f32x16& q, f32x16& k, f32x16& v) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) { q[r] = 0.f; k[r] = 0.f; }
    h8 fr[2][4];
    auto ld = [&](int s, h8* f) __attribute__((always_inline)) {
      const _Float16* fq = W + UL::Q + s * UL::FRAG + lane * 8;
      const _Float16* fk = W + UL::K + s * UL::FRAG + lane * 8;
      f[0] = *reinterpret_cast<const h8*>(fq); f[1] = *reinterpret_cast<const h8*>(fq + 512);
      f[2] = *reinterpret_cast<const h8*>(fk); f[3] = *reinterpret_cast<const h8*>(fk + 512);
    };
    ld(0, fr[0]);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (s + 1 < KS) ld(s + 1, fr[(s + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      const h8* f = fr[s & 1];
      q = mma3(f[0], f[1], xh[s], xl[s], q);
      k = mma3(f[2], f[3], xh[s], xl[s], k);
      __builtin_amdgcn_sched_barrier(0);
    }
    // V's MFMAs left to the scheduler, which can place the RoPE / split VALU of q, k (which
    // follows in program order and does not depend on V) between them
    v_mfma(W, v);
  };
  // the bias / mask rows of unit u's heads (added to the scores in attend)
  auto load_bias = [&](int u, f32x16* bia) __attribute__((always_inline)) {
#pragma unroll
    for (int hh = 0; hh < HPU; ++hh)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const auto v4 = __builtin_amdgcn_raw_buffer_load_b128(rs_mb, mb_lane + 32 * q, mb_wave + (u * HPU + hh) * 4096, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e) bia[hh][4 * q + e] = __uint_as_float(v4[e]);
      }
  };
  // scale + RoPE of q, k; the unit's heads: S^T = bias + K Q^T (rows = keys j, lane =
  // query i), softmax, O^T = V^T P^T
  auto attend = [&](f32x16& q, f32x16& k, const f32x16& v, const f32x16* bia) __attribute__((always_inline)) {
    if (TILE || PIPE) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float4 a = ropeL[(0 + j) * 64 + lane], bq = ropeL[(2 + j) * 64 + lane];
        const float4 ck = ropeL[(4 + j) * 64 + lane], dk = ropeL[(6 + j) * 64 + lane];
        rcq[4 * j] = a.x; rcq[4 * j + 1] = a.y; rcq[4 * j + 2] = a.z; rcq[4 * j + 3] = a.w;
        rsq[4 * j] = bq.x; rsq[4 * j + 1] = bq.y; rsq[4 * j + 2] = bq.z; rsq[4 * j + 3] = bq.w;
        rck[4 * j] = ck.x; rck[4 * j + 1] = ck.y; rck[4 * j + 2] = ck.z; rck[4 * j + 3] = ck.w;
        rsk[4 * j] = dk.x; rsk[4 * j + 1] = dk.y; rsk[4 * j + 2] = dk.z; rsk[4 * j + 3] = dk.w;
      }
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
    Op<BF> qf[2], kf[2], vf[2];  // [k-step]
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float tq[8], tk[8], tv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { tq[e] = q[8 * s + e]; tk[e] = k[8 * s + e]; tv[e] = v[8 * s + e] * sv; }
      qf[s].set(tq, bad);
      kf[s].set(tk, bad);
      vf[s].set(tv, bad);
    }
    f32x16 o;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = 0.f;
#pragma unroll
    for (int hh = 0; hh < HPU; ++hh) {
      // K Q^T from zero, then the bias / mask in one add: accumulated onto the bias, every
      // MFMA of the chain rounded at the bias's ulp (one rounding, as the reference's
      // qk^T + bias, where the bias dominates small activations)
      f32x16 sc_;
#pragma unroll
      for (int r = 0; r < 16; ++r) sc_[r] = 0.f;
#pragma unroll
      for (int s = 0; s < 2; ++s)
        if (HPU == 1 || s == hh) sc_ = mmo(kf[s], qf[s], sc_);
#pragma unroll
      for (int r = 0; r < 16; ++r) sc_[r] += bia[hh][r];
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc_[r]);
      mx = xh_max(mx);
      // exp(s - mx) as v_exp_f32 (2^x) of fma(s, log2 e, -mx log2 e): masked -inf -> 0
      const float mxl = mx * csm;
      float sum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sc_[r] = __builtin_amdgcn_exp2f(fmaf(sc_[r], csm, -mxl));
        sum += sc_[r];
      }
      sum = xh_sum(sum);
      const float inv = 16.f / sum;  // P * 2^4 (wsc header note)
#pragma unroll
      for (int r = 0; r < 16; ++r) sc_[r] *= inv;
      // O^T[dd][i] = sum_j V^T[dd][j] P^T[j][i]; lanes of the unit's other head masked
      const bool mine = HPU == 1 || (lc / DH) == hh;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float tp[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) tp[e] = sc_[8 * s + e];
        Op<BF> pf, va = vf[s];
        pf.set(tp, bad);
        if (!mine) va.zero();
        o = mmo(va, pf, o);
      }
    }
    return o;
  };
  // projection: Y[c][i] += sum_dd Wp[c][u*32 + dd] O^T[dd][i]
  auto proj = [&](const _Float16* W, const f32x16& o) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float to[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) to[e] = o[8 * s + e];
      h8 oh, ol;
      split8<false>(to, oh, ol, bad);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const _Float16* fp = W + UL::P + (ct * 2 + s) * UL::FRAG + lane * 8;
        pacc[ct] = mma3(*reinterpret_cast<const h8*>(fp), *reinterpret_cast<const h8*>(fp + 512), oh, ol, pacc[ct]);
      }
    }
  };
  // unit u's slice has landed in every wave's pieces: LDS-DMA completion is tracked by
  // the issuing wave's vmcnt only, so each wave drains it before the barrier
  auto unit_barrier = [&](int u) __attribute__((always_inline)) {
    stamp(2 + 2 * u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stamp(3 + 2 * u);
  };
  stamp(1);
  if (dbg & 16) {
    // timing only: no unit loop (prologue + epilogue cost)
  } else if (PIPE) {
    // Software-pipelined units (C = 64, two waves per SIMD): step j runs the qkv MFMAs of
    // unit j beside the RoPE / splits / softmax / PV / projection of unit j - 1, so the
    // MFMA pipe has independent work while the attention VALU runs (with one unit per step
    // both waves of a SIMD reached their VALU phases together and the pipe idled). Ring
    // slot j holds [qkv(j) | proj(j - 1)] (load_step), so two 32-KB slots still suffice.
    f32x16 q, k, v;
#pragma unroll
    for (int r = 0; r < 16; ++r) { q[r] = 0.f; k[r] = 0.f; v[r] = 0.f; }
#pragma unroll
    for (int j = 0; j <= UNITS; ++j) {
      _Float16* W = wsm + (j & 1) * UL::HALVES;
      unit_barrier(j);
      f32x16 bia[HPU];
      if (j >= 1) load_bias(j - 1, bia);
      if (j + 1 <= UNITS) load_step(j + 1, wsm + ((j + 1) & 1) * UL::HALVES);
      if (T0 && j == UNITS) {
        // the x tile again for the residual epilogue, into the fragments' place (no wave reads
        // them after step UNITS - 1): in flight during the last unit's attention
        const int r = lane >> 3, qq = (lane & 7) ^ r;
        int roff = trow[0];
#pragma unroll
        for (int i = 1; i < 8; ++i) roff = r == i ? trow[i] : roff;
#pragma unroll
        for (int i = 0; i < C / NW; ++i) {
          const int c = wave + i * NW;
          __builtin_amdgcn_global_load_lds((const void*)(xb + (long)c * sc + roff + 4 * qq),
                                           (lds_ptr_t)(tileT + c * 256), 16, 0, 0);
        }
      }
      f32x16 qn, kn, vn;
      if (j < UNITS) {
        // per k-step: the wave's X fragments from LDS, then q, k, v's three MFMAs each
#pragma unroll
        for (int r = 0; r < 16; ++r) { qn[r] = 0.f; kn[r] = 0.f; vn[r] = 0.f; }
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const h8 xhs = xfr[(2 * s) * 64 + lane], xls = xfr[(2 * s + 1) * 64 + lane];
          const _Float16* fq = W + UL::Q + s * UL::FRAG + lane * 8;
          const _Float16* fk = W + UL::K + s * UL::FRAG + lane * 8;
          const _Float16* fv = W + UL::V + s * UL::FRAG + lane * 8;
          qn = mma3(*reinterpret_cast<const h8*>(fq), *reinterpret_cast<const h8*>(fq + 512), xhs, xls, qn);
          kn = mma3(*reinterpret_cast<const h8*>(fk), *reinterpret_cast<const h8*>(fk + 512), xhs, xls, kn);
          vn = mma3(xhs, xls, *reinterpret_cast<const h8*>(fv), *reinterpret_cast<const h8*>(fv + 512), vn);
        }
      }
      if (j >= 1) {
        const f32x16 o = attend(q, k, v, bia);
        proj(W, o);
      }
      if (j < UNITS) { q = qn; k = kn; v = vn; }
    }
  } else {
    for (int u = 0; u < UNITS; ++u) {
      _Float16* W = wsm + (u & 1) * UL::HALVES;
      unit_barrier(u);  // ... and slot (u+1)&1 is free
      // the unit's bias / mask rows, issued ahead of the next unit's weight DMA: vmcnt
      // counts in issue order, so waiting for them does not wait for the DMA
      f32x16 bia[HPU];
      load_bias(u, bia);
      if (u + 1 < UNITS) load_unit(u + 1, wsm + ((u + 1) & 1) * UL::HALVES);
      if (!active) continue;
      f32x16 q, k, v;
      if (TILE) {
        qkv_mfma(W, q, k, v);
      } else {
        qk_mfma(W, q, k);
        v_mfma(W, v);
      }
      const f32x16 o = attend(q, k, v, bia);
      proj(W, o);
    }
  }
  stamp(18);
  if (TILE && PIPE && !(dbg & 16)) {  // the re-loaded x tile (every wave's pieces) has landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // the loop's splits: one finite check of the token's accumulators (see split8)
  {
    float chk = 0.f;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) chk += pacc[ct][r];
    bad |= tok_ok && !__builtin_isfinite(chk);
  }
  if (bad) atomicOr(range_flag, 2);
  // MODE 1 with 2-pixel groups: a lane's token is (pixel, frame), so a direct store touches
  // 16 frame planes per instruction, 8 bytes each, and every 64-B line is written by 8
  // waves. Instead the workgroup's 16 consecutive pixels x D frames x C channels go through
  // LDS ([c][t][16 px], rows padded for conflict-free lane writes) and leave as 64-B rows.
  const bool lds_epi = !T1 && MODE == 1 && C == 64 && NW == 8 && temporal_slots(g) == 16 && groups_per_sample % NW == 0 &&
                       (g.H * g.W) % 16 == 0 && (osc & 3) == 0 && (st & 3) == 0 && (((uintptr_t)out) & 15) == 0;
  if (T1) {
    // residual from the tile, the result back into it (each (channel, frame, pixel) is one
    // lane's), then the tile leaves as 16-B pieces (the DMA's mapping in reverse)
    const float spj = wsc[3];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ch = ct * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        float* tp = tileT + ch * 256 + t1idx;
        const float xv = *tp;
        *tp = pacc[ct][r] * spj + (xv + (xv - m1) * rden1 * parL[ch]);
      }
    __syncthreads();
    float* o0 = ob + hw0;
    const int lt = lane % PER, lq = lane / PER;  // id & 63 == lane below (NW * 64 is a multiple of 64)
#pragma unroll
    for (int i = 0; i < C * 64 / (NW * 64); ++i) {
      const int id = tid + i * NW * 64;
      const int c = id >> 6;
      const float4 v = *reinterpret_cast<const float4*>(tileT + c * 256 + 4 * lane);
      if (lt < g.D) *reinterpret_cast<float4*>(o0 + (long)c * osc + (long)lt * st + 4 * lq) = v;
    }
    stamp(19);
  } else if (MODE == 1 && lds_epi) {
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
    if (active) {
      const int hw0 = (wg * NW) % groups_per_sample * 2;
      float* o0 = ob + hw0;
      for (int i = tid; i < C * g.D * 4; i += NW * 64) {
        const int q = i & 3, ctr = i >> 2;
        const int t = ctr % g.D, c = ctr / g.D;
        const float4 v = *reinterpret_cast<const float4*>(T + c * CS + t * RS + 4 * q);
        *reinterpret_cast<float4*>(o0 + (long)c * osc + (long)t * st + 4 * q) = v;
      }
    }
    stamp(19);
  } else if (active && me.valid) {
    if (dbg & 8) {  // timing only: no epilogue loads / stores (one store keeps the work live)
      float acc = 0.f;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc += pacc[ct][r];
      if (acc == 12345.f) ob[me.pos] = acc;
    } else {
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
          // MODE 0: proj bias; MODE 1: gamma
          const float pb = T0 ? parL[64 + cu + 4 * h] : ldb(rs_b, 16 * h, cu * 4);
          const float y = pacc[ct][r] * spj;
          if (T0) {
            // residual from the tile, the result back into it (each (channel, token) is one lane's)
            float* tp = tileT + (cu + 4 * h) * 256 + tidx;
            *tp = (y + pb) + *tp;
          } else {
            const float xv = ldb(rs_x, vex, (int)(cu * sc * 4));
            float res;
            if (MODE == 0) res = (y + pb) + xv;
            else res = y + (xv + (xv - m1) * rden1 * pb);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(res), rs_o, veo, (int)(cu * osc * 4), 0);
          }
        }
      }
    }
    stamp(19);
  }
  if (T0) {
    // the tile leaves as whole 128-B lines: chunk id -> (channel, row, stored chunk), its
    // global chunk undoes the row's swizzle
    __syncthreads();
#pragma unroll
    for (int j = 0; j < C * 64 / (NW * 64); ++j) {
      const int id = tid + j * NW * 64;
      const int c = id >> 6, r = (id >> 3) & 7, qs = id & 7;
      int roff = trow[0];
#pragma unroll
      for (int i = 1; i < 8; ++i) roff = r == i ? trow[i] : roff;
      const float4 v = *reinterpret_cast<const float4*>(tileT + c * 256 + r * 32 + qs * 4);
      if (!((rowpad >> r) & 1)) *reinterpret_cast<float4*>(ob + (long)c * osc + roff + 4 * (qs ^ r)) = v;
    }
  }
}

// The MODE 1 tile path (kernel, T1): D <= 32 frames (16 or 32 slots per pixel), whole workgroups
// of 16 / 8 pixels inside a sample, 16-B aligned rows; x and out share their channel / frame
// strides (temporal_x3). EXTDM_X3_TILE1_16=1: only D = 16, the round-4 scope (A/B).
bool attn_x3_tile1_ok(const View& x, const View& out, const AttnGeom& g, int groups) {
  static const bool off = [] { const char* v = getenv("EXTDM_X3_NO_TILE"); return v && v[0] && v[0] != '0'; }();
  static const bool only16 = [] { const char* v = getenv("EXTDM_X3_TILE1_16"); return v && v[0] && v[0] != '0'; }();
  const int per = temporal_slots(g);
  return !off && g.mode == 1 && g.D >= 1 && g.D <= 32 && (!only16 || g.D == 16) && (g.H * g.W) % (256 / per) == 0 &&
         groups % 8 == 0 && x.st == (long)x.H * x.W &&
         x.st % 4 == 0 && x.sc % 4 == 0 && x.sb % 4 == 0 && out.sc % 4 == 0 && out.sb % 4 == 0 && out.st == x.st &&
         ((uintptr_t)x.p & 15) == 0 && ((uintptr_t)out.p & 15) == 0;
}

// The MODE 0 tile path (kernel header, "tile path"): 2x4x4 windows over W = 32 without
// padding, so that a workgroup's 8 windows are one row of windows; 16-B aligned rows;
// in place (x and out the same view).
bool attn_x3_tile_ok(const View& x, const View& out, const AttnGeom& g, int groups) {
  static const bool off = [] { const char* v = getenv("EXTDM_X3_NO_TILE"); return v && v[0] && v[0] != '0'; }();
  return !off && g.mode == 0 && g.ws0 == 2 && g.ws1 == 4 && g.ws2 == 4 && g.W == 32 && g.Wp == 32 && g.H == g.Hp &&
         g.D >= 1 && g.Dp <= g.D + 1 && groups % 8 == 0 && x.p == out.p && x.sc == out.sc && x.sb == out.sb && x.st == out.st &&
         x.st == (long)x.H * x.W && x.sc % 4 == 0 && x.sb % 4 == 0 && ((uintptr_t)x.p & 15) == 0;
}

template <int C, int MODE, int DH, int NW, bool BF>
void launch_nw(hipStream_t s, const View& x, const View& out, const AttnGeom& g, int groups, const float* gamma,
               const float* lw, const float* lb, const void* wpk, const float* wsc, const float* bp,
               const float* mbias, int npat, const float* rcos, const float* rsin, float q_scale) {
  static const int dbg = [] { const char* v = getenv("EXTDM_X3_DBG"); return v ? atoi(v) : 0; }();
  // MODE 1 at C = 64, 8 waves: the epilogue's [C][16 frames][16 px] staging tile (rows of
  // 20, channels of 328 floats) reuses the ring
  const size_t ring = (size_t)2 * UnitLayout<C>::HALVES * sizeof(_Float16);
  const bool tile = C == 64 && NW == 8 &&
                    (MODE == 0 ? attn_x3_tile_ok(x, out, g, groups) : attn_x3_tile1_ok(x, out, g, groups));
  size_t lds = (MODE == 1 && C == 64 && NW == 8) ? std::max(ring, (size_t)C * 328 * sizeof(float)) : ring;
  // tile / C = 64: behind the ring the x tile (C * 256 floats), 192 floats of norm / bias
  // parameters, the RoPE factors (8 x 64 float4), then the e_w reduction slots (MODE 1's
  // non-tile epilogue staging may overlap them: dead by then)
  const size_t behind = (tile || C == 64) ? (size_t)C * 8 * 32 + 192 + 8 * 64 * 4 : 0;
  lds = std::max(lds, ring + (behind + NW) * sizeof(float));
  // per device, once: the dynamic-LDS limit
  static std::once_flag once[64];
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::call_once(once[dev & 63], [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_x3_kernel<C, MODE, DH, NW, false, BF>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (C == 64 && NW == 8)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_x3_kernel<C, MODE, DH, NW, C == 64 && NW == 8, BF>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  });
  const int total = x.B * groups;
  const int grid = (total + NW - 1) / NW;
  long long* ts = nullptr;
  if (dbg & 32) {  // diagnostic: per-wave s_memtime stamps, mean phase durations to stderr
    (void)hipMalloc(&ts, (size_t)total * 24 * sizeof(long long));
    (void)hipMemsetAsync(ts, 0, (size_t)total * 24 * sizeof(long long), s);
  }
  constexpr bool TILE_OK = C == 64 && NW == 8;
  // EXTDM_X3_TILE_DBG=1 (diagnostic): the route's geometry per launch to stderr
  static const bool tdbg = getenv("EXTDM_X3_TILE_DBG") != nullptr;
  if (tdbg)
    fprintf(stderr, "attn_x3 MODE %d C %d tile %d: D %d Dp %d H %d Hp %d W %d Wp %d ws %d %d %d groups %d sc %ld sb %ld st %ld p %p\n",
            MODE, C, (int)tile, g.D, g.Dp, g.H, g.Hp, g.W, g.Wp, g.ws0, g.ws1, g.ws2, groups, x.sc, x.sb, x.st, (void*)x.p);
  auto kern = tile ? &attn_x3_kernel<C, MODE, DH, NW, TILE_OK, BF> : &attn_x3_kernel<C, MODE, DH, NW, false, BF>;
  note_kernel("attn_x3_kernel<%d, %d, %d, %d, %s, %s>", C, MODE, DH, NW, tile && TILE_OK ? "true" : "false",
              BF ? "true" : "false");
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NW * 64), lds, s, x.p, out.p, x.sb, x.sc, x.st, out.sb, out.sc, g, gamma,
                     lw, lb, reinterpret_cast<const _Float16*>(wpk), wsc, bp, mbias, npat, rcos, rsin, q_scale, groups,
                     total, x3_range_ptr(), dbg, ts);
  if (ts) {
    std::vector<long long> h((size_t)total * 24);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), ts, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
    (void)hipFree(ts);
    double acc[24] = {0};
    long n = 0;
    for (int w = 0; w < total; ++w) {
      const long long* t = &h[(size_t)w * 24];
      if (t[0] == 0 || t[19] == 0) continue;
      ++n;
      for (int k = 1; k < 20; ++k) acc[k] += (double)(t[k] - t[k - 1]);
    }
    fprintf(stderr, "attn_x3<C=%d,MODE=%d,DH=%d,NW=%d,BF> stamps over %ld waves (cycles): prologue %.0f", C, MODE, DH, NW, n,
            acc[1] / n);
    for (int u = 0; u < 8; ++u) fprintf(stderr, " | u%d wait %.0f body %.0f", u, acc[3 + 2 * u] / n, acc[4 + 2 * u] / n);
    fprintf(stderr, " | tail %.0f epilogue %.0f", acc[18] / n, acc[19] / n);
    double p[4] = {0, 0, 0, 0};  // prologue: tile wait / LN statistics / normalise + split / rest
    for (int w = 0; w < total; ++w) {
      const long long* t = &h[(size_t)w * 24];
      if (t[0] == 0 || t[19] == 0 || t[20] == 0) continue;
      p[0] += (double)(t[20] - t[0]); p[1] += (double)(t[21] - t[20]); p[2] += (double)(t[22] - t[21]);
      p[3] += (double)(t[1] - t[22]);
    }
    fprintf(stderr, " || prologue: tile-wait %.0f stats %.0f norm+split %.0f rope+rest %.0f\n", p[0] / n, p[1] / n,
            p[2] / n, p[3] / n);
  }
}

template <int C, int MODE, int DH, bool BF>
void launch(hipStream_t s, const View& x, const View& out, const AttnGeom& g, int groups, const float* gamma,
            const float* lw, const float* lb, const void* wpk, const float* wsc, const float* bp,
            const float* mbias, int npat, const float* rcos, const float* rsin, float q_scale) {
  static const int nw = [] { const char* v = getenv("EXTDM_X3_ATTN_NW"); return v ? atoi(v) : 0; }();
  // C = 128 needs > 256 VGPRs: one wave per SIMD
  if (C == 64 && nw != 4)
    launch_nw<C, MODE, DH, 8, BF>(s, x, out, g, groups, gamma, lw, lb, wpk, wsc, bp, mbias, npat, rcos, rsin, q_scale);
  else
    launch_nw<C, MODE, DH, 4, BF>(s, x, out, g, groups, gamma, lw, lb, wpk, wsc, bp, mbias, npat, rcos, rsin, q_scale);
}

// bf16: the BF16_ATTN attention core, instantiated for dim_head 32 (attn_x3_supported)
template <int MODE, int DH>
bool dispatch_c(hipStream_t s, const View& x, const View& out, const AttnGeom& g, int groups, const float* gamma,
                const float* lw, const float* lb, const void* wpk, const float* wsc, const float* bp,
                const float* mbias, int npat, const float* rcos, const float* rsin, float q_scale, bool bf16) {
  if constexpr (DH == 32) {
    if (bf16) {
      if (x.C == 64) launch<64, MODE, DH, true>(s, x, out, g, groups, gamma, lw, lb, wpk, wsc, bp, mbias, npat, rcos, rsin, q_scale);
      else if (x.C == 128) launch<128, MODE, DH, true>(s, x, out, g, groups, gamma, lw, lb, wpk, wsc, bp, mbias, npat, rcos, rsin, q_scale);
      else return false;
      return true;
    }
  } else {
    if (bf16) return false;
  }
  if (x.C == 64) launch<64, MODE, DH, false>(s, x, out, g, groups, gamma, lw, lb, wpk, wsc, bp, mbias, npat, rcos, rsin, q_scale);
  else if (x.C == 128) launch<128, MODE, DH, false>(s, x, out, g, groups, gamma, lw, lb, wpk, wsc, bp, mbias, npat, rcos, rsin, q_scale);
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
            const void* wpk, const float* wsc, const float* bp, const float* mbias, int npat,
            const float* rcos, const float* rsin, float q_scale, bool bf16) {
  const int N = g.ws0 * g.ws1 * g.ws2;
  if (!attn_x3_supported(x.C, N, dim_head, heads) || !extent_ok(x, g)) return false;
  const int groups = (g.Dp / g.ws0) * (g.Hp / g.ws1) * (g.Wp / g.ws2);
  if (dim_head == 32)
    return dispatch_c<0, 32>(s, x, x, g, groups, gamma, nullptr, nullptr, wpk, wsc, bp, mbias, npat, rcos,
                             rsin, q_scale, bf16);
  return dispatch_c<0, 16>(s, x, x, g, groups, gamma, nullptr, nullptr, wpk, wsc, bp, mbias, npat, rcos, rsin,
                           q_scale, bf16);
}

bool temporal_x3(hipStream_t s, const View& x, const View& out, const AttnGeom& g, int heads, int dim_head,
                 const float* gamma, const float* ln_w, const float* ln_b, const void* wpk, const float* wsc,
                 const float* mbias, const float* rcos, const float* rsin, float q_scale, bool bf16) {
  const int npat = 1;
  if (!attn_x3_supported(x.C, g.D, dim_head, heads) || g.D > 32 || !extent_ok(x, g) || !extent_ok(out, g)) return false;
  if (out.sc != x.sc || out.st != x.st) return false;
  const int ppb = 32 / temporal_slots(g);
  const int groups = (g.H * g.W + ppb - 1) / ppb;
  if (dim_head == 32)
    return dispatch_c<1, 32>(s, x, out, g, groups, gamma, ln_w, ln_b, wpk, wsc, nullptr, mbias, npat, rcos,
                             rsin, q_scale, bf16);
  return dispatch_c<1, 16>(s, x, out, g, groups, gamma, ln_w, ln_b, wpk, wsc, nullptr, mbias, npat, rcos, rsin,
                           q_scale, bf16);
}

}  // namespace extdm
