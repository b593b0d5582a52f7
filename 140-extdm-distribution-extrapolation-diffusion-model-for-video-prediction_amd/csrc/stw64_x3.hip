// Fused Residual(PreNorm(STWAttentionLayer)) over 3-D windows of up to 64 tokens: the
// ada / ada_u22 denoisers' 4x4x4 windows (…_ada.py:408-559, …_ada_u22.py:531-700; the
// layer as u12:138-158, 408-559, 961-963), in place on x:
//   x[:, win] += proj(attn(qkv(chanLN(x[:, win])))) + b
// qkv and proj run on f16x3 MFMA (three v_mfma_f32_32x32x16_f16 per fp32 product, the
// convention of stw_x3.hip); the attention contractions QK^T and PV run either as f16x3
// (BF = false, EXTDM_PRECISION_F16X3: fp32-faithful) or on v_mfma_f32_32x32x16_bf16
// (BF = true, EXTDM_PRECISION_BF16_ATTN: q, k, v and the probabilities rounded to bf16,
// fp32 accumulation — the UCF-101 256 configuration's "bf16 MFMA attention").
//
// A window is two WAVES, each owning one 32-token tile (tokens 32 tt .. 32 tt + 31 of the
// window, tt = wave & 1); a workgroup holds NW / 2 windows. Per wave (lane = token lc, half h):
//  1. the lane loads exactly the channels of its MFMA k-slices (16 s + 8 h + e) of its token,
//     channel-LayerNorms them (mean / variance over the two halves), scales them by the
//     wave's power of two and keeps them as fp16 hi / lo fragments in registers;
//  2. per unit of 32 qkv rows (one dim-32 head or two dim-16 heads), the unit's packed weights
//     (the stw_x3.hip layout, packed_attn_x3) arriving through a two-slot LDS-DMA ring:
//       Q^T, K^T = Wq Xn^T, Wk Xn^T (rows = head dims, lane = token), V = Xn Wv^T
//       scale + RoPE (rotary position = window token index), split into MFMA operands;
//     the wave's K and V operand fragments go to LDS (8 KB per wave; bf16: 4 KB), one
//     barrier, and each wave then reads the K / V fragments of BOTH tiles of its window:
//       S^T[kt] = K[kt] Q^T + bias          (kt = 0, 1: 64 keys x the wave's 32 queries)
//       softmax over the 64 keys (in-lane over 32 registers, then the partner half lane ^ 32)
//       O^T    = sum_kt V[kt]^T P[kt]^T    (P^T straight from the score registers)
//       Y     += Wp O^T                    (projection accumulators, C / 32 tiles)
//     nothing of q, k, v, the scores or O touches HBM;
//  3. epilogue: Y + bias + residual to the token's positions (buffer stores; padded tokens'
//     offsets lie past the descriptor's extent).
// Bias + masks: one table [npat][8 heads][64 queries][64 keys] per layer (stw_mask_bias64,
// runtime.cpp): the dense relative-position bias, -100 where a shifted window's region labels
// differ (u12:414-436), -inf for keys past the window's N tokens, times the scores' factor
// 2^(e_q + e_k) (stw_x3.hip operand-scale note). A lane reads its query's row: 4 x 16-B
// pieces per key tile and head.
#include <algorithm>
#include <cstdlib>
#include <mutex>

#include "attn_x3_ops.h"

namespace extdm {

namespace {

using namespace attn_ops;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// Packed unit slice (halves) — the stw_x3.hip layout (attn_x3_unit_halves): [q: C/16 frags]
// [k: C/16][v: C/16][proj: C/32 tiles x 2 k-steps], each frag = [hi|lo][64 lanes][8]
template <int C>
struct UL64 {
  static constexpr int KS = C / 16;
  static constexpr int FRAG = 2 * 512;
  static constexpr int Q = 0, K = KS * FRAG, V = 2 * KS * FRAG, P = 3 * KS * FRAG;
  static constexpr int HALVES = 3 * KS * FRAG + (C / 32) * 2 * FRAG;
};

// TILE (host check stw64_tile_ok; C = 64 on 8 waves): the workgroup's NW / 2 windows are consecutive
// along W (one (wd, wh) window row, W a multiple of 16, no H / W padding), so together they cover
// C x 4 frames x 4 rows x 16 columns of x. That block is staged once into LDS by coalesced 8-B
// loads per lane (each 64-B row segment read by 8 adjacent lanes; a shifted row wraps only between
// 8-B pieces), the lanes read their token's channels from it (row stride 20, channel stride 324
// floats: the 32 tokens of a half-wave hit 32 banks, the two halves the other 32), and the epilogue
// writes Y + bias back into it and leaves as the same 8-B pieces plus the residual — instead of
// per-lane 4-B accesses that touch 16 lines per instruction (the per-lane prologue and epilogue
// took 40-55 % of the kernel: EXTDM_STW64_DBG knock-outs, KTH / UCF level 0). The tile aliases the
// K / V exchange region (used only inside the unit loop).
template <int C, int DH, int NW, bool BF, bool TILE>
__global__ __launch_bounds__(NW * 64) void stw64_x3_kernel(float* x, long sb, long sc, long st, AttnGeom g,
                                                           const float* __restrict__ gamma,
                                                           const _Float16* __restrict__ wpk,
                                                           const float* __restrict__ wsc,  // 2^-s: q, k, v, proj, exp2
                                                           const float* __restrict__ bp,
                                                           const float* __restrict__ mbias, int npat,
                                                           const float* __restrict__ rcos,
                                                           const float* __restrict__ rsin, float q_scale,
                                                           int groups_per_sample, int total_groups,
                                                           int* __restrict__ range_flag, int dbg) {
  using UL = UL64<C>;
  constexpr int KS = UL::KS;
  constexpr int UNITS = 8 * DH / 32;  // heads 8
  constexpr int HPU = 32 / DH;
  constexpr int RH = DH / 2;
  constexpr int CT = C / 32;
  constexpr int XS = 2 * 2 * Op<BF>::SLOTS;  // exchange slots per lane: K and V, 2 k-steps
  constexpr bool FOLD = C == 64;             // q / k scales folded into the RoPE factors
  extern __shared__ __attribute__((aligned(16))) _Float16 wsm[];
  h8* const xch = reinterpret_cast<h8*>(wsm + 2 * UL::HALVES);  // [NW][XS][64 lanes]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tt = wave & 1;
  const int h = lane >> 5, lc = lane & 31;
  // XCD-contiguous workgroup order (grid a multiple of 8, host): workgroup b runs on XCD b mod 8 and
  // takes logical slot (b mod 8) G / 8 + b / 8, so the workgroups whose tiles share 128-B output
  // lines (the two 16-column halves of a 32-column row) run on one XCD and their partial lines merge
  // in its L2 instead of leaving it as two half-line write-backs
  const int G8 = (int)gridDim.x;
  const int bid = ((G8 & 7) || (dbg & 64)) ? (int)blockIdx.x : (int)((blockIdx.x & 7) * (G8 >> 3) + (blockIdx.x >> 3));
  const int gidx = bid * (NW / 2) + (wave >> 1);  // the wave's window
  const bool active = gidx < total_groups;
  const int b = active ? gidx / groups_per_sample : 0;
  const int grp = active ? gidx % groups_per_sample : 0;
  float* const xb = x + (long)b * sb;
  constexpr int WPG = NW / 2;       // windows per workgroup
  constexpr int TC = 4 * WPG;       // tile columns
  constexpr int TRS = TC + 4;       // tile row stride (floats)
  constexpr int TCS = 16 * TRS + 4; // tile channel stride: 8 TCS = 32 mod 64 banks
  constexpr int NPC = 16 * TC / 2;  // 8-B pieces per channel
  constexpr int PPW = TILE ? C * NPC / (NW * 64) : 1;  // piece instructions per wave
  static_assert(!TILE || (C * NPC) % (NW * 64) == 0, "tile pieces per wave");
  float* const tileL = reinterpret_cast<float*>(wsm + 2 * UL::HALVES);

  // buffer descriptors: the lane's token (and channel half) in the 32-bit offset, the channel
  // row in the wave-uniform soffset, invalid tokens past the extent (host checks 31 bits)
  constexpr int OOB = 0x40000000;
  const int x_bytes = (int)(((long)(C - 1) * sc + (long)g.D * st) * 4);
  const auto rs_x = __builtin_amdgcn_make_buffer_rsrc(xb, 0, x_bytes, 0x00020000);
  const auto rs_g = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(gamma), 0, C * 4, 0x00020000);
  const auto rs_mb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(mbias), 0, npat * 8 * 4096 * 4, 0x00020000);
  auto ldb = [](const __amdgpu_buffer_rsrc_t& r, int vo, int so) __attribute__((always_inline)) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
  };

  // a unit's weight slice by LDS-DMA, UL::HALVES / 512 pieces of 1 KiB over the waves
  static_assert((UL::HALVES / 512) % NW == 0, "unit slice pieces per wave");
  auto load_unit = [&](int u, _Float16* dst) __attribute__((always_inline)) {
    const _Float16* src = wpk + (long)u * UL::HALVES;
#pragma unroll
    for (int i = 0; i < UL::HALVES / 512 / NW; ++i) {
      const int pc = wave + i * NW;
      __builtin_amdgcn_global_load_lds((const void*)(src + pc * 512 + lane * 8), (lds_ptr_t)(dst + pc * 512), 16, 0, 0);
    }
  };
  load_unit(0, wsm);

  // ---- the lane's token: window (wd, wh, ww) of grp, token tk = 32 tt + lc ----
  const int nWw = g.Wp / g.ws2, nWh = g.Hp / g.ws1, nWd = g.Dp / g.ws0;
  const int ww = grp % nWw, wh = (grp / nWw) % nWh, wd = grp / (nWw * nWh);
  const int N = g.ws0 * g.ws1 * g.ws2;
  const int tk = 32 * tt + lc;
  long pos;
  bool valid;
  {
    const int td = tk / (g.ws1 * g.ws2), th = (tk / g.ws2) % g.ws1, tw = tk % g.ws2;
    const int od = (wd * g.ws0 + td + g.ss0) % g.Dp, oh = (wh * g.ws1 + th + g.ss1) % g.Hp,
              ow = (ww * g.ws2 + tw + g.ss2) % g.Wp;
    valid = active && tk < N && od < g.D && oh < g.H && ow < g.W;
    pos = (long)od * st + (long)oh * g.W + ow;
  }
  // window class of the bias / mask table: bit d for the last window along a shifted dim d
  const int pat = npat > 1 ? ((g.ss0 && wd == nWd - 1 ? 1 : 0) | (g.ss1 && wh == nWh - 1 ? 2 : 0) |
                              (g.ss2 && ww == nWw - 1 ? 4 : 0))
                           : 0;
  const int mb_lane = (tk * 64 + 4 * h) * 4;
  const int mb_wave = __builtin_amdgcn_readfirstlane(pat * 8 * 4096 * 4);
  // TILE: the workgroup's first window (all its windows share (b, wd, wh)) and the lane's k-th
  // 8-B piece: LDS float offset, global byte offset (past the extent for a padded frame)
  const int grp0 = TILE ? (bid * WPG) % groups_per_sample : 0;
  const int ww0 = grp0 % nWw, wh0 = (grp0 / nWw) % nWh, wd0 = grp0 / (nWw * nWh);
  // piece i of the lane: channel c0 + CPI i, the same (frame, row, column pair) for every i, so the
  // offsets are a base + i x a stride (32-bit: the host checks the sample's extent < 2^30 B)
  constexpr int CPI = NW * 64 / NPC;  // channels per wave instruction
  static_assert(!TILE || (NW * 64) % NPC == 0, "whole channels per piece instruction");
  struct Piece { int lbase, gbase; };
  auto piece_base = [&](int ln) __attribute__((always_inline)) {
    const int q = wave * 64 + ln;
    const int c = q / NPC, rem = q % NPC, pr = rem / (TC / 2), k = rem % (TC / 2);
    const int f = pr >> 2, r = pr & 3;
    // (the shifted coordinates stay below twice the padded extent: a conditional subtract, not a
    // division)
    int gd = wd0 * 4 + f + g.ss0, gh = wh0 * 4 + r + g.ss1, gw = ww0 * 4 + 2 * k + g.ss2;
    gd -= gd >= g.Dp ? g.Dp : 0;
    gh -= gh >= g.Hp ? g.Hp : 0;
    gw -= gw >= g.Wp ? g.Wp : 0;
    Piece pc;
    pc.lbase = c * TCS + pr * TRS + 2 * k;
    pc.gbase = active && gd < g.D ? (c * (int)sc + gd * (int)st + gh * g.W + gw) * 4 : OOB;
    return pc;
  };
  const int gstep = CPI * (int)sc * 4;  // bytes per piece index
  auto goff_of = [&](const Piece& pc, int i) __attribute__((always_inline)) {
    return pc.gbase == OOB ? OOB : pc.gbase + i * gstep;
  };
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  if (TILE) {
    u32x2 pv[PPW];
    const Piece pc = piece_base(lane);
#pragma unroll
    for (int i = 0; i < PPW; ++i) pv[i] = __builtin_amdgcn_raw_buffer_load_b64(rs_x, goff_of(pc, i), 0, 0);
#pragma unroll
    for (int i = 0; i < PPW; ++i) *reinterpret_cast<u32x2*>(tileL + pc.lbase + i * CPI * TCS) = pv[i];
    __syncthreads();
  }
  // the lane's token in the tile: frame td, row th, column 4 (window in the workgroup) + tw
  const int tpos = ((tk >> 4) * 4 + ((tk >> 2) & 3)) * TRS + 4 * (wave >> 1) + (tk & 3);

  // ---- 1. channel LayerNorm into register fragments ----
  const float sq0 = wsc[0] * q_scale, sk0 = wsc[1], sv0 = wsc[2], csm = wsc[4];
  const int vpro = valid ? (int)((8 * h * sc + pos) * 4) : OOB;  // channel 8h + (16k + e)
  int bad = 0;
  h8 xh[KS], xl[KS];
  float gi = 1.f;
  {
    float xv[KS][8];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xv[k][e] = TILE ? tileL[(16 * k + 8 * h + e) * TCS + tpos] : ldb(rs_x, vpro, (int)((16 * k + e) * sc * 4));
        s += xv[k][e];
      }
    s = xh_sum(s);
    const float m1 = s / C;
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = xv[k][e] - m1; v += d * d; }
    v = xh_sum(v);
    // padded tokens normalise to 0 through a 0 factor (stw_x3.hip: no select per element); packed
    // pairs, the same operation order as the scalar ((x - m) rv) gamma
    const float rv = (1.f / sqrtf(v / C + 1e-5f)) * (valid ? 1.f : 0.f);
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const f2 t = (pair(xv[k][e], xv[k][e + 1]) - splat(m1)) * splat(rv) *
                     pair(ldb(rs_g, 32 * h, (16 * k + e) * 4), ldb(rs_g, 32 * h, (16 * k + e + 1) * 4));
        xv[k][e] = t.x; xv[k][e + 1] = t.y;
      }
    // the wave's largest |value| to [2^8, 2^9) (stw_x3.hip: e_w; exact power-of-two scaling,
    // folded back through the q / k / v factors, so the two waves of a window may differ)
    float am = 0.f;
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(xv[k][e]));
    am = xh_max(am);
#pragma unroll
    for (int off = 1; off < 32; off <<= 1) am = fmaxf(am, __shfl_xor(am, off));
    int ew = am > 0.f && am < INFINITY ? 9 - __builtin_amdgcn_frexp_expf(am) : 0;
    ew = ew < -100 ? -100 : (ew > 100 ? 100 : ew);
    const float gs = __builtin_amdgcn_ldexpf(1.f, ew);
    gi = __builtin_amdgcn_ldexpf(1.f, -ew);
#pragma unroll
    for (int k = 0; k < KS; ++k) {
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const f2 t = pair(xv[k][e], xv[k][e + 1]) * splat(gs);
        xv[k][e] = t.x; xv[k][e + 1] = t.y;
      }
      split8(xv[k], xh[k], xl[k], bad);
    }
  }
  const float sq = sq0 * gi, sk = sk0 * gi, sv = sv0 * gi;

  f32x16 pacc[CT];
#pragma unroll
  for (int i = 0; i < CT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) pacc[i][r] = 0.f;

  // RoPE factors of the lane's (token, dim pair) registers, the same for every unit
  float rcq[8], rsq[8], rck[8], rsk[8];
#pragma unroll
  for (int r = 0; r < 16; r += 2) {
    const int pi = (dof(r, h) % DH) >> 1;
    const float c = rcos[tk * RH + pi], sn = rsin[tk * RH + pi];
    rcq[r >> 1] = FOLD ? c * sq : c; rsq[r >> 1] = FOLD ? sn * sq : sn;
    rck[r >> 1] = FOLD ? c * sk : c; rsk[r >> 1] = FOLD ? sn * sk : sn;
  }

  h8* const mine = xch + wave * XS * 64 + lane;
  const h8* const kv0 = xch + (wave & ~1) * XS * 64 + lane;  // the window's key tile 0
  const h8* const kv1 = kv0 + XS * 64;                        // and key tile 1
  constexpr int VOFF = 2 * Op<BF>::SLOTS * 64;                 // V behind K in a wave's slots

  // dbg (EXTDM_STW64_DBG, timing diagnostics only, results invalid): 16 = no unit loop
  for (int u = 0; u < ((dbg & 16) ? 0 : UNITS); ++u) {
    const _Float16* W = wsm + (u & 1) * UL::HALVES;
    // unit u's slice has landed (LDS-DMA completion is per issuing wave: drain, then barrier),
    // slot (u + 1) & 1 and every wave's exchange slots of unit u - 1 are free
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // the bias / mask rows of the unit's first head, issued ahead of the next unit's weight DMA
    // (vmcnt retires in issue order, so waiting for them does not wait for the DMA); a second
    // head's (dim 16) are issued once the first head's have been added, into the same registers
    f32x16 bia[2];
    auto load_bias = [&](int hh) __attribute__((always_inline)) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const auto v4 = __builtin_amdgcn_raw_buffer_load_b128(rs_mb, mb_lane + (32 * kt + 8 * q) * 4,
                                                                mb_wave + (u * HPU + hh) * 4096 * 4, 0);
#pragma unroll
          for (int e = 0; e < 4; ++e) bia[kt][4 * q + e] = __uint_as_float(v4[e]);
        }
    };
    load_bias(0);
    if (u + 1 < UNITS) load_unit(u + 1, wsm + ((u + 1) & 1) * UL::HALVES);

    Op<BF> qf[2];
    if (active) {
      // Q^T, K^T (rows = dims, lane = token): the next k-step's fragments read from LDS while
      // this step's MFMAs run (stw_x3.hip qkv_mfma)
      f32x16 q, k, v;
#pragma unroll
      for (int r = 0; r < 16; ++r) { q[r] = 0.f; k[r] = 0.f; v[r] = 0.f; }
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
      // V (rows = tokens, lane = dim)
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const _Float16* fv = W + UL::V + s * UL::FRAG + lane * 8;
        v = mma3(xh[s], xl[s], *reinterpret_cast<const h8*>(fv), *reinterpret_cast<const h8*>(fv + 512), v);
      }
      // scale, RoPE on (d, d + 1) = registers (r, r + 1), as packed pairs:
      // (x0, x1) <- (x0, x1) c + (-x1, x0) s
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        float q0 = q[r], q1 = q[r + 1], k0 = k[r], k1 = k[r + 1];
        if (!FOLD) { q0 *= sq; q1 *= sq; k0 *= sk; k1 *= sk; }
        q[r] = fmaf(q0, rcq[r >> 1], -(q1 * rsq[r >> 1]));
        q[r + 1] = fmaf(q1, rcq[r >> 1], q0 * rsq[r >> 1]);
        k[r] = fmaf(k0, rck[r >> 1], -(k1 * rsk[r >> 1]));
        k[r + 1] = fmaf(k1, rck[r >> 1], k0 * rsk[r >> 1]);
      }
      // operands; this wave's K and V go to its exchange slots
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float tq[8], tk_[8], tv[8];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          tq[e] = q[8 * s + e]; tq[e + 1] = q[8 * s + e + 1];
          tk_[e] = k[8 * s + e]; tk_[e + 1] = k[8 * s + e + 1];
          const f2 t = pair(v[8 * s + e], v[8 * s + e + 1]) * splat(sv);  // both tiles' V at one scale
          tv[e] = t.x; tv[e + 1] = t.y;
        }
        Op<BF> kf, vf;
        qf[s].set(tq, bad);
        kf.set(tk_, bad);
        vf.set(tv, bad);
        kf.put(mine + s * Op<BF>::SLOTS * 64);
        vf.put(mine + VOFF + s * Op<BF>::SLOTS * 64);
      }
    }
    __syncthreads();  // both tiles' K / V are in LDS
    if (!active) continue;

    // O^T per head: a dim-16 unit's two heads accumulate apart over the whole V (no per-lane
    // masking of the other head's V rows: 64 v_cndmask per unit) and the epilogue takes rows
    // 0-7 of the registers (dims 0-15: head 0) from o[0] and rows 8-15 from o[1]
    f32x16 o[HPU];
#pragma unroll
    for (int hh = 0; hh < HPU; ++hh)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[hh][r] = 0.f;
#pragma unroll
    for (int hh = 0; hh < HPU; ++hh) {
      // S^T[kt] = bias + K[kt] Q^T (rows = keys of tile kt, lane = query): the bias / mask rows are
      // the chain's initial accumulator (no separate add; the chain rounds at the bias's scale)
      f32x16 sc_[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        sc_[kt] = bia[kt];
#pragma unroll
        for (int s = 0; s < 2; ++s)
          if (HPU == 1 || s == hh) {
            Op<BF> kf;
            kf.get((kt ? kv1 : kv0) + s * Op<BF>::SLOTS * 64);
            sc_[kt] = mmo(kf, qf[s], sc_[kt]);
          }
      }
      if (hh + 1 < HPU) load_bias(hh + 1);
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc_[kt][r]);
      mx = xh_max(mx);
      // P' = 16 exp(s - mx) = v_exp_f32 of fma(s, log2 e 2^-(e_q+e_k), 4 - mx ...) (masked -inf -> 0),
      // unnormalised: O is scaled by 16 / sum P' after PV (16 or 8 products instead of 32)
      const float sum = xh_sum(exp2_sum<2>(sc_, csm, mx * csm - 4.f));
      const float inv = 16.f * __builtin_amdgcn_rcpf(sum);  // O carries P = 16 p
      // O^T[dd][i] += sum_j V^T[dd][j] P'^T[j][i]
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float tp[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) tp[e] = sc_[kt][8 * s + e];
          Op<BF> pf, vf;
          pf.set(tp, bad);
          vf.get((kt ? kv1 : kv0) + VOFF + s * Op<BF>::SLOTS * 64);
          o[hh] = mmo(vf, pf, o[hh]);
        }
      // the head's rows: all 16 registers (dim 32), registers 8 hh .. 8 hh + 7 (dim 16)
#pragma unroll
      for (int r = 0; r < 16; r += 2)
        if (HPU == 1 || (r >> 3) == hh) {
          const f2 t = pair(o[hh][r], o[hh][r + 1]) * splat(inv);
          o[hh][r] = t.x; o[hh][r + 1] = t.y;
        }
    }
    // projection: Y[c][i] += sum_dd Wp[c][u*32 + dd] O^T[dd][i] (f16x3)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float to[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) to[e] = o[HPU == 1 ? 0 : s][8 * s + e];
      h8 oh, ol;
      split8<false>(to, oh, ol, bad);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const _Float16* fp = W + UL::P + (ct * 2 + s) * UL::FRAG + lane * 8;
        pacc[ct] = mma3(*reinterpret_cast<const h8*>(fp), *reinterpret_cast<const h8*>(fp + 512), oh, ol, pacc[ct]);
      }
    }
  }
  // one finite check of the token's accumulators covers the loop's unchecked splits (stw_x3.hip)
  {
    float chk = 0.f;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) chk += pacc[ct][r];
    bad |= valid && !__builtin_isfinite(chk);
  }
  if (bad) atomicOr(range_flag, 2);
  // ---- 3. bias + residual, in place (row cu + 4h of register r) ----
  if (TILE && !(dbg & 8)) {
    // Y + bias into the tile (its exchange alias is free once every wave is past the loop), then
    // the tile's 8-B pieces + the residual leave as the prologue's coalesced pieces; padded
    // frames' offsets lie past the extent (stores dropped). The sum order is the per-lane
    // path's: (Y + bias) + x.
    const float spj = wsc[3];
    const auto rs_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bp), 0, C * 4, 0x00020000);
    __syncthreads();
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const int cu = ct * 32 + (r & 3) + 8 * (r >> 2);  // r + 1: row cu + 1
        const f2 y = pair(pacc[ct][r], pacc[ct][r + 1]) * splat(spj) +
                     pair(ldb(rs_b, 16 * h, cu * 4), ldb(rs_b, 16 * h, (cu + 1) * 4));
        tileL[(cu + 4 * h) * TCS + tpos] = y.x;
        tileL[(cu + 1 + 4 * h) * TCS + tpos] = y.y;
      }
    __syncthreads();
    u32x2 xr[PPW];
    // an opaque lane id: the two offsets recomputed here rather than kept live through the unit
    // loop from the prologue (hipcc would CSE them)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const Piece pc = piece_base(ln);
#pragma unroll
    for (int i = 0; i < PPW; ++i) xr[i] = __builtin_amdgcn_raw_buffer_load_b64(rs_x, goff_of(pc, i), 0, 0);
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const u32x2 y = *reinterpret_cast<const u32x2*>(tileL + pc.lbase + i * CPI * TCS);
      const f2 sum2 = __builtin_bit_cast(f2, y) + __builtin_bit_cast(f2, xr[i]);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, sum2), rs_x, goff_of(pc, i), 0, 0);
    }
  } else if (dbg & 8) {  // timing only: no epilogue loads / stores (one store keeps the work live)
    float acc = 0.f;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc += pacc[ct][r];
    if (acc == 12345.f) xb[pos] = acc;
  } else if (valid) {
    const float spj = wsc[3];
    const int vex = (int)((4 * h * sc + pos) * 4);
    const auto rs_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bp), 0, C * 4, 0x00020000);
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int cu = ct * 32 + (r & 3) + 8 * (r >> 2);
        const float pb = ldb(rs_b, 16 * h, cu * 4);
        const float xv = ldb(rs_x, vex, (int)(cu * sc * 4));
        const float res = (pacc[ct][r] * spj + pb) + xv;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(res), rs_x, vex, (int)(cu * sc * 4), 0);
      }
  }
}

// The TILE path's geometry (kernel note): 4x4x4 windows without H / W padding, W a multiple of 16
// (whole 4-window groups per window row), 8-B aligned rows; EXTDM_STW64_NO_TILE=1 forces the
// per-lane path (A/B)
bool stw64_tile_ok(const View& x, const AttnGeom& g, int groups) {
  static const bool off = [] { const char* v = getenv("EXTDM_STW64_NO_TILE"); return v && v[0] && v[0] != '0'; }();
  return !off && x.C == 64 && g.ws0 == 4 && g.ws1 == 4 && g.ws2 == 4 && g.H == g.Hp && g.W == g.Wp && g.W % 16 == 0 &&
         groups % 4 == 0 && x.st == (long)x.H * x.W && x.sc % 2 == 0 && x.sb % 2 == 0 && x.st % 2 == 0 &&
         ((uintptr_t)x.p & 7) == 0;
}

template <int C, int DH, int NW, bool BF>
void launch(hipStream_t s, const View& x, const AttnGeom& g, int groups, const float* gamma, const void* wpk,
            const float* wsc, const float* bp, const float* mbias, int npat, const float* rcos, const float* rsin,
            float q_scale) {
  constexpr int XS = 2 * 2 * Op<BF>::SLOTS;
  constexpr bool TILE_OK = C == 64 && NW == 8;
  const bool tile = TILE_OK && stw64_tile_ok(x, g, groups);
  const size_t ring = (size_t)2 * UL64<C>::HALVES * sizeof(_Float16);
  const size_t xch = (size_t)NW * XS * 64 * 16;
  const size_t tileb = (size_t)C * (16 * (2 * NW + 4) + 4) * sizeof(float);  // TCS floats per channel
  const size_t lds = ring + (tile ? std::max(xch, tileb) : xch);
  static std::once_flag once[64];
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::call_once(once[dev & 63], [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&stw64_x3_kernel<C, DH, NW, BF, false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (TILE_OK)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&stw64_x3_kernel<C, DH, NW, BF, TILE_OK>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  });
  const int total = x.B * groups;
  // EXTDM_STW64_XCD=0: dispatch order (A/B); else the grid rounded up to a multiple of 8 for the
  // XCD-contiguous order (the extra workgroups' windows lie past `total`: inactive)
  static const bool xcd = [] { const char* v = getenv("EXTDM_STW64_XCD"); return !(v && v[0] == '0'); }();
  int grid = (total + NW / 2 - 1) / (NW / 2);
  if (xcd && grid >= 64) grid = (grid + 7) & ~7;
  note_kernel("stw64_x3_kernel<%d, %d, %d, %s, %s>", C, DH, NW, BF ? "true" : "false", tile ? "true" : "false");
  static const int dbg0 = [] { const char* v = getenv("EXTDM_STW64_DBG"); return v ? atoi(v) : 0; }();
  const int dbg = dbg0 | (xcd && grid >= 64 ? 0 : 64);  // 64: dispatch order (no remap)
  auto kern = tile ? &stw64_x3_kernel<C, DH, NW, BF, TILE_OK> : &stw64_x3_kernel<C, DH, NW, BF, false>;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NW * 64), lds, s, x.p, x.sb, x.sc, x.st, g, gamma,
                     reinterpret_cast<const _Float16*>(wpk), wsc, bp, mbias, npat, rcos, rsin, q_scale, groups, total,
                     x3_range_ptr(), dbg);
}

template <int DH, bool BF>
bool dispatch(hipStream_t s, const View& x, const AttnGeom& g, int groups, const float* gamma, const void* wpk,
              const float* wsc, const float* bp, const float* mbias, int npat, const float* rcos, const float* rsin,
              float q_scale) {
  // C = 64: 8 waves (two per SIMD, 128 KB of LDS); C = 128: 4 waves (one per SIMD: its
  // registers), ring 128 KB + exchange 32 KB = the whole 160 KB
  if (x.C == 64) launch<64, DH, 8, BF>(s, x, g, groups, gamma, wpk, wsc, bp, mbias, npat, rcos, rsin, q_scale);
  else if (x.C == 128) launch<128, DH, 4, BF>(s, x, g, groups, gamma, wpk, wsc, bp, mbias, npat, rcos, rsin, q_scale);
  else return false;
  return true;
}

}  // namespace

bool stw64_x3_supported(int C, int ntok, int dim_head, int heads) {
  return heads == 8 && (C == 64 || C == 128) && ntok <= 64 && (dim_head == 32 || dim_head == 16) &&
         attn_x3_unit_halves(C) == (C == 64 ? UL64<64>::HALVES : UL64<128>::HALVES);
}

bool stw64_x3(hipStream_t s, const View& x, const AttnGeom& g, int heads, int dim_head, const float* gamma,
              const void* wpk, const float* wsc, const float* bp, const float* mbias, int npat, const float* rcos,
              const float* rsin, float q_scale, bool bf16) {
  const int N = g.ws0 * g.ws1 * g.ws2;
  if (!stw64_x3_supported(x.C, N, dim_head, heads)) return false;
  // 31-bit buffer offsets per sample
  if (((long)(x.C - 1) * x.sc + (long)g.D * x.st) * 4 >= (1L << 30) || x.st != (long)x.H * x.W) return false;
  const int groups = (g.Dp / g.ws0) * (g.Hp / g.ws1) * (g.Wp / g.ws2);
  if (dim_head == 32) {
    return bf16 ? dispatch<32, true>(s, x, g, groups, gamma, wpk, wsc, bp, mbias, npat, rcos, rsin, q_scale)
                : dispatch<32, false>(s, x, g, groups, gamma, wpk, wsc, bp, mbias, npat, rcos, rsin, q_scale);
  }
  return bf16 ? dispatch<16, true>(s, x, g, groups, gamma, wpk, wsc, bp, mbias, npat, rcos, rsin, q_scale)
              : dispatch<16, false>(s, x, g, groups, gamma, wpk, wsc, bp, mbias, npat, rcos, rsin, q_scale);
}

}  // namespace extdm
