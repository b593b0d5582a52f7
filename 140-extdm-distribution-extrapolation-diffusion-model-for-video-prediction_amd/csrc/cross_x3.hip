// TrajWarp cross-attention on fp16 MFMA with the f16x3 split (see conv_x3.hip):
// ScaledDotProductAttention inside MultiHeadAttentionOp (u12:719-773),
//     O_h = softmax(Q_h K_h^T / sqrt(32)) V_h,   head h = channels 32h .. 32h+31,
// Q [B][C][NQ], K, V [B][C][NK] fp32 (channel-major, the 1x1-conv outputs).
//
// The low halves are stored scaled, lo = fp16((v - hi) * 2^11), so that they stay
// normal in fp16 for |v| down to 2^-14 (post-ReLU features and probabilities are
// often small); hi*hi and the two cross terms accumulate in separate fp32
// accumulators, combined as acc_hh + 2^-11 acc_x. The scores also keep the lo*lo term
// (softmax turns their absolute error into relative error of every probability).
//
// A block owns one (b, head) and 128 queries (4 waves x 32). The key loop stages
// 64-key chunks of K and V once per block (register prefetch of the next chunk
// during the current chunk's MFMAs):
//   Ks[hl][key][32 dims]  -- A operand of S^T = K·Q^T (lane = key row, 8 dims);
//   Vs[hl][dim][64 keys]  -- A operand of O^T = V^T·P^T, keys in the accumulator's
//                            register order (16s + 8(e>>2) + 4h + (e&3)), so P^T is
//                            the S^T accumulator itself (registers 8s..8s+7 = step s).
// 16-byte chunks are XOR-swizzled for conflict-free ds_read_b128 over 16 lanes.
#include "kernels.h"

namespace extdm {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

constexpr int KC = 64;  // keys per chunk
constexpr float LO_UP = 2048.f, LO_DN = 1.f / 2048.f;

// hi = fp16(v), lo = fp16((v - hi) * 2^11), into vector elements
#define SPLIT_S(V, HI, LO)                              \
  do {                                                  \
    const float v_ = split_src(V);                      \
    const _Float16 a_ = (_Float16)v_;                   \
    HI = a_;                                            \
    LO = (_Float16)((v_ - (float)a_) * LO_UP);          \
  } while (0)

__global__ __launch_bounds__(256) void cross_attn_x3_kernel(const float* __restrict__ Q, const float* __restrict__ K,
                                                            const float* __restrict__ V, float* __restrict__ O, int C,
                                                            int heads, int NQ, int NK, int* __restrict__ range) {
  __shared__ __attribute__((aligned(16))) _Float16 Ks[2 * KC * 32];
  __shared__ __attribute__((aligned(16))) _Float16 Vs[2 * 32 * KC];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lc = lane & 31, h = lane >> 5;
  const int nqb = (NQ + 127) / 128;
  const int qb = blockIdx.x % nqb;
  const int hd = (blockIdx.x / nqb) % heads;
  const int b = blockIdx.x / (nqb * heads);
  const int qi = qb * 128 + wave * 32 + lc;
  const bool qvalid = qi < NQ;
  const float* qp = Q + ((long)b * C + hd * 32) * NQ;
  const float* kp = K + ((long)b * C + hd * 32) * NK;
  const float* vp = V + ((long)b * C + hd * 32) * NK;
  int bad = 0;

  // Q^T as the B operand (lane = query, k-step s = dims 16s + 8h + e), pre-scaled by
  // 1/sqrt(dk)
  h8 qh[2], ql[2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = qvalid ? qp[(long)(16 * s + 8 * h + e) * NQ + qi] * 0.17677669529663687f : 0.f;
      bad |= fabsf(v) >= 65504.f;
      SPLIT_S(v, qh[s][e], ql[s][e]);
    }

  // staging roles: K -- key kk = lane of the chunk, dims 8*wave .. +7 (one 256-B row
  // segment per load instruction); V -- dim vd, keys 8*vg .. +7 of the chunk
  const int vd = tid >> 3, vg = tid & 7;
  float kr[8], vr[8];
  auto load = [&](int j0) {
    const int kj = j0 + lane;
#pragma unroll
    for (int e = 0; e < 8; ++e) kr[e] = kj < NK ? kp[(long)(8 * wave + e) * NK + kj] : 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int vj = j0 + 8 * vg + e;
      vr[e] = vj < NK ? vp[(long)vd * NK + vj] : 0.f;
    }
  };
  auto store = [&]() {
    h8 hi, lo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bad |= fabsf(kr[e]) >= 65504.f;
      SPLIT_S(kr[e], hi[e], lo[e]);
    }
    // row = key (64 B), chunk = dim group, swizzled by bits 2-3 of the key
    const int kc = wave ^ ((lane >> 2) & 3);
    *reinterpret_cast<h8*>(Ks + lane * 32 + kc * 8) = hi;
    *reinterpret_cast<h8*>(Ks + KC * 32 + lane * 32 + kc * 8) = lo;
    // keys 8vg + i -> step s = vg >> 1, half hh = i >> 2, element 4(vg & 1) + (i & 3)
    h4 h0, h1, l0, l1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bad |= (fabsf(vr[i]) >= 65504.f) | (fabsf(vr[i + 4]) >= 65504.f);
      SPLIT_S(vr[i], h0[i], l0[i]);
      SPLIT_S(vr[i + 4], h1[i], l1[i]);
    }
    const int s = vg >> 1, eo = 4 * (vg & 1), sw = (vd >> 1) & 7;
    _Float16* row = Vs + vd * KC;
    *reinterpret_cast<h4*>(row + (((2 * s) ^ sw) * 8) + eo) = h0;
    *reinterpret_cast<h4*>(row + (((2 * s + 1) ^ sw) * 8) + eo) = h1;
    *reinterpret_cast<h4*>(row + 32 * KC + (((2 * s) ^ sw) * 8) + eo) = l0;
    *reinterpret_cast<h4*>(row + 32 * KC + (((2 * s + 1) ^ sw) * 8) + eo) = l1;
  };

  f32x16 oh, ox;
#pragma unroll
  for (int r = 0; r < 16; ++r) { oh[r] = 0.f; ox[r] = 0.f; }
  float m = -INFINITY, l = 0.f;

  load(0);
  for (int j0 = 0; j0 < NK; j0 += KC) {
    __syncthreads();  // every wave is done with the previous chunk
    store();
    __syncthreads();
    if (j0 + KC < NK) load(j0 + KC);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      // ---- S^T (rows = keys 32t + dof, lane = query) ----
      f32x16 sh, sx, sxx;
#pragma unroll
      for (int r = 0; r < 16; ++r) { sh[r] = 0.f; sx[r] = 0.f; sxx[r] = 0.f; }
      const int krow = 32 * t + lc;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const _Float16* ap = Ks + krow * 32 + (((2 * s + h) ^ ((krow >> 2) & 3)) * 8);
        const h8 ah = *reinterpret_cast<const h8*>(ap);
        const h8 al = *reinterpret_cast<const h8*>(ap + KC * 32);
        sh = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, qh[s], sh, 0, 0, 0);
        sx = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, qh[s], sx, 0, 0, 0);
        sx = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, ql[s], sx, 0, 0, 0);
        sxx = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, ql[s], sxx, 0, 0, 0);
      }
      // ---- online softmax over the 32 keys (16 in-lane + the partner half) ----
      float cm = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = j0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float sv = j < NK ? sh[r] + (sx[r] + sxx[r] * LO_DN) * LO_DN : -INFINITY;
        sh[r] = sv;
        cm = fmaxf(cm, sv);
      }
      cm = fmaxf(cm, __shfl_xor(cm, 32));
      const float mn = fmaxf(m, cm);
      if (mn == -INFINITY) continue;  // a fully padded tail (never the first tile)
      // exp(x - mn) as v_exp_f32 (2^x) of fma(x, log2 e, -mn log2 e); exp(-inf) = 0
      const float mnl = mn * 1.44269504088896341f;
      const float alpha = __builtin_amdgcn_exp2f(fmaf(m, 1.44269504088896341f, -mnl));
      float ps = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sh[r] = __builtin_amdgcn_exp2f(fmaf(sh[r], 1.44269504088896341f, -mnl));
        ps += sh[r];
      }
      ps += __shfl_xor(ps, 32);
      l = l * alpha + ps;
      m = mn;
#pragma unroll
      for (int r = 0; r < 16; ++r) { oh[r] *= alpha; ox[r] *= alpha; }
      // ---- O^T += V^T·P^T, P^T straight from the accumulator registers ----
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        h8 ph, pl;
#pragma unroll
        for (int e = 0; e < 8; ++e) SPLIT_S(sh[8 * s2 + e], ph[e], pl[e]);
        const int c = 2 * (2 * t + s2) + h;
        const _Float16* vp2 = Vs + lc * KC + ((c ^ ((lc >> 1) & 7)) * 8);
        const h8 vh = *reinterpret_cast<const h8*>(vp2);
        const h8 vl = *reinterpret_cast<const h8*>(vp2 + 32 * KC);
        oh = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, ph, oh, 0, 0, 0);
        ox = __builtin_amdgcn_mfma_f32_32x32x16_f16(vl, ph, ox, 0, 0, 0);
        ox = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, pl, ox, 0, 0, 0);
      }
    }
  }
  if (bad) atomicOr(range, 1);
  if (qvalid) {
    float* ob = O + ((long)b * C + hd * 32) * NQ + qi;
    const float il = 1.f / l;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int dd = (r & 3) + 8 * (r >> 2) + 4 * h;
      ob[(long)dd * NQ] = (oh[r] + ox[r] * LO_DN) * il;
    }
  }
}

// ---- pre-split K / V (the cond cache: k and v depend on the cond frames only) ----
// kvp[b][head][key tile kt][k | v][s][hl][64 lanes][8]: the MFMA A fragments of one
// 32-key tile, split once per sampling call exactly as the staged kernel splits them:
//   K (S^T = K·Q^T): lane (h, lc) element e = K[dim 16s + 8h + e][key 32kt + lc];
//   V (O^T = V^T·P^T): lane (h, lc) element e = V[dim lc][key 32kt + 16s + 8(e>>2) + 4h + (e&3)]
// (keys >= NK are zero; their scores are masked).
__global__ __launch_bounds__(256) void cross_kv_split_kernel(const float* __restrict__ K, const float* __restrict__ V,
                                                             _Float16* __restrict__ kvp, int C, int heads, int NK,
                                                             int nkt, long total, int* __restrict__ range) {
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;  // (b, head, kt, kv, s, lane)
  if (gid >= total) return;
  const int lane = (int)(gid & 63);
  long r = gid >> 6;
  const int s = (int)(r & 1); r >>= 1;
  const int kv = (int)(r & 1); r >>= 1;
  const int kt = (int)(r % nkt); r /= nkt;
  const int hd = (int)(r % heads);
  const int b = (int)(r / heads);
  const int h = lane >> 5, lc = lane & 31;
  const float* src = (kv ? V : K) + ((long)b * C + hd * 32) * NK;
  h8 hi, lo;
  int bad = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int dim = kv ? lc : 16 * s + 8 * h + e;
    const int key = kv ? 32 * kt + 16 * s + 8 * (e >> 2) + 4 * h + (e & 3) : 32 * kt + lc;
    const float v = key < NK ? src[(long)dim * NK + key] : 0.f;
    bad |= fabsf(v) >= 65504.f;
    SPLIT_S(v, hi[e], lo[e]);
  }
  if (bad) atomicOr(range, 1);
  _Float16* d = kvp + ((((((long)b * heads + hd) * nkt + kt) * 2 + kv) * 2 + s) * 2) * 512 + lane * 8;
  *reinterpret_cast<h8*>(d) = hi;
  *reinterpret_cast<h8*>(d + 512) = lo;
}

// The same attention with the fragments read straight from kvp (L2-resident: 28 query
// blocks share a (b, head) slice): no LDS staging, no splits of K / V, no barriers.
// Per 32-key tile the arithmetic is the staged kernel's, operation for operation.
// scaled-lo split of a pair into elements e, e + 1 (compiler-visible: the values come
// from and go to MFMAs): hi = fp16 pair, lo = fp16((v - hi) * 2^11) via v_fma_mix_f32
__device__ __forceinline__ void split2s(float a, float b, h8& hi, h8& lo, int e) {
  f16x2_t ph, pl;
  const float a_ = split_src(a), b_ = split_src(b);
  ph = __builtin_convertvector((f32x2_t){a_, b_}, f16x2_t);
  const float one = split_src(1.0f);
  const float la = __builtin_fmaf(-(float)ph.x, one, a_) * LO_UP;
  const float lb = __builtin_fmaf(-(float)ph.y, one, b_) * LO_UP;
  pl = __builtin_convertvector((f32x2_t){la, lb}, f16x2_t);
  hi[e] = ph.x; hi[e + 1] = ph.y;
  lo[e] = pl.x; lo[e + 1] = pl.y;
}

// Per 32-key tile the VALU is the bound (MFMA 14 x 32 cycles against ~260 vector
// instructions per tile in the first form), so the loop carries only what the tile needs:
//  - the K lo x Q lo scores term rides in the cross-term accumulator (Q's unscaled lo as
//    a third fragment, qd): one fma combines a score instead of two;
//  - 1/sqrt(dk) and log2 e folded into Q: scores come out in log2 units;
//  - lazy rescaling: the running maximum a lane's probabilities are taken against moves
//    only when a new score exceeds it by more than 2^4 in probability (any lane of the
//    wave: one wave-uniform branch), so the 48 accumulator multiplies and the alpha exp
//    are off the common path; P <= 2^4 is taken as P' = 2^11 P (<= 2^15, in the exp2
//    argument), whose lo half fp16(P' - hi') needs no scaling multiply (split2u): V's
//    scaled lo x P' hi then sits at 2^22 in its own accumulator (ox2);
//  - the key mask only in a partial tail tile (wave-uniform branch);
//  - two tiles per loop trip over two fragment sets (no register rotation copies).
// A wave owns QS sets of 32 queries: each K / V fragment read from L2 serves QS sets
// (QS = 2 halves the L2 fragment traffic: 7.5 GB per B = 64 launch at QS = 1).
// unscaled split of a pair of probabilities already scaled by 2^11 (P' = 2^11 P <= 2^15):
// hi' = fp16 pair = 2^11 fp16(P) in the normal range, lo' = fp16(P' - hi') (the difference
// exact in fp32): the scaled-lo pair without its multiply
__device__ __forceinline__ void split2u(float a, float b, h8& hi, h8& lo, int e) {
  const float a_ = split_src(a), b_ = split_src(b);
  const f16x2_t ph = __builtin_convertvector((f32x2_t){a_, b_}, f16x2_t);
  const float one = split_src(1.0f);
  const float la = __builtin_fmaf(-(float)ph.x, one, a_);
  const float lb = __builtin_fmaf(-(float)ph.y, one, b_);
  const f16x2_t pl = __builtin_convertvector((f32x2_t){la, lb}, f16x2_t);
  hi[e] = ph.x; hi[e + 1] = ph.y;
  lo[e] = pl.x; lo[e + 1] = pl.y;
}

template <int QS>
__global__ __launch_bounds__(256) void cross_attn_x3p_kernel(const float* __restrict__ Q,
                                                             const _Float16* __restrict__ kvp, float* __restrict__ O,
                                                             int C, int heads, int NQ, int NK, int nkt,
                                                             int* __restrict__ range) {
  constexpr float LOG2E = 1.44269504088896341f;
  constexpr float TAU = 4.f;  // log2 of the largest probability before a rescale (P' <= 2^15)
  constexpr int QB = 128 * QS;  // queries per block
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lc = lane & 31, h = lane >> 5;
  const int nqb = (NQ + QB - 1) / QB;
  // XCD-aware block order (conv_x3.hip tile note): the query blocks of one (b, head) on one
  // XCD, so its pre-split K / V come from that XCD's L2
  const int bid = (gridDim.x & 7) ? (int)blockIdx.x : (int)((blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3));
  const int qb = bid % nqb;
  const int hd = (bid / nqb) % heads;
  const int b = bid / (nqb * heads);
  const float* qp = Q + ((long)b * C + hd * 32) * NQ;
  int bad = 0;
  // qh = fp16(v), ql = fp16((v - hi) 2^11), qd = fp16(v - hi) (the lo x lo term's operand)
  h8 qh[QS][2], ql[QS][2], qd[QS][2];
#pragma unroll
  for (int u = 0; u < QS; ++u) {
    const int qi = qb * QB + (wave * QS + u) * 32 + lc;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v =
            qi < NQ ? qp[(long)(16 * s + 8 * h + e) * NQ + qi] * (0.17677669529663687f * LOG2E) : 0.f;
        bad |= fabsf(v) >= 65504.f;
        const float v_ = split_src(v);
        const _Float16 a_ = (_Float16)v_;
        qh[u][s][e] = a_;
        ql[u][s][e] = (_Float16)((v_ - (float)a_) * LO_UP);
        qd[u][s][e] = (_Float16)(v_ - (float)a_);
      }
  }
  const _Float16* base = kvp + ((long)b * heads + hd) * nkt * 8 * 512 + lane * 8;
  // fragments of a tile: [k | v][s][hl], 1 KiB apart
  h8 f0[8], f1[8];
  auto load = [&](int kt, h8* dst) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; ++i) dst[i] = *reinterpret_cast<const h8*>(base + ((long)kt * 8 + i) * 512);
  };
  // O' = 2^11 O as oh (V hi x P' hi) + ox (V hi x P' lo) + 2^-11 ox2 (V scaled lo x P' hi)
  f32x16 oh[QS], ox[QS], ox2[QS];
  float mk[QS], l[QS];  // mk: the reference maximum, log2 units; l = sum of P'
#pragma unroll
  for (int u = 0; u < QS; ++u) {
#pragma unroll
    for (int r = 0; r < 16; ++r) { oh[u][r] = 0.f; ox[u][r] = 0.f; ox2[u][r] = 0.f; }
    mk[u] = -INFINITY;
    l[u] = 0.f;
  }
  auto tile = [&](int kt, const h8* f) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < QS; ++u) {
      f32x16 sh, sx;
#pragma unroll
      for (int r = 0; r < 16; ++r) { sh[r] = 0.f; sx[r] = 0.f; }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const h8 ah = f[2 * s], al = f[2 * s + 1];
        sh = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, qh[u][s], sh, 0, 0, 0);
        sx = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, qh[u][s], sx, 0, 0, 0);
        sx = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, ql[u][s], sx, 0, 0, 0);
        sx = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, qd[u][s], sx, 0, 0, 0);
      }
      float cm = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; r += 2) {  // packed pairs (v_pk_fma_f32)
        const f2 t = pk_fma(pair(sx[r], sx[r + 1]), splat(LO_DN), pair(sh[r], sh[r + 1]));
        sh[r] = t.x; sh[r + 1] = t.y;
        cm = fmaxf(cm, fmaxf(t.x, t.y));
      }
      const int j0 = 32 * kt;
      if (j0 + 32 > NK) {  // partial tail tile (wave-uniform)
        cm = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int j = j0 + (r & 3) + 8 * (r >> 2) + 4 * h;
          sh[r] = j < NK ? sh[r] : -INFINITY;
          cm = fmaxf(cm, sh[r]);
        }
      }
      cm = fmaxf(cm, __shfl_xor(cm, 32));
      if (__any(cm > mk[u] + TAU)) {  // rare after the first tile
        const float mn = fmaxf(mk[u], cm);
        const float alpha = __builtin_amdgcn_exp2f(mk[u] - mn);  // 0 on the first tile
        l[u] *= alpha;
#pragma unroll
        for (int r = 0; r < 16; ++r) { oh[u][r] *= alpha; ox[u][r] *= alpha; ox2[u][r] *= alpha; }
        mk[u] = mn;
      }
      const float mkb = mk[u] - 11.f;  // P' = 2^11 P
      f2 ps2 = splat(0.f);
#pragma unroll
      for (int r = 0; r < 16; r += 2) {  // packed argument and sum (v_pk_add_f32)
        f2 a = pair(sh[r], sh[r + 1]) - splat(mkb);
        a.x = __builtin_amdgcn_exp2f(a.x);
        a.y = __builtin_amdgcn_exp2f(a.y);
        sh[r] = a.x; sh[r + 1] = a.y;
        ps2 += a;
      }
      const float ps = ps2.x + ps2.y;
      l[u] += ps + __shfl_xor(ps, 32);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        h8 ph, pl;
#pragma unroll
        for (int e = 0; e < 8; e += 2) split2u(sh[8 * s2 + e], sh[8 * s2 + e + 1], ph, pl, e);
        const h8 vh = f[4 + 2 * s2], vl = f[5 + 2 * s2];
        oh[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, ph, oh[u], 0, 0, 0);
        ox2[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vl, ph, ox2[u], 0, 0, 0);
        ox[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, pl, ox[u], 0, 0, 0);
      }
    }
  };
  // two tiles per trip over the two fragment sets, the odd tail after the loop: no exit in
  // the middle of a trip (that form kept the O accumulators in different registers on the
  // two paths: a loop-carried copy of all 48 per trip); the last trip's set-0 load re-reads
  // the final tile instead of branching around it
  load(0, f0);
  int kt = 0;
  for (; kt + 1 < nkt; kt += 2) {
    load(kt + 1, f1);
    tile(kt, f0);
    load(min(kt + 2, nkt - 1), f0);
    tile(kt + 1, f1);
  }
  if (kt < nkt) tile(kt, f0);
  if (bad) atomicOr(range, 1);
#pragma unroll
  for (int u = 0; u < QS; ++u) {
    const int qi = qb * QB + (wave * QS + u) * 32 + lc;
    if (qi < NQ) {
      float* ob = O + ((long)b * C + hd * 32) * NQ + qi;
      const float il = 1.f / l[u];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int dd = (r & 3) + 8 * (r >> 2) + 4 * h;
        ob[(long)dd * NQ] = fmaf(ox2[u][r], LO_DN, oh[u][r] + ox[u][r]) * il;
      }
    }
  }
}

}  // namespace

size_t cross_kv_halves(int B, int C, int heads, int NK) {
  return (size_t)B * heads * ((NK + 31) / 32) * 8 * 512;
}

bool cross_kv_split(hipStream_t s, const float* k, const float* v, _Float16* kvp, int B, int C, int heads, int NK) {
  if (C != 32 * heads || NK < 1) return false;
  const int nkt = (NK + 31) / 32;
  const long total = (long)B * heads * nkt * 2 * 2 * 64;
  hipLaunchKernelGGL(cross_kv_split_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, k, v, kvp, C, heads,
                     NK, nkt, total, x3_range_ptr());
  return true;
}

bool cross_attention_x3p(hipStream_t s, const float* q, const _Float16* kvp, float* o, int B, int C, int heads, int NQ,
                         int NK) {
  if (C != 32 * heads || NK < 1 || NQ < 1) return false;
  // QS = 1: QS = 2 needs 256 VGPRs (one wave per SIMD) and measured 0.63 -> 0.94 ms at
  // B = 64; EXTDM_CROSS_QS=2 selects it (A/B)
  static const int qs_env = [] { const char* e = getenv("EXTDM_CROSS_QS"); return e ? atoi(e) : 0; }();
  const int qs = qs_env == 2 ? 2 : 1;
  const unsigned nblocks = (unsigned)(B * heads * ((NQ + 128 * qs - 1) / (128 * qs)));
  hipLaunchKernelGGL(qs == 2 ? cross_attn_x3p_kernel<2> : cross_attn_x3p_kernel<1>, dim3(nblocks), dim3(256), 0, s,
                     q, kvp, o, C, heads, NQ, NK, (NK + 31) / 32, x3_range_ptr());
  return true;
}

bool cross_attention_x3(hipStream_t s, const float* q, const float* k, const float* v, float* o, int B, int C,
                        int heads, int NQ, int NK) {
  if (C != 32 * heads || NK < 1 || NQ < 1) return false;
  const unsigned nblocks = (unsigned)(B * heads * ((NQ + 127) / 128));
  hipLaunchKernelGGL(cross_attn_x3_kernel, dim3(nblocks), dim3(256), 0, s, q, k, v, o, C, heads, NQ, NK,
                     x3_range_ptr());
  return true;
}

}  // namespace extdm
