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

}  // namespace

bool cross_attention_x3(hipStream_t s, const float* q, const float* k, const float* v, float* o, int B, int C,
                        int heads, int NQ, int NK) {
  if (C != 32 * heads || NK < 1 || NQ < 1) return false;
  const unsigned nblocks = (unsigned)(B * heads * ((NQ + 127) / 128));
  hipLaunchKernelGGL(cross_attn_x3_kernel, dim3(nblocks), dim3(256), 0, s, q, k, v, o, C, heads, NQ, NK,
                     x3_range_ptr());
  return true;
}

}  // namespace extdm
