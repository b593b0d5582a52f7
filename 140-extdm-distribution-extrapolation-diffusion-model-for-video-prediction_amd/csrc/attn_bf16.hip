// bf16-MFMA attention core for EXTDM_PRECISION_BF16_ATTN (the UCF-101 256 configuration
// of BASELINE: "bf16 MFMA attention"): the QK^T and PV contractions of
//   STW window self-attention    WindowAttention3D + STWAttentionLayer, u12:408-559
//                                (shifted 3-D windows of <= 64 tokens: ada / ada_u22 4x4x4)
//   temporal attention per pixel Attention, u12:252-302 (<= 32 frames)
// on v_mfma_f32_32x32x16_bf16 with fp32 accumulation; everything around them (the qkv /
// proj 1x1 convs, LayerNorms, residuals) stays f16x3 / fp32.
//
// One wave per (token group, head), up to 64 tokens as two 32-token tiles:
//   lane = (token column c = lane & 31, half h = lane >> 5); an operand fragment holds the
//   8 dims 16s + 8h .. +7 of k-step s (dim_head 32: s = 0, 1), so rotary pairs stay in-lane.
//   S^T[kt][qt] = K[kt] Q[qt]^T   (4 tiles x 2 k-steps): a lane holds 16 keys of its query
//   softmax over the 64 keys: in-lane over (kt, r), then the partner half (lane ^ 32)
//   O^T[qt]    += V^T P^T         P^T straight from the score registers as the B operand
//   (k-step = registers 8s'..8s'+7 of one key tile, keys in the accumulator's row order);
//   V^T is read from an LDS copy of V in that same key order.
// Masks as the fp32 kernels (attn.hip): shifted-window region mismatch adds -100, padded
// keys and (temporal) other pixels' frames are -inf.
#include "kernels.h"

namespace extdm {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int dof(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ int region_label(int c, int P, int w, int s) {
  if (s == 0) return 2;
  if (c >= P - s) return 2;
  if (c >= P - w) return 1;
  return 0;
}

struct TokB {
  long pos;
  int valid, exists, lab, rpos;
};

// token tk (0..63) of group grp: its position, whether it is a real in-image token,
// its shifted-window region label (MODE 0) or pixel slot (MODE 1), and its rotary /
// bias position (window token index, or frame)
template <int MODE>
__device__ __forceinline__ TokB token_b(int tk, const AttnGeom& g, long st, int grp, int per) {
  TokB o;
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
    const int p = tk / per, t = tk % per;
    const int hw = grp * (64 / per) + p;
    o.exists = t < g.D && hw < HW;
    o.valid = o.exists;
    o.pos = (long)t * st + (o.exists ? hw : 0);
    o.lab = p;
    o.rpos = t;
  }
  return o;
}

template <int MODE>
__global__ __launch_bounds__(256) void attn_bf16_kernel(const float* __restrict__ qkv, long qsb, long qsc, long st,
                                                        float* __restrict__ o, long osb, long osc, AttnGeom g,
                                                        int heads, int groups_per_sample, int total_groups,
                                                        const float* __restrict__ bias_dense, int bstride,
                                                        const float* __restrict__ rcos,
                                                        const float* __restrict__ rsin, float q_scale) {
  __shared__ float Vs[4][64][33];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  // a block = one token group, its waves walk the heads
  const int gidx = blockIdx.x;
  if (gidx >= total_groups) return;
  const int b = gidx / groups_per_sample, grp = gidx % groups_per_sample;
  const int per = g.D <= 16 ? 16 : 32;  // MODE 1: frames slot per pixel
  const TokB tq[2] = {token_b<MODE>(c, g, st, grp, per), token_b<MODE>(32 + c, g, st, grp, per)};
  const int hid = heads * 32;
  const float* qb = qkv + (long)b * qsb;
  const bool shifted = MODE == 0 && (g.ss0 | g.ss1 | g.ss2) != 0;
  // masks of the 16 keys a lane's score registers hold, per (query tile, key tile): bit r
  // of neg[qt][kt] = -inf (padded key, or another pixel's frame), of mis[qt][kt] = -100
  // (shifted-window region mismatch)
  unsigned neg[2][2] = {{0u, 0u}, {0u, 0u}}, mis[2][2] = {{0u, 0u}, {0u, 0u}};
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const TokB kk = token_b<MODE>(kt * 32 + dof(r, h), g, st, grp, per);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const bool other = kk.lab != tq[qt].lab;
        neg[qt][kt] |= (unsigned)(!kk.exists || (MODE == 1 && other)) << r;
        mis[qt][kt] |= (unsigned)(MODE == 0 && shifted && other) << r;
      }
    }
  for (int hd = wave; hd < heads; hd += 4) {
    // ---- Q, K fragments (token per lane, 16 dims each), rotary in-lane, V to LDS ----
    bf8 qf[2][2], kf[2][2];  // [tile][k-step]
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float qv[16], kv[16];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int d = 16 * s + 8 * h + e;
          const bool ok = tq[t].valid;
          qv[8 * s + e] = ok ? qb[(long)(hd * 32 + d) * qsc + tq[t].pos] : 0.f;
          kv[8 * s + e] = ok ? qb[(long)(hid + hd * 32 + d) * qsc + tq[t].pos] : 0.f;
        }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int d = 16 * s + 8 * h + e;
          Vs[wave][t * 32 + c][d] = tq[t].valid ? qb[(long)(2 * hid + hd * 32 + d) * qsc + tq[t].pos] : 0.f;
        }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const int pi = (16 * s + 8 * h + e) >> 1;
          const float cs = rcos[tq[t].rpos * 16 + pi], sn = rsin[tq[t].rpos * 16 + pi];
          const float q0 = qv[8 * s + e] * q_scale, q1 = qv[8 * s + e + 1] * q_scale;
          const float k0 = kv[8 * s + e], k1 = kv[8 * s + e + 1];
          qv[8 * s + e] = q0 * cs - q1 * sn;
          qv[8 * s + e + 1] = q1 * cs + q0 * sn;
          kv[8 * s + e] = k0 * cs - k1 * sn;
          kv[8 * s + e + 1] = k1 * cs + k0 * sn;
        }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          qf[t][s][e] = (__bf16)qv[8 * s + e];
          kf[t][s][e] = (__bf16)kv[8 * s + e];
        }
    }
    __syncthreads();  // Vs of this head visible to the wave's V^T reads (and to nobody else)
    // ---- scores S^T[kt][qt], softmax over the keys of each query ----
    f32x16 sc[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[kt][qt][r] = 0.f;
#pragma unroll
        for (int s = 0; s < 2; ++s)
          sc[kt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kt][s], qf[qt][s], sc[kt][qt], 0, 0, 0);
      }
    f32x16 out[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const TokB& me = tq[qt];
      const float* bd = bias_dense + ((long)hd * bstride + me.rpos) * bstride;
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kpos = kt * 32 + dof(r, h);  // key token; its bias column
          float sv = sc[kt][qt][r] + bd[MODE == 0 ? kpos : kpos % per];
          if ((mis[qt][kt] >> r) & 1) sv += -100.f;
          if ((neg[qt][kt] >> r) & 1) sv = -INFINITY;
          sc[kt][qt][r] = sv;
          mx = fmaxf(mx, sv);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      float sum = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = expf(sc[kt][qt][r] - mx);
          sc[kt][qt][r] = p;
          sum += p;
        }
      sum += __shfl_xor(sum, 32);
      const float inv = 1.f / sum;
      // ---- O^T[qt] = V^T P^T over 4 k-steps of 16 keys ----
#pragma unroll
      for (int r = 0; r < 16; ++r) out[qt][r] = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf8 pf, vf;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            pf[e] = (__bf16)(sc[kt][qt][8 * s + e] * inv);
            vf[e] = (__bf16)Vs[wave][kt * 32 + dof(8 * s + e, h)][c];
          }
          out[qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, out[qt], 0, 0, 0);
        }
    }
    // out[qt][r] = O[query qt*32 + c][dim dof(r, h)]
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      if (!tq[qt].valid) continue;
      float* ob = o + (long)b * osb + tq[qt].pos;
#pragma unroll
      for (int r = 0; r < 16; ++r) ob[(long)(hd * 32 + dof(r, h)) * osc] = out[qt][r];
    }
    __syncthreads();  // Vs reuse by the next head
  }
}

}  // namespace

bool attention_bf16(hipStream_t s, const View& qkv, const View& o, const AttnGeom& g, int heads, int dim_head,
                    const float* bias_dense, int bstride, const float* rope_cos, const float* rope_sin,
                    float q_scale) {
  if (dim_head != 32 || qkv.st != o.st) return false;
  int groups;
  if (g.mode == 0) {
    if (g.ws0 * g.ws1 * g.ws2 > 64) return false;
    groups = (g.Dp / g.ws0) * (g.Hp / g.ws1) * (g.Wp / g.ws2);
  } else {
    if (g.D > 32) return false;
    const int ppw = 64 / (g.D <= 16 ? 16 : 32);
    groups = (g.H * g.W + ppw - 1) / ppw;
  }
  const int total = qkv.B * groups;
  if (g.mode == 0)
    hipLaunchKernelGGL(attn_bf16_kernel<0>, dim3(total), dim3(256), 0, s, qkv.p, qkv.sb, qkv.sc, qkv.st, o.p, o.sb,
                       o.sc, g, heads, groups, total, bias_dense, bstride, rope_cos, rope_sin, q_scale);
  else
    hipLaunchKernelGGL(attn_bf16_kernel<1>, dim3(total), dim3(256), 0, s, qkv.p, qkv.sb, qkv.sc, qkv.st, o.p, o.sb,
                       o.sc, g, heads, groups, total, bias_dense, bstride, rope_cos, rope_sin, q_scale);
  return true;
}

}  // namespace extdm
