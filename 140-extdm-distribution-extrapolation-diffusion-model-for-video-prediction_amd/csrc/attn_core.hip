// Attention core (the QK^T and PV contractions on qkv produced by a 1x1 conv) of
//   STW window self-attention    WindowAttention3D + STWAttentionLayer, u12:408-559
//                                (shifted 3-D windows of <= 64 tokens: ada / ada_u22 4x4x4)
//   temporal attention per pixel Attention, u12:252-302 (<= 32 frames)
// in two arithmetics (template X3):
//   X3 = true   f16x3 (hi / lo fp16 operands, three v_mfma_f32_32x32x16_f16 per product,
//               fp32-faithful; conv_x3.hip): the F16X3 path for the shapes the fused
//               kernels do not cover (C = 256 windows, 64-token windows)
//   X3 = false  bf16 (v_mfma_f32_32x32x16_bf16): EXTDM_PRECISION_BF16_ATTN, the UCF-101 256
//               configuration of BASELINE ("bf16 MFMA attention")
// Everything around the core (LayerNorms, the qkv / proj 1x1 convs, residuals) runs as f16x3.
//
// One wave per (token group, head); a group is NT 32-token tiles: NT = 2 for 64-token
// windows, NT = 1 for windows of <= 32 tokens and for temporal groups (32 / T' pixels'
// frames, T' = 16 or 32 slots), so no block of the score matrix is wholly masked.
//   lane = (token column c = lane & 31, half h = lane >> 5); an operand fragment holds the
//   8 dims 16s + 8h .. +7 of k-step s (dim_head 32: s = 0, 1; dim_head 16: s = 0 only, the
//   ada denoiser's C = 256 windows), so rotary pairs stay in-lane. At dim_head 16 the O^T tile's
//   rows 16-31 (V^T rows past the head) are zero and not stored.
//   S^T[kt][qt] = K[kt] Q[qt]^T   (NT^2 tiles x 2 k-steps): a lane holds 16 keys of its query
//   softmax over the keys: in-lane over (kt, r), then the partner half (lane ^ 32)
//   O^T[qt]    += V^T P^T         P^T straight from the score registers as the B operand
//   (k-step = registers 8s'..8s'+7 of one key tile, keys in the accumulator's row order);
//   V^T is read from an LDS copy of V in that same key order.
// Masks as the fp32 kernels (attn.hip): shifted-window region mismatch adds -100, padded
// keys and (temporal) other pixels' frames are -inf.
#include <cstdlib>

#include "kernels.h"

namespace extdm {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

// operand fragment of 8 k-elements: bf16, or the f16x3 hi / lo pair
template <bool X3> struct Frag;
template <> struct Frag<false> {
  bf8 v;
  template <bool CHECK = true>
  __device__ void set(const float* x, int& bad) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (__bf16)x[e];
    (void)bad;
  }
};
template <> struct Frag<true> {
  h8 hi, lo;
  // hi = fp16(x), lo = fp16((x - hi) * 2^11): the scaled lo stays normal down to |x| ~ 2^-14
  // (q / k / v here are 1x1-conv outputs of any scale, probabilities in [0, 1]); the cross
  // products accumulate apart from hi * hi (mma below, as cross_x3.hip).
  // CHECK: OR |x| >= 65504 (fp16 overflow of hi) into bad; probabilities skip it.
  // Compiler-visible VALU, not the split2 asm of kernels.h: the fragments feed MFMAs, and
  // only compiler-visible VALU gets its MFMA hazard waits.
  template <bool CHECK = true>
  __device__ void set(const float* x, int& bad) {
    float m = 0.f;
    const float one = split_src(1.0f);
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const float w0 = split_src(x[e]), w1 = split_src(x[e + 1]);
      if (CHECK) m = fmaxf(fmaxf(m, fabsf(w0)), fabsf(w1));
      const f16x2_t ph = __builtin_convertvector((f32x2_t){w0, w1}, f16x2_t);
      hi[e] = ph.x; hi[e + 1] = ph.y;
      lo[e] = (_Float16)(__builtin_fmaf(-(float)ph.x, one, w0) * X3_LO_UP);
      lo[e + 1] = (_Float16)(__builtin_fmaf(-(float)ph.y, one, w1) * X3_LO_UP);
    }
    if (CHECK) bad |= m >= 65504.f;
  }
};
// c += A * B (rows of A x columns of B over 16 k); f16x3: c += A_hi B_hi, x += the two cross
// products with a scaled lo (x carries 2^11; fin combines c + 2^-11 x)
__device__ __forceinline__ void mma(const Frag<false>& a, const Frag<false>& b, f32x16& c, f32x16&) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v, b.v, c, 0, 0, 0);
}
__device__ __forceinline__ void mma(const Frag<true>& a, const Frag<true>& b, f32x16& c, f32x16& x) {
  x = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.lo, b.hi, x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.hi, b.lo, x, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.hi, b.hi, c, 0, 0, 0);
}
template <bool X3>
__device__ __forceinline__ void fin(f32x16& c, const f32x16& x) {
  if (X3) {
#pragma unroll
    for (int r = 0; r < 16; ++r) c[r] = __builtin_fmaf(x[r], 1.f / X3_LO_UP, c[r]);
  }
}

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

// token tk (0 .. 32 NT - 1) of group grp: its position, whether it is a real in-image
// token, its shifted-window region label (MODE 0) or pixel slot (MODE 1), and its rotary /
// bias position (window token index, or frame)
template <int MODE, int NT>
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
    const int hw = grp * (32 * NT / per) + p;
    o.exists = t < g.D && hw < HW;
    o.valid = o.exists;
    o.pos = (long)t * st + (o.exists ? hw : 0);
    o.lab = p;
    o.rpos = t;
  }
  return o;
}

template <int MODE, bool X3, int NT, int DH>
__global__ __launch_bounds__(256) void attn_core_kernel(const float* __restrict__ qkv, long qsb, long qsc, long st,
                                                        float* __restrict__ o, long osb, long osc, AttnGeom g,
                                                        int heads, int groups_per_sample, int total_groups,
                                                        const float* __restrict__ bias_dense, int bstride,
                                                        const float* __restrict__ rcos,
                                                        const float* __restrict__ rsin, float q_scale,
                                                        int* __restrict__ range_flag, int xcd) {
  constexpr int KST = DH / 16;  // k-steps of the QK^T contraction
  constexpr int RH = DH / 2;     // rotary pairs per head
  __shared__ float Vs[4][32 * NT][33];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  // a block = one token group, its waves walk the heads. xcd: XCD-contiguous group order (grid a
  // multiple of 8): neighbouring windows, which read the same 128-B lines of qkv (a 4-wide window
  // row is 16 B of each line), run on one XCD and share its L2
  const int G8 = (int)gridDim.x;
  const int gidx = xcd ? (int)((blockIdx.x & 7) * (G8 >> 3) + (blockIdx.x >> 3)) : (int)blockIdx.x;
  if (gidx >= total_groups) return;
  const int b = gidx / groups_per_sample, grp = gidx % groups_per_sample;
  const int per = g.D <= 16 ? 16 : 32;  // MODE 1: frame slots per pixel
  TokB tq[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) tq[t] = token_b<MODE, NT>(32 * t + c, g, st, grp, per);
  const int hid = heads * DH;
  const float* qb = qkv + (long)b * qsb;
  const bool shifted = MODE == 0 && (g.ss0 | g.ss1 | g.ss2) != 0;
  // masks of the 16 keys a lane's score registers hold, per (query tile, key tile): bit r
  // of neg[qt][kt] = -inf (padded key, or another pixel's frame), of mis[qt][kt] = -100
  // (shifted-window region mismatch)
  unsigned neg[NT][NT], mis[NT][NT];
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
#pragma unroll
    for (int qt = 0; qt < NT; ++qt) neg[qt][kt] = mis[qt][kt] = 0u;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const TokB kk = token_b<MODE, NT>(kt * 32 + dof(r, h), g, st, grp, per);
#pragma unroll
      for (int qt = 0; qt < NT; ++qt) {
        const bool other = kk.lab != tq[qt].lab;
        neg[qt][kt] |= (unsigned)(!kk.exists || (MODE == 1 && other)) << r;
        mis[qt][kt] |= (unsigned)(MODE == 0 && shifted && other) << r;
      }
    }
  }
  int bad = 0;
  for (int hd = wave; hd < heads; hd += 4) {
    // ---- Q, K fragments (token per lane, 16 dims each), rotary in-lane, V to LDS ----
    Frag<X3> qf[NT][KST], kf[NT][KST];  // [tile][k-step]
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float qv[8 * KST], kv[8 * KST];
      const bool ok = tq[t].valid;
#pragma unroll
      for (int s = 0; s < KST; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int d = 16 * s + 8 * h + e;
          qv[8 * s + e] = ok ? qb[(long)(hd * DH + d) * qsc + tq[t].pos] : 0.f;
          kv[8 * s + e] = ok ? qb[(long)(hid + hd * DH + d) * qsc + tq[t].pos] : 0.f;
          Vs[wave][t * 32 + c][d] = ok ? qb[(long)(2 * hid + hd * DH + d) * qsc + tq[t].pos] : 0.f;
        }
#pragma unroll
      for (int s = 0; s < KST; ++s)
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const int pi = (16 * s + 8 * h + e) >> 1;
          const float cs = rcos[tq[t].rpos * RH + pi], sn = rsin[tq[t].rpos * RH + pi];
          const float q0 = qv[8 * s + e] * q_scale, q1 = qv[8 * s + e + 1] * q_scale;
          const float k0 = kv[8 * s + e], k1 = kv[8 * s + e + 1];
          qv[8 * s + e] = q0 * cs - q1 * sn;
          qv[8 * s + e + 1] = q1 * cs + q0 * sn;
          kv[8 * s + e] = k0 * cs - k1 * sn;
          kv[8 * s + e + 1] = k1 * cs + k0 * sn;
        }
#pragma unroll
      for (int s = 0; s < KST; ++s) {
        qf[t][s].set(qv + 8 * s, bad);
        kf[t][s].set(kv + 8 * s, bad);
      }
    }
    // Vs[wave] is private to the wave: a wave-level fence + barrier orders its writes before
    // the V^T reads (a block barrier here would diverge when heads % 4 != 0)
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int qt = 0; qt < NT; ++qt) {
      // ---- scores S^T[kt] of query tile qt, softmax over the keys of each query ----
      f32x16 sc[NT];
#pragma unroll
      for (int kt = 0; kt < NT; ++kt) {
        f32x16 sx;
#pragma unroll
        for (int r = 0; r < 16; ++r) { sc[kt][r] = 0.f; sx[r] = 0.f; }
#pragma unroll
        for (int s = 0; s < KST; ++s) mma(kf[kt][s], qf[qt][s], sc[kt], sx);
        fin<X3>(sc[kt], sx);
      }
      const TokB& me = tq[qt];
      const float* bd = bias_dense + ((long)hd * bstride + me.rpos) * bstride;
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < NT; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kpos = kt * 32 + dof(r, h);  // key token; its bias column
          float sv = sc[kt][r] + bd[MODE == 0 ? kpos : kpos % per];
          if ((mis[qt][kt] >> r) & 1) sv += -100.f;
          if ((neg[qt][kt] >> r) & 1) sv = -INFINITY;
          sc[kt][r] = sv;
          mx = fmaxf(mx, sv);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      // exp(s - mx) as v_exp_f32 (2^x) of fma(s, log2 e, -mx log2 e): masked -inf -> 0
      const float mxl = mx * 1.44269504088896341f;
      float sum = 0.f;
#pragma unroll
      for (int kt = 0; kt < NT; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f(fmaf(sc[kt][r], 1.44269504088896341f, -mxl));
          sc[kt][r] = p;
          sum += p;
        }
      sum += __shfl_xor(sum, 32);
      const float inv = 1.f / sum;
      // ---- O^T = V^T P^T over 2 NT k-steps of 16 keys ----
      f32x16 out, ox;
#pragma unroll
      for (int r = 0; r < 16; ++r) { out[r] = 0.f; ox[r] = 0.f; }
#pragma unroll
      for (int kt = 0; kt < NT; ++kt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float pv[8], vv[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            pv[e] = sc[kt][8 * s + e] * inv;
            vv[e] = DH == 32 || c < DH ? Vs[wave][kt * 32 + dof(8 * s + e, h)][c] : 0.f;
          }
          Frag<X3> pf, vf;
          pf.template set<false>(pv, bad);
          vf.set(vv, bad);
          mma(vf, pf, out, ox);
        }
      fin<X3>(out, ox);
      // out[r] = O[query qt*32 + c][dim dof(r, h)]
      if (me.valid) {
        float* ob = o + (long)b * osb + me.pos;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (DH == 32 || dof(r, h) < DH) ob[(long)(hd * DH + dof(r, h)) * osc] = out[r];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // Vs reuse by the wave's next head
    __builtin_amdgcn_wave_barrier();
  }
  if (X3 && bad) atomicOr(range_flag, 2);
}

}  // namespace

bool attention_core(hipStream_t s, const View& qkv, const View& o, const AttnGeom& g, int heads, int dim_head,
                    const float* bias_dense, int bstride, const float* rope_cos, const float* rope_sin, float q_scale,
                    bool bf16) {
  if ((dim_head != 32 && dim_head != 16) || qkv.st != o.st) return false;
  if (dim_head == 16 && (g.mode != 0 || bf16)) return false;  // dim 16: the ada C = 256 windows, f16x3
  int groups, nt = 1;
  if (g.mode == 0) {
    const int N = g.ws0 * g.ws1 * g.ws2;
    if (N > 64) return false;
    nt = N > 32 ? 2 : 1;
    groups = (g.Dp / g.ws0) * (g.Hp / g.ws1) * (g.Wp / g.ws2);
  } else {
    if (g.D > 32) return false;
    const int ppw = 32 / (g.D <= 16 ? 16 : 32);  // pixels per 32-token group
    groups = (g.H * g.W + ppw - 1) / ppw;
  }
  const int total = qkv.B * groups;
  int* flag = x3_range_ptr();
  // EXTDM_CORE_XCD=0: dispatch order (A/B)
  static const bool xcd_on = [] { const char* v = getenv("EXTDM_CORE_XCD"); return !(v && v[0] == '0'); }();
  const int xcd = xcd_on && total >= 64 ? 1 : 0;
  const int grid = xcd ? (total + 7) & ~7 : total;
#define CORE_GO(M, X, NT_, DH_)                                                                              \
  do {                                                                                                       \
  note_kernel("attn_core_kernel<%d, %s, %d, %d>", M, X ? "true" : "false", NT_, DH_);                         \
  hipLaunchKernelGGL((attn_core_kernel<M, X, NT_, DH_>), dim3(grid), dim3(256), 0, s, qkv.p, qkv.sb, qkv.sc,      \
                     qkv.st, o.p, o.sb, o.sc, g, heads, groups, total, bias_dense, bstride, rope_cos, rope_sin,    \
                     q_scale, flag, xcd);                                                                     \
  } while (0)
  if (dim_head == 16) {
    if (nt == 2) CORE_GO(0, true, 2, 16);
    else CORE_GO(0, true, 1, 16);
  } else if (g.mode == 0 && nt == 2) {
    if (bf16) CORE_GO(0, false, 2, 32);
    else CORE_GO(0, true, 2, 32);
  } else if (g.mode == 0) {
    if (bf16) CORE_GO(0, false, 1, 32);
    else CORE_GO(0, true, 1, 32);
  } else {
    if (bf16) CORE_GO(1, false, 1, 32);
    else CORE_GO(1, true, 1, 32);
  }
#undef CORE_GO
  return true;
}

}  // namespace extdm
