// Implicit-GEMM convolution on fp16 MFMA with the f16x3 split (see conv_x3.hip): the
// convs the direct kernel does not take -- strided Downsample (1,4,4)/s2 (u12:124-135),
// the ConvTranspose parity GEMMs (u12:117-121), nearest-x2 up convs and small-Cin convs
// such as init_noise_conv 3->256 7x7 (u12:914) and the LFAE convs (util.py:69-149).
//   C[m][n] = sum_k A[m][k] B[k][n],  m = output channel, n = (b, t, oy, ox),
//   k = (ci, ky, kx); B = im2col gathered on the fly from up to two channel sources.
// Block tile BM x 128 x 32 (two MFMA k-steps), 256 threads = 4 waves, LDS double buffer
// with a register prefetch of the next K tile (as conv.hip's fp32 kernel).
// A is pre-packed per (mtile, ktile) as [step][m32][hi|lo][lane][8] (lane-linear 16-B
// fragments, rows pre-scaled by powers of two, undone by gscale[m] in the epilogue);
// B is split into hi / lo while staging, as [hi|lo][step][n][16 k] with the 16-B halves
// of a row swapped on bit 3 of n (conflict-free ds_read_b128 over 16 lanes).
#include <algorithm>
#include <cstdlib>

#include "kernels.h"

namespace extdm {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

constexpr int BN = 128;
constexpr int BK = 32;

struct GArgs {
  const float* in0; const float* in1;
  long i0b, i0c, i0t, i1b, i1c, i1t;
  int C0, Cin, Hin, Win;
  const _Float16* w; const float* wscale; int nkt;
  float* out; long ob, oc, ot;
  int Cout, Ho, Wo, T, B;
  int OWfull;
  int stride, pad;
  ConvEpi e;
  long N;
  int* range;
  int in_bytes;  // FAST: byte extent of in0 (the buffer descriptor's range; < 2^30)
  const _Float16* wt; int nkt_t;  // TAPK: the tap-major packing (nullptr: none)
};

__device__ __forceinline__ float act_apply(float v, int act) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_GELU: return 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
    case ACT_SILU: return v / (1.f + expf(-v));
    case ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    default: return v;
  }
}

// FAST (KH * KW divides 32, no nearest-up, one source; the host checks the byte extents fit
// 31 bits): a thread's 16 gather elements per K tile have the same taps (ky, kx) in every
// tile -- the tile's channels are the only change, and they are wave-uniform -- so the
// element's in-image test and its byte offset are computed once, and each load is a buffer
// load with that offset (an invalid tap's offset lies past the extent: the load returns 0)
// and the tile's channel offset in soffset: no per-element address math or branch.
// TAPK (tap-major K, k = tap * Cin + ci; Cin and the first source's channels multiples of 8,
// 32-bit byte offsets; the host checks): a thread's 8-element gather group is 8 channels of
// one tap of one source, so the tap, its in-image test and the pixel's byte offset are
// computed once per group, the channel planes are wave-uniform bases (saddr loads), and the
// nearest-x2 up convs gather the same way. For the 3x3 / 7x7 / up convs the ci-major order
// leaves to the per-element path (32 % KH * KW != 0).
template <int KH, int KW, int BM, int MODE, bool FAST = false, bool TAPK = false>
__global__ __launch_bounds__(256) void conv_gemm_x3_kernel(GArgs a) {
  constexpr int WAVES_M = BM >= 64 ? 2 : 1;
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int TM = BM / (32 * WAVES_M);
  constexpr int TN = BN / (32 * WAVES_N);
  constexpr int KK = KH * KW;
  constexpr int M32 = BM / 32;
  constexpr int AH = 2 * M32 * 2 * 512;  // halves per A tile (2 steps, hi + lo)
  constexpr int BH = 2 * 2 * BN * 16;    // halves per B tile ([hl][step][n][16])
  constexpr int APASS = AH / 2048;       // 16-B chunks of 256 threads per A tile

  extern __shared__ __attribute__((aligned(16))) _Float16 smg[];
  _Float16* As0 = smg;
  _Float16* As1 = smg + AH;
  _Float16* Bs0 = smg + 2 * AH;
  _Float16* Bs1 = Bs0 + BH;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WAVES_N;
  const int wn = wave % WAVES_N;
  const int h = lane >> 5, lc = lane & 31;
  // XCD-aware column-tile order (conv_x3.hip tile note): XCD k takes a contiguous range of
  // column tiles, so the input rows neighbouring tiles both gather come from its L2
  const long nb = (gridDim.x & 7) ? (long)blockIdx.x : (long)((blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3));
  const long n0 = nb * BN;
  const int mt = blockIdx.y;
  const int par = blockIdx.z;  // deconv parity (py, px)
  const int py = par >> 1, px = par & 1;
  const _Float16* wbase = a.w + ((long)par * gridDim.y + mt) * a.nkt * AH;  // a.w / a.nkt: the launch's packing

  // ---- per-thread gather column (B operand): column col, k groups kg and kg + 2 ----
  const int col = tid & (BN - 1);
  const int kg = tid >> 7;  // 0/1, uniform per wave
  const long n = n0 + col;
  const bool nvalid = n < a.N;
  int iy0 = 0, ix0 = 0;
  long base0 = 0, base1 = 0;
  {
    long nn = nvalid ? n : 0;
    const int ox = (int)(nn % a.Wo); nn /= a.Wo;
    const int oy = (int)(nn % a.Ho); nn /= a.Ho;
    const int t = (int)(nn % a.T);
    const int b = (int)(nn / a.T);
    if (MODE == MODE_DECONV) {
      iy0 = oy - (1 - py);
      ix0 = ox - (1 - px);
    } else {
      iy0 = oy * a.stride - a.pad;
      ix0 = ox * a.stride - a.pad;
    }
    base0 = (long)b * a.i0b + (long)t * a.i0t;
    base1 = (long)b * a.i1b + (long)t * a.i1t;
  }
  const int Hv = MODE == MODE_UP2 ? 2 * a.Hin : a.Hin;
  const int Wv = MODE == MODE_UP2 ? 2 * a.Win : a.Win;
  const int K = a.Cin * KK;

  float breg[2][8];
  u32x4 areg[APASS];  // ext_vector (HIP's uint4 struct kept the array in scratch)
  int bad = 0;

  static_assert(!FAST || (BK % KK == 0 && MODE != MODE_UP2), "FAST: taps repeat per K tile");
  constexpr int CPT = BK / KK;  // channels per K tile (FAST)
  constexpr int OOB = 0x40000000;
  int voff[2][8];
  // the range is the tensor's extent: an invalid tap's offset (OOB) lies past it and reads 0
  const auto rs_in = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.in0), 0, a.in_bytes, 0x00020000);
  if (FAST) {
#pragma unroll
    for (int g2 = 0; g2 < 2; ++g2)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int kl = 8 * (kg + 2 * g2) + e;  // wave-uniform
        const int tap = kl % KK;
        const int iy = iy0 + tap / KW, ix = ix0 + tap % KW;
        const bool ok = nvalid && iy >= 0 && iy < Hv && ix >= 0 && ix < Wv;
        voff[g2][e] = ok ? (int)((base0 + (long)iy * a.Win + ix) * 4) : OOB;
      }
  }

  auto load_tile = [&](int kt) __attribute__((always_inline)) {
    if (TAPK) {
#pragma unroll
      for (int g2 = 0; g2 < 2; ++g2) {
        const int kb = __builtin_amdgcn_readfirstlane(kt * BK + 8 * (kg + 2 * g2));
        const int tap = kb / a.Cin, ci0 = kb - tap * a.Cin;
        const int ky = tap / KW, kx = tap - ky * KW;
        const int iy = iy0 + ky, ix = ix0 + kx;
        const bool ok = nvalid && tap < KK && iy >= 0 && iy < Hv && ix >= 0 && ix < Wv;
        const int sy = MODE == MODE_UP2 ? (iy >> 1) : iy;
        const int sx = MODE == MODE_UP2 ? (ix >> 1) : ix;
        const bool s1 = ci0 >= a.C0;  // wave-uniform
        const unsigned vo = ok ? (unsigned)(((s1 ? base1 : base0) + (long)sy * a.Win + sx) * 4) : 0u;
        const float* plane = s1 ? a.in1 + (long)(ci0 - a.C0) * a.i1c : a.in0 + (long)(ci0 < a.Cin ? ci0 : 0) * a.i0c;
        const int cst4 = (int)((s1 ? a.i1c : a.i0c) * 4);
        // the group's first channel plane as the (uniform) buffer base: pixel offset in
        // voffset, channel e's plane offset in soffset
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(plane), 0, -1, 0x00020000);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)vo, e * cst4, 0));
          breg[g2][e] = ok ? v : 0.f;
        }
      }
      const u32x4* ap = reinterpret_cast<const u32x4*>(wbase + (long)kt * AH);
#pragma unroll
      for (int p = 0; p < APASS; ++p) areg[p] = ap[p * 256 + tid];
      return;
    }
    if (FAST) {
#pragma unroll
      for (int g2 = 0; g2 < 2; ++g2)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int ci = __builtin_amdgcn_readfirstlane(kt * CPT + (8 * (kg + 2 * g2) + e) / KK);
          const int cl = ci < a.Cin ? ci : a.Cin - 1;  // the K tail reads a real channel, zeroed
          const float v = __uint_as_float(
              __builtin_amdgcn_raw_buffer_load_b32(rs_in, voff[g2][e], (int)(cl * a.i0c * 4), 0));
          breg[g2][e] = ci < a.Cin ? v : 0.f;
        }
      const u32x4* ap = reinterpret_cast<const u32x4*>(wbase + (long)kt * AH);
#pragma unroll
      for (int p = 0; p < APASS; ++p) areg[p] = ap[p * 256 + tid];
      return;
    }
#pragma unroll
    for (int g2 = 0; g2 < 2; ++g2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = __builtin_amdgcn_readfirstlane(kt * BK + 8 * (kg + 2 * g2) + e);
        const int ci = k / KK;
        const int r = k - ci * KK;
        const int ky = r / KW;
        const int kx = r - ky * KW;
        const int iy = iy0 + ky, ix = ix0 + kx;
        float v = 0.f;
        if (nvalid && k < K && iy >= 0 && iy < Hv && ix >= 0 && ix < Wv) {
          const int sy = MODE == MODE_UP2 ? (iy >> 1) : iy;
          const int sx = MODE == MODE_UP2 ? (ix >> 1) : ix;
          const float* src = ci < a.C0 ? a.in0 + base0 + (long)ci * a.i0c
                                       : a.in1 + base1 + (long)(ci - a.C0) * a.i1c;
          v = src[(long)sy * a.Win + sx];
        }
        breg[g2][e] = v;
      }
    }
    const u32x4* ap = reinterpret_cast<const u32x4*>(wbase + (long)kt * AH);
#pragma unroll
    for (int p = 0; p < APASS; ++p) areg[p] = ap[p * 256 + tid];
  };
  auto store_tile = [&](_Float16* As, _Float16* Bs) __attribute__((always_inline)) {
#pragma unroll
    for (int g2 = 0; g2 < 2; ++g2) {
      const int g = kg + 2 * g2;  // 8-k group: step g >> 1, half g & 1
      unsigned hw[4], lw[4];
      float am = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        split2s(breg[g2][2 * e], breg[g2][2 * e + 1], hw[e], lw[e]);
        amax2(am, breg[g2][2 * e], breg[g2][2 * e + 1]);
      }
      bad |= am >= 65504.f;
      const h8 hi = __builtin_bit_cast(h8, u32x4{hw[0], hw[1], hw[2], hw[3]});
      const h8 lo = __builtin_bit_cast(h8, u32x4{lw[0], lw[1], lw[2], lw[3]});
      _Float16* d = Bs + ((g >> 1) * BN + col) * 16 + 8 * ((g & 1) ^ ((col >> 3) & 1));
      *reinterpret_cast<h8*>(d) = hi;
      *reinterpret_cast<h8*>(d + 2 * BN * 16) = lo;
    }
    u32x4* ad = reinterpret_cast<u32x4*>(As);
#pragma unroll
    for (int p = 0; p < APASS; ++p) ad[p * 256 + tid] = areg[p];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  load_tile(0);
  store_tile(As0, Bs0);
  __syncthreads();
  for (int kt = 0; kt < a.nkt; ++kt) {
    const _Float16* As = (kt & 1) ? As1 : As0;
    const _Float16* Bs = (kt & 1) ? Bs1 : Bs0;
    // unconditional prefetch (the last tile re-loads itself into the idle buffer): under a
    // condition hipcc kept the A prefetch registers in scratch
    load_tile(kt + 1 < a.nkt ? kt + 1 : kt);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      h8 ah[TM], al[TM], ad[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const _Float16* p = As + ((s * M32 + wm * TM + i) * 2) * 512 + lane * 8;
        ah[i] = *reinterpret_cast<const h8*>(p);
        al[i] = *reinterpret_cast<const h8*>(p + 512);
        ad[i] = lo_dn(ah[i]);  // pairs with the scaled B lo (split2s, kernels.h)
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nc = (wn * TN + j) * 32 + lc;
        const _Float16* p = Bs + (s * BN + nc) * 16 + 8 * (h ^ ((nc >> 3) & 1));
        bh[j] = *reinterpret_cast<const h8*>(p);
        bl[j] = *reinterpret_cast<const h8*>(p + 2 * BN * 16);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          // the scaled-lo product last: its lo_dn VALU is off the head of the chain (-3 %,
          // interleaved A/B at B = 64)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ad[i], bl[j], acc[i][j], 0, 0, 0);
        }
    }
    store_tile((kt & 1) ? As0 : As1, (kt & 1) ? Bs0 : Bs1);
    __syncthreads();
  }
  if (bad) atomicOr(a.range, 1);

  // ---- epilogue (C/D map: col = lane & 31, row = (r&3) + 8(r>>2) + 4h) ----
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const long nn0 = n0 + (wn * TN + j) * 32 + lc;
    if (nn0 >= a.N) continue;
    long nn = nn0;
    const int ox = (int)(nn % a.Wo); nn /= a.Wo;
    const int oy = (int)(nn % a.Ho); nn /= a.Ho;
    const int t = (int)(nn % a.T);
    const int b = (int)(nn / a.T);
    long pix;
    if (MODE == MODE_DECONV) pix = (long)(2 * oy + py) * a.OWfull + (2 * ox + px);
    else pix = (long)oy * a.Wo + ox;
    const long obase = (long)b * a.ob + (long)t * a.ot + pix;
    const long rbase = (long)b * a.e.res_sb + (long)t * a.e.res_st + pix;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mt * BM + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m >= a.Cout) continue;
        float v = acc[i][j][r] * a.wscale[m];
        if (a.e.bias) v += a.e.bias[m];
        if (a.e.res) v += a.e.res[rbase + (long)m * a.e.res_sc];
        if (a.e.post_scale) {
          const long pi = a.e.post_per_channel ? (long)m : (long)b * a.Cout + m;
          v = v * a.e.post_scale[pi] + a.e.post_shift[pi];
        }
        v = act_apply(v, a.e.act);
        a.out[obase + (long)m * a.oc] = v;
      }
    }
  }
}

template <int KH, int KW, int BM, int MODE, bool FAST, bool TAPK = false>
void launch_f(hipStream_t s, const GArgs& a, dim3 grid) {
  constexpr int AH = 2 * (BM / 32) * 2 * 512, BH = 2 * 2 * BN * 16;
  const size_t lds = (size_t)2 * (AH + BH) * sizeof(_Float16);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_gemm_x3_kernel<KH, KW, BM, MODE, FAST, TAPK>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((conv_gemm_x3_kernel<KH, KW, BM, MODE, FAST, TAPK>), grid, dim3(256), lds, s, a);
}

// the tap-major gather (TAPK above): a tap-major packing, whole 8-channel groups per source,
// every pixel's byte offset (frame base included) below 2^32
bool gemm_tapk_ok(const GArgs& a, int two) {
  static const bool off = [] { const char* v = getenv("EXTDM_GEMM_NOTAPK"); return v && v[0] && v[0] != '0'; }();
  if (off || !a.wt || a.Cin % 8 != 0 || a.C0 % 8 != 0) return false;
  auto ext = [&](long sb, long sc, long st, int C) {
    return ((long)(a.B - 1) * sb + (long)(C - 1) * sc + (long)(a.T - 1) * st + (long)a.Hin * a.Win) * 4;
  };
  // the pixel part of an offset: (b, t) frame base + in-plane position (channel 0); the
  // soffset of channel 7 of a group
  const long e0 = ext(a.i0b, 0, a.i0t, 1), e1 = two ? ext(a.i1b, 0, a.i1t, 1) : 0;
  const long c7 = 7 * 4 * std::max(a.i0c, two ? a.i1c : 0L);
  return e0 + c7 < (1L << 32) - 1 && e1 + c7 < (1L << 32) - 1 && c7 < (1L << 31);
}

// the fast gather (FAST above): taps that repeat per K tile, one source, 31-bit byte offsets
bool gemm_fast_ok(const GArgs& a, int kk, int mode) {
  static const bool off = [] { const char* v = getenv("EXTDM_GEMM_NOFAST"); return v && v[0] && v[0] != '0'; }();
  if (off || BK % kk != 0 || mode == MODE_UP2 || a.Cin != a.C0) return false;
  const long bytes = ((long)(a.B - 1) * a.i0b + (long)(a.Cin - 1) * a.i0c + (long)(a.T - 1) * a.i0t +
                      (long)a.Hin * a.Win) * 4;
  return bytes < (1L << 30);
}
int gemm_in_bytes(const GArgs& a) {
  return (int)(((long)(a.B - 1) * a.i0b + (long)(a.Cin - 1) * a.i0c + (long)(a.T - 1) * a.i0t +
                (long)a.Hin * a.Win) * 4);
}

template <int KH, int KW, int BM, int MODE>
void launch(hipStream_t s, const GArgs& a, dim3 grid, bool two) {
  if constexpr (BK % (KH * KW) != 0 || MODE == MODE_UP2) {
    if (gemm_tapk_ok(a, two)) {
      GArgs f = a;
      f.w = a.wt;
      f.nkt = a.nkt_t;
      launch_f<KH, KW, BM, MODE, false, true>(s, f, grid);
      return;
    }
  }
  if constexpr (BK % (KH * KW) == 0 && MODE != MODE_UP2) {
    if (gemm_fast_ok(a, KH * KW, MODE)) {
      GArgs f = a;
      f.in_bytes = gemm_in_bytes(a);
      launch_f<KH, KW, BM, MODE, true>(s, f, grid);
      return;
    }
  }
  launch_f<KH, KW, BM, MODE, false>(s, a, grid);
}

template <int KH, int KW, int MODE>
bool launch_bm(hipStream_t s, const GArgs& a, int bm, dim3 grid, bool two) {
  if (bm == 128) launch<KH, KW, 128, MODE>(s, a, grid, two);
  else if (bm == 64) launch<KH, KW, 64, MODE>(s, a, grid, two);
  else if (bm == 32) launch<KH, KW, 32, MODE>(s, a, grid, two);
  else return false;
  return true;
}

}  // namespace

int gemm_x3_bm(int M) { return conv_bm(M); }

bool conv_gemm_x3_forward(hipStream_t s, const View& out, const View& in0, const View* in1, const PackedW& w,
                          int stride, int pad, const ConvEpi& epi) {
  if (!w.gx) return false;
  GArgs a{};
  a.in0 = in0.p; a.i0b = in0.sb; a.i0c = in0.sc; a.i0t = in0.st;
  a.C0 = in0.C;
  if (in1) { a.in1 = in1->p; a.i1b = in1->sb; a.i1c = in1->sc; a.i1t = in1->st; a.Cin = in0.C + in1->C; }
  else { a.in1 = in0.p; a.i1b = in0.sb; a.i1c = in0.sc; a.i1t = in0.st; a.Cin = in0.C; }
  a.Hin = in0.H; a.Win = in0.W;
  a.w = reinterpret_cast<const _Float16*>(w.gx); a.wscale = w.gscale; a.nkt = w.gnkt;
  a.out = out.p; a.ob = out.sb; a.oc = out.sc; a.ot = out.st;
  a.Cout = out.C; a.T = out.T; a.B = out.B;
  a.stride = stride; a.pad = pad;
  a.e = epi;
  a.OWfull = out.W;
  a.range = x3_range_ptr();
  a.wt = reinterpret_cast<const _Float16*>(w.gxt);
  a.nkt_t = w.gnkt_t;
  if (w.mode == MODE_DECONV) { a.Ho = in0.H; a.Wo = in0.W; }
  else { a.Ho = out.H; a.Wo = out.W; }
  a.N = (long)a.B * a.T * a.Ho * a.Wo;
  if (a.Cin * w.KH * w.KW > a.nkt * BK || out.C > w.M) return false;
  const int bm = w.gbm;
  dim3 grid((unsigned)((a.N + BN - 1) / BN), (unsigned)((w.M + bm - 1) / bm), w.mode == MODE_DECONV ? 4 : 1);
  const int kh = w.KH, kw = w.KW, mode = w.mode;
  if (mode == MODE_DECONV) {
    if (kh == 2 && kw == 2) return launch_bm<2, 2, MODE_DECONV>(s, a, bm, grid, in1 != nullptr);
    return false;
  }
  if (mode == MODE_UP2) {
    if (kh == 3 && kw == 3) return launch_bm<3, 3, MODE_UP2>(s, a, bm, grid, in1 != nullptr);
    return false;
  }
  if (kh == 1 && kw == 1) return launch_bm<1, 1, MODE_CONV>(s, a, bm, grid, in1 != nullptr);
  if (kh == 3 && kw == 3) return launch_bm<3, 3, MODE_CONV>(s, a, bm, grid, in1 != nullptr);
  if (kh == 4 && kw == 4) return launch_bm<4, 4, MODE_CONV>(s, a, bm, grid, in1 != nullptr);
  if (kh == 7 && kw == 7) return launch_bm<7, 7, MODE_CONV>(s, a, bm, grid, in1 != nullptr);
  return false;
}

}  // namespace extdm
