// Implicit-GEMM (1,k,k) convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Covers every conv / linear of the sampling path (u12:124-135, 165, 191,
// 453-455, 661-665, 703-704, 750-753, 810, 913-914, 986-1003; LFAE util.py:69-149):
//   C[m][n] = sum_k A[m][k] * B[k][n]
//   m = output channel, n = (b, t, oy, ox) output pixel, k = (ci, ky, kx)
//   A = packed weights [Kpad][Mpad] (k-major, so a BK x BM tile is contiguous)
//   B = im2col gathered on the fly from up to two channel sources (fused cat)
// Block tile BM x 128 x BK16, 256 threads = 4 waves, LDS double buffer with a
// register prefetch of the next K tile. f32 MFMA is exact f32 (a k-ordered
// fmaf chain), so numerics are those of an fp32 conv.
// MODE_DECONV runs ConvTranspose(1,4,4)/s2/p1 as four 2x2 parity convs
// (blockIdx.z = parity); MODE_UP2 reads a nearest-x2-upsampled input.
#include <cstdlib>
#include <stdexcept>

#include "kernels.h"

namespace extdm {

namespace {

constexpr int BN = 128;
constexpr int BK = 16;

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct ConvArgs {
  const float* in0; const float* in1;
  long i0b, i0c, i0t, i1b, i1c, i1t;
  int C0, Cin, Hin, Win;
  const float* w; int Kpad, Mpad, K;
  float* out; long ob, oc, ot;
  int Cout, Ho, Wo, T, B;  // Ho/Wo: pixel grid the GEMM iterates (parity grid for deconv)
  int OWfull;              // full output row width (for deconv addressing)
  int stride, pad;
  ConvEpi e;
  long N;
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

template <int KH, int KW, int BM, int MODE>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvArgs a) {
  constexpr int WAVES_M = BM >= 64 ? 2 : 1;
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int TM = BM / (32 * WAVES_M);
  constexpr int TN = BN / (32 * WAVES_N);
  constexpr int KK = KH * KW;

  __shared__ float As[2][BK][BM];
  __shared__ float Bs[2][BK][BN];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WAVES_N;
  const int wn = wave % WAVES_N;
  const long n0 = (long)blockIdx.x * BN;
  const int m0 = blockIdx.y * BM;
  const int par = blockIdx.z;               // deconv parity (py, px)
  const int py = par >> 1, px = par & 1;
  const float* wbase = a.w + (MODE == MODE_DECONV ? (long)par * a.Kpad * a.Mpad : 0);

  // ---- per-thread gather column (B operand) ----
  const int col = tid & (BN - 1);
  const int krow = tid >> 7;  // 0/1, uniform per wave
  const long n = n0 + col;
  const bool nvalid = n < a.N;
  int iy0 = 0, ix0 = 0;
  long base0 = 0, base1 = 0;
  {
    long nn = nvalid ? n : 0;
    int ox = (int)(nn % a.Wo); nn /= a.Wo;
    int oy = (int)(nn % a.Ho); nn /= a.Ho;
    int t = (int)(nn % a.T);
    int b = (int)(nn / a.T);
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

  float breg[BK / 2];
  constexpr int NA4 = BK * BM / 4;  // float4 loads per A tile (<= 512)
  float4 areg0 = make_float4(0.f, 0.f, 0.f, 0.f), areg1 = areg0;

  auto load_tile = [&](int k0) {
#pragma unroll
    for (int j = 0; j < BK / 2; ++j) {
      const int k = __builtin_amdgcn_readfirstlane(k0 + krow + 2 * j);
      const int ci = k / KK;
      const int r = k - ci * KK;
      const int ky = r / KW;
      const int kx = r - ky * KW;
      const int iy = iy0 + ky, ix = ix0 + kx;
      float v = 0.f;
      if (nvalid && k < a.K && iy >= 0 && iy < Hv && ix >= 0 && ix < Wv) {
        const int sy = MODE == MODE_UP2 ? (iy >> 1) : iy;
        const int sx = MODE == MODE_UP2 ? (ix >> 1) : ix;
        const float* src = ci < a.C0 ? a.in0 + base0 + (long)ci * a.i0c
                                     : a.in1 + base1 + (long)(ci - a.C0) * a.i1c;
        v = src[(long)sy * a.Win + sx];
      }
      breg[j] = v;
    }
    if (tid < NA4) {
      const int row = tid / (BM / 4), c4 = tid % (BM / 4);
      areg0 = *reinterpret_cast<const float4*>(wbase + (long)(k0 + row) * a.Mpad + m0 + c4 * 4);
    }
    if constexpr (NA4 > 256) {
      const int idx = tid + 256;
      const int row = idx / (BM / 4), c4 = idx % (BM / 4);
      areg1 = *reinterpret_cast<const float4*>(wbase + (long)(k0 + row) * a.Mpad + m0 + c4 * 4);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int j = 0; j < BK / 2; ++j) Bs[buf][krow + 2 * j][col] = breg[j];
    if (tid < NA4) {
      const int row = tid / (BM / 4), c4 = tid % (BM / 4);
      *reinterpret_cast<float4*>(&As[buf][row][c4 * 4]) = areg0;
    }
    if constexpr (NA4 > 256) {
      const int idx = tid + 256;
      const int row = idx / (BM / 4), c4 = idx % (BM / 4);
      *reinterpret_cast<float4*>(&As[buf][row][c4 * 4]) = areg1;
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = a.Kpad / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  const int lrow = lane >> 5, lcol = lane & 31;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load_tile((kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i] = As[buf][kk + lrow][(wm * TM + i) * 32 + lcol];
#pragma unroll
      for (int j = 0; j < TN; ++j) bv[j] = Bs[buf][kk + lrow][(wn * TN + j) * 32 + lcol];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tile(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue ----
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const long nn0 = n0 + (wn * TN + j) * 32 + lcol;
    if (nn0 >= a.N) continue;
    long nn = nn0;
    int ox = (int)(nn % a.Wo); nn /= a.Wo;
    int oy = (int)(nn % a.Ho); nn /= a.Ho;
    int t = (int)(nn % a.T);
    int b = (int)(nn / a.T);
    long pix;
    if (MODE == MODE_DECONV) pix = (long)(2 * oy + py) * a.OWfull + (2 * ox + px);
    else pix = (long)oy * a.Wo + ox;
    const long obase = (long)b * a.ob + (long)t * a.ot + pix;
    const long rbase = (long)b * a.e.res_sb + (long)t * a.e.res_st + pix;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * lrow;
        if (m >= a.Cout) continue;
        float v = acc[i][j][r];
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

bool getenv_flag(const char* n) {
  static int cached = -1;
  if (cached < 0) { const char* v = getenv(n); cached = (v && v[0] && v[0] != '0') ? 1 : 0; }
  return cached == 1;
}

template <int KH, int KW, int MODE>
void launch_bm(hipStream_t s, const ConvArgs& a, int bm, dim3 grid_n) {
  dim3 block(256);
  if (bm == 128) {
    dim3 g(grid_n.x, (a.Cout + 127) / 128, grid_n.z);
    hipLaunchKernelGGL((conv_gemm_kernel<KH, KW, 128, MODE>), g, block, 0, s, a);
  } else if (bm == 64) {
    dim3 g(grid_n.x, (a.Cout + 63) / 64, grid_n.z);
    hipLaunchKernelGGL((conv_gemm_kernel<KH, KW, 64, MODE>), g, block, 0, s, a);
  } else {
    dim3 g(grid_n.x, (a.Cout + 31) / 32, grid_n.z);
    hipLaunchKernelGGL((conv_gemm_kernel<KH, KW, 32, MODE>), g, block, 0, s, a);
  }
}

}  // namespace

int conv_forward(hipStream_t s, const View& out, const View& in0, const View* in1, const PackedW& w,
                 int stride, int pad, const ConvEpi& epi_in) {
  int slots = 0;
  if (w.mode == MODE_CONV && stride == 1 && w.KH == 1 && w.KW == 1 && pad == 0 && !in1 &&
      pw_x3_forward(s, out, in0, w, epi_in))
    return 0;
  if (w.wv && conv_narrow_forward(s, out, in0, in1, w, stride, pad, epi_in)) return 0;
  if (w.mode == MODE_CONV && stride == 1 && w.KH == w.KW && pad == w.KH / 2 &&
      conv_x3_forward(s, out, in0, in1, w, epi_in, &slots))
    return slots;
  if (epi_in.res_aff) throw std::invalid_argument("conv: residual GroupNorm needs the f16x3 direct conv");
  ConvEpi epi = epi_in;  // the other paths leave the statistics to the caller
  epi.stats = nullptr;
  if (conv_gemm_x3_forward(s, out, in0, in1, w, stride, pad, epi)) return 0;
  if (w.mode == MODE_CONV && stride == 1 && w.KH == w.KW && pad == w.KH / 2 && !getenv_flag("EXTDM_NO_HALO") &&
      conv_halo_forward(s, out, in0, in1, w, epi))
    return 0;
  ConvArgs a{};
  a.in0 = in0.p; a.i0b = in0.sb; a.i0c = in0.sc; a.i0t = in0.st;
  a.C0 = in0.C;
  if (in1) { a.in1 = in1->p; a.i1b = in1->sb; a.i1c = in1->sc; a.i1t = in1->st; a.Cin = in0.C + in1->C; }
  else { a.in1 = in0.p; a.i1b = in0.sb; a.i1c = in0.sc; a.i1t = in0.st; a.Cin = in0.C; }
  a.Hin = in0.H; a.Win = in0.W;
  a.w = w.w; a.Kpad = w.Kpad; a.Mpad = w.Mpad; a.K = w.K;
  a.out = out.p; a.ob = out.sb; a.oc = out.sc; a.ot = out.st;
  a.Cout = out.C; a.T = out.T; a.B = out.B;
  a.stride = stride; a.pad = pad;
  a.e = epi;
  a.OWfull = out.W;
  if (w.mode == MODE_DECONV) { a.Ho = in0.H; a.Wo = in0.W; }
  else { a.Ho = out.H; a.Wo = out.W; }
  a.N = (long)a.B * a.T * a.Ho * a.Wo;
  const int bm = conv_bm(w.M);  // the packer padded Mpad to a multiple of this tile
  dim3 gn((unsigned)((a.N + BN - 1) / BN), 1, w.mode == MODE_DECONV ? 4 : 1);
  const int kh = w.KH, kw = w.KW;
  if (w.mode == MODE_DECONV) { launch_bm<2, 2, MODE_DECONV>(s, a, bm, gn); return 0; }
  if (w.mode == MODE_UP2) { launch_bm<3, 3, MODE_UP2>(s, a, bm, gn); return 0; }
  if (kh == 1 && kw == 1) launch_bm<1, 1, MODE_CONV>(s, a, bm, gn);
  else if (kh == 3 && kw == 3) launch_bm<3, 3, MODE_CONV>(s, a, bm, gn);
  else if (kh == 4 && kw == 4) launch_bm<4, 4, MODE_CONV>(s, a, bm, gn);
  else if (kh == 7 && kw == 7) launch_bm<7, 7, MODE_CONV>(s, a, bm, gn);
  return 0;
}

}  // namespace extdm
