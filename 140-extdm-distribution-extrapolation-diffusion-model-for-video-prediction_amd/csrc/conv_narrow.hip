// Direct fp32 VALU convolution for the KS x KS convs with few output channels: the LFAE heads
// the MFMA tiles pad badly -- Generator.final 64 -> 3 7x7 (model/LFAE/generator.py:59, 198-199),
// the PixelwiseFlowPredictor's mask (K = regions + 1) and occlusion (1) 7x7 over the hourglass
// output (model/LFAE/pixelwise_flow_predictor.py:31-34, 140-150). On the implicit GEMM these ran at 5.6 (final,
// 3 of 32 rows live) and 13 TFLOP/s (mask, 65 of 128 rows), both gather-bound; here every FMA
// is a useful one and the arithmetic is exact fp32 (fmaf chains).
//
// Tile: TH x TW = 16 x 64 output pixels of one frame, 256 threads, each one row strip of PX = 4
// pixels x COT output channels (grid.y = output-channel groups). Input channels go through LDS
// CB = 4 at a time as (TH + KS - 1) x (TW + KS - 1) halo planes, zero outside the image; the next
// stage is prefetched into registers while the current one is used. The weights [group][ci][tap][COT]
// ([group][ci][tap][COT padded to 4]) go through LDS with them and are read at wave-uniform addresses
// (broadcast), COT per tap.
#include <cstdlib>
#include <stdexcept>

#include "kernels.h"

namespace extdm {

namespace {

constexpr int TH = 16, TW = 64, CB = 4, NT = 256, PX = 4;

struct NArgs {
  const float* in0; const float* in1;
  long i0b, i0c, i0t, i1b, i1c, i1t;
  int C0, Cin, H, W, T;
  const float* w;  // [G][Cin][KS * KS][COTP], zero past M and COT
  float* out; long ob, oc, ot;
  int Cout, ntw;
  ConvEpi e;
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

template <int KS, int COT>
__global__ __launch_bounds__(NT, COT >= 8 ? 2 : 3) void conv_narrow_kernel(NArgs a) {
  constexpr int R = KS / 2, XR = TH + KS - 1, XC = TW + KS - 1;
  constexpr int PLANE = XR * XC, NLD = (CB * PLANE + NT - 1) / NT, NX = PX + KS - 1;
  constexpr int COTP = (COT + 3) & ~3;  // a tap's weights padded to whole float4 reads
  constexpr int WST = CB * KS * KS * COTP, NLW = (WST + NT - 1) / NT;  // weights per stage
  static_assert(NX % 2 == 0 && XC % 2 == 0, "float2 window reads");
  static_assert(CB == 4, "the staging selects one of four channel planes");
  __shared__ __attribute__((aligned(16))) float xs[CB * PLANE];
  __shared__ __attribute__((aligned(16))) float ws[WST];

  const int tid = threadIdx.x;
  const int tyi = blockIdx.x / a.ntw, txi = blockIdx.x - tyi * a.ntw;
  const int y0 = tyi * TH, x0 = txi * TW;
  const int g = blockIdx.y;
  const int b = blockIdx.z / a.T, t = blockIdx.z - b * a.T;
  const float* s0 = a.in0 + (long)b * a.i0b + (long)t * a.i0t;
  const float* s1 = a.in1 + (long)b * a.i1b + (long)t * a.i1t;
  const int ty = tid >> 4, tx = (tid & 15) * PX;

  // the staging element i = tid + j * NT is (c, row, col) of the halo planes in every stage:
  // c << 24 | its in-plane offset, or -1 outside the image / past the planes, computed once
  int off[NLD];
#pragma unroll
  for (int j = 0; j < NLD; ++j) {
    const int i = tid + j * NT;
    const int c = i / PLANE, r = i - c * PLANE;
    const int row = r / XC, col = r - row * XC;
    const int iy = y0 - R + row, ix = x0 - R + col;
    off[j] = (i < CB * PLANE && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) ? (c << 24) | (iy * a.W + ix) : -1;
  }
  const float* wg = a.w + (long)g * a.Cin * KS * KS * COTP;
  float pre[NLD], prw[NLW];
  auto load = [&](int st) __attribute__((always_inline)) {
    // the stage's CB channel planes (wave-uniform; a channel past Cin reads plane 0, zeroed),
    // then unconditional loads from a clamped in-bounds address, zeroed after
    const float* cp[CB];
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int ch = st * CB + c < a.Cin ? st * CB + c : 0;
      cp[c] = ch < a.C0 ? s0 + (long)ch * a.i0c : s1 + (long)(ch - a.C0) * a.i1c;
    }
    const int nc = a.Cin - st * CB;
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int c = off[j] >> 24;
      const bool ok = off[j] >= 0 && c < nc;
      const float* src = c == 0 ? cp[0] : (c == 1 ? cp[1] : (c == 2 ? cp[2] : cp[3]));
      const float v = src[ok ? (off[j] & 0xffffff) : 0];
      pre[j] = ok ? v : 0.f;
    }
    // [ci][tap][COTP] of the stage's CB channels: one contiguous block
    const long w0 = (long)st * WST, wn = (long)a.Cin * KS * KS * COTP;
#pragma unroll
    for (int j = 0; j < NLW; ++j) {
      const int i = tid + j * NT;
      prw[j] = (i < WST && w0 + i < wn) ? wg[w0 + i] : 0.f;
    }
  };
  auto store = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int i = tid + j * NT;
      if (i < CB * PLANE) xs[i] = pre[j];
    }
#pragma unroll
    for (int j = 0; j < NLW; ++j) {
      const int i = tid + j * NT;
      if (i < WST) ws[i] = prw[j];
    }
  };

  float acc[COT][PX];
#pragma unroll
  for (int o = 0; o < COT; ++o)
#pragma unroll
    for (int q = 0; q < PX; ++q) acc[o][q] = 0.f;

  const int nst = (a.Cin + CB - 1) / CB;
  load(0);
  store();
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    if (st + 1 < nst) load(st + 1);
    const int nc = a.Cin - st * CB < CB ? a.Cin - st * CB : CB;
    for (int c = 0; c < nc; ++c) {
#pragma unroll 1
      for (int ky = 0; ky < KS; ++ky) {
        float xv[NX];
        const float* xr = xs + c * PLANE + (ty + ky) * XC + tx;
#pragma unroll
        for (int j = 0; j < NX; j += 2) {
          const float2 v = *reinterpret_cast<const float2*>(xr + j);
          xv[j] = v.x;
          xv[j + 1] = v.y;
        }
        const float4* wr = reinterpret_cast<const float4*>(ws + (c * KS + ky) * KS * COTP);  // uniform: broadcast
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) {
          float wv[COTP];
#pragma unroll
          for (int u = 0; u < COTP / 4; ++u) {
            const float4 w4 = wr[kx * (COTP / 4) + u];
            wv[4 * u] = w4.x; wv[4 * u + 1] = w4.y; wv[4 * u + 2] = w4.z; wv[4 * u + 3] = w4.w;
          }
#pragma unroll
          for (int o = 0; o < COT; ++o)
#pragma unroll
            for (int q = 0; q < PX; ++q) acc[o][q] = fmaf(xv[q + kx], wv[o], acc[o][q]);
        }
      }
    }
    __syncthreads();
    if (st + 1 < nst) {
      store();
      __syncthreads();
    }
  }

  const int oy = y0 + ty;
  if (oy >= a.H) return;
  const long obase = (long)b * a.ob + (long)t * a.ot + (long)oy * a.W;
  const long rbase = (long)b * a.e.res_sb + (long)t * a.e.res_st + (long)oy * a.W;
#pragma unroll
  for (int o = 0; o < COT; ++o) {
    const int m = g * COT + o;
    if (m >= a.Cout) break;
#pragma unroll
    for (int q = 0; q < PX; ++q) {
      const int ox = x0 + tx + q;
      if (ox >= a.W) break;
      float v = acc[o][q];
      if (a.e.bias) v += a.e.bias[m];
      if (a.e.res) v += a.e.res[rbase + (long)m * a.e.res_sc + ox];
      if (a.e.post_scale) {
        const long pi = a.e.post_per_channel ? (long)m : (long)b * a.Cout + m;
        v = v * a.e.post_scale[pi] + a.e.post_shift[pi];
      }
      a.out[obase + (long)m * a.oc + ox] = act_apply(v, a.e.act);
    }
  }
}

template <int KS, int COT>
void launch(hipStream_t s, const NArgs& a, dim3 grid) {
  hipLaunchKernelGGL((conv_narrow_kernel<KS, COT>), grid, dim3(NT), 0, s, a);
}

}  // namespace

bool narrow_off() {
  static const bool off = [] { const char* v = getenv("EXTDM_NO_NARROW"); return v && v[0] && v[0] != '0'; }();
  return off;
}

int narrow_cot(int KS, int M) {
  if (KS != 7 || !(M <= 16 || (M % 32 != 0 && M <= 80))) return 0;
  // fewest padded rows, each group's input staging priced at two output channels' FMAs
  static const int cands[] = {16, 13, 8, 4, 3, 2, 1};
  int best = 0;
  long bestcost = 1L << 30;
  for (int c : cands) {
    const long groups = (M + c - 1) / c, cost = groups * c + 2 * groups;
    if (cost < bestcost) { bestcost = cost; best = c; }
  }
  return best;
}

bool conv_narrow_forward(hipStream_t s, const View& out, const View& in0, const View* in1, const PackedW& w,
                         int stride, int pad, const ConvEpi& epi) {
  if (!w.wv || narrow_off() || w.mode != MODE_CONV || stride != 1 || w.KH != w.KW || pad != w.KH / 2 ||
      epi.res_aff)
    return false;
  const int cin = in1 ? in0.C + in1->C : in0.C;
  if (cin * w.KH * w.KW != w.K || out.C != w.M || in0.H != out.H || in0.W != out.W ||
      (in1 && (in1->H != out.H || in1->W != out.W)) || in0.T != out.T || (long)out.B * out.T > 65535)
    return false;
  NArgs a{};
  a.in0 = in0.p; a.i0b = in0.sb; a.i0c = in0.sc; a.i0t = in0.st; a.C0 = in0.C;
  if (in1) { a.in1 = in1->p; a.i1b = in1->sb; a.i1c = in1->sc; a.i1t = in1->st; }
  else { a.in1 = in0.p; a.i1b = in0.sb; a.i1c = in0.sc; a.i1t = in0.st; }
  a.Cin = cin; a.H = out.H; a.W = out.W; a.T = out.T;
  a.w = w.wv;
  a.out = out.p; a.ob = out.sb; a.oc = out.sc; a.ot = out.st;
  a.Cout = out.C;
  a.ntw = (out.W + TW - 1) / TW;
  a.e = epi;
  const int nth = (out.H + TH - 1) / TH;
  dim3 grid((unsigned)(a.ntw * nth), (unsigned)((w.M + w.vcot - 1) / w.vcot), (unsigned)(out.B * out.T));
  if (w.KH != 7) return false;
  switch (w.vcot) {
    case 16: launch<7, 16>(s, a, grid); break;
    case 13: launch<7, 13>(s, a, grid); break;
    case 8: launch<7, 8>(s, a, grid); break;
    case 4: launch<7, 4>(s, a, grid); break;
    case 3: launch<7, 3>(s, a, grid); break;
    case 2: launch<7, 2>(s, a, grid); break;
    case 1: launch<7, 1>(s, a, grid); break;
    default: return false;
  }
  return true;
}

}  // namespace extdm
