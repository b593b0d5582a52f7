// Direct (1,k,k) convolution, stride 1, "same" padding, k in {1, 3, 7}, on
// fp32 MFMA with LDS-staged halo tiles — the hot conv of the sampling path
// (Block.proj u12:165, init_conv / init_noise_conv u12:913-914, every 1x1
// projection, LFAE decoder convs util.py:69-149).
//
// A block owns BM output channels x 128 output pixels, the pixels being NP
// whole-width row bands of TH rows (NP*TH*W = 128). Per K stage it stages
//   X: CIB input channels x NP planes x (TH+k-1) rows x (W+k-1) cols (zero halo)
//   A: the matching weights, pre-packed [mtile][stage][step][half][BM]
// in LDS (double buffered, next stage prefetched into registers). The MFMA
// loop then needs no index arithmetic: for step (ci', ky, kx) every lane reads
//   A: As[step][half][m]             and   B: Xs[half*CH + ci'][pixel + ky*RS + kx]
// where lane half h (the MFMA's k parity) takes input channel ci' + h*CH.
// Each input element is fetched from HBM/L2 once per (block, stage) instead of
// k*k times as in an im2col gather.
#include <algorithm>

#include "kernels.h"

namespace extdm {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

struct HaloArgs {
  const float* in0; const float* in1;
  long i0b, i0c, i0t, i1b, i1c, i1t;
  int C0, Cin, H, W, T, P;
  const float* w; int stages;
  float* out; long ob, oc, ot; int Cout;
  int TH, NP, nrow_tiles, RS, XPC;
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

template <int KS> struct XMax;
template <> struct XMax<1> { static constexpr int v = 128; };
template <> struct XMax<3> { static constexpr int v = 288; };
template <> struct XMax<7> { static constexpr int v = 560; };

template <int KS, int BM, int CH, int BNP>
__global__ __launch_bounds__(256) void conv_halo_kernel(HaloArgs a) {
  constexpr int KK = KS * KS;
  constexpr int PAD = KS / 2;
  constexpr int CIB = 2 * CH;
  constexpr int STEPS = CH * KK;
  constexpr int AFL = STEPS * 2 * BM;          // A floats per stage
  constexpr int XJ = (CIB * XMax<KS>::v + 255) / 256;
  // BNP = pixels per block tile: 128 (2x2 waves) or 32 (4 waves stacked over BM = 128)
  constexpr int WAVES_N = BNP == 128 ? (BM >= 64 ? 2 : 4) : 1;
  constexpr int WAVES_M = 4 / WAVES_N;
  constexpr int TM = BM / (32 * WAVES_M);
  constexpr int TN = BNP / (32 * WAVES_N);
  static_assert(TM >= 1 && TN >= 1, "bad tile");

  extern __shared__ float smem[];
  const int XFL = CIB * a.XPC;
  float* As0 = smem;
  float* Xs0 = smem + AFL;
  float* As1 = Xs0 + XFL;
  float* Xs1 = As1 + AFL;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int h = lane >> 5, lc = lane & 31;
  const int tile = blockIdx.x;
  const int plane0 = (tile / a.nrow_tiles) * a.NP;
  const int row0 = (tile % a.nrow_tiles) * a.TH;
  const int mtile = blockIdx.y;
  const int THK = a.TH + KS - 1;
  const float* wt = a.w + (long)mtile * a.stages * AFL;

  // ---- per-thread X staging slots (same every stage; only the channel moves) ----
  int xci[XJ];     // channel within the stage, -1 = no slot
  int xoff[XJ];    // iy*W + ix or -1 for a zero (halo / out-of-range) element
  long xb0[XJ], xb1[XJ];
#pragma unroll
  for (int j = 0; j < XJ; ++j) {
    const int e = tid + 256 * j;
    xci[j] = -1; xoff[j] = -1; xb0[j] = 0; xb1[j] = 0;
    if (e < XFL) {
      const int cl = e / a.XPC;
      const int rem = e - cl * a.XPC;
      const int p = rem / (THK * a.RS);
      const int r2 = rem - p * THK * a.RS;
      const int rr = r2 / a.RS, cc = r2 - rr * a.RS;
      const int q = plane0 + p;
      const int iy = row0 + rr - PAD, ix = cc - PAD;
      xci[j] = cl;
      if (q < a.P && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) {
        xoff[j] = iy * a.W + ix;
        const int b = q / a.T, t = q - (q / a.T) * a.T;
        xb0[j] = (long)b * a.i0b + (long)t * a.i0t;
        xb1[j] = (long)b * a.i1b + (long)t * a.i1t;
      }
    }
  }

  float xr[XJ];
  // A: contiguous in global and LDS -> LDS-DMA (global_load_lds_dwordx4), 1 KiB per wave-instruction
  constexpr int NPIECE = (AFL + 255) / 256;
#define HALO_LOAD(ST, AS)                                                                         \
  do {                                                                                            \
    _Pragma("unroll") for (int j = 0; j < XJ; ++j) {                                              \
      float v = 0.f;                                                                              \
      const int ci = (ST) * CIB + xci[j];                                                         \
      if (xoff[j] >= 0 && ci < a.Cin)                                                             \
        v = ci < a.C0 ? a.in0[xb0[j] + (long)ci * a.i0c + xoff[j]]                                 \
                      : a.in1[xb1[j] + (long)(ci - a.C0) * a.i1c + xoff[j]];                       \
      xr[j] = v;                                                                                  \
    }                                                                                             \
    const float* src_ = wt + (long)(ST) * AFL;                                                    \
    for (int pc = wave; pc < NPIECE; pc += 4) {                                                   \
      if (pc * 256 + lane * 4 < AFL)                                                              \
        __builtin_amdgcn_global_load_lds((const void*)(src_ + pc * 256 + lane * 4),               \
                                         (lds_ptr_t)((AS) + pc * 256), 16, 0, 0);                 \
    }                                                                                             \
  } while (0)
#define HALO_STORE(XS)                                                                            \
  do {                                                                                            \
    _Pragma("unroll") for (int j = 0; j < XJ; ++j) {                                              \
      if (tid + 256 * j < XFL) (XS)[tid + 256 * j] = xr[j];                                       \
    }                                                                                             \
  } while (0)

  // ---- per-lane operand bases ----
  int boff[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = (wn * TN + j) * 32 + lc;  // pixel within the block tile
    const int p = n / (a.TH * a.W);
    const int r = (n / a.W) % a.TH;
    const int c = n % a.W;
    boff[j] = h * CH * a.XPC + (p * THK + r) * a.RS + c;
  }
  const int aoff = h * BM + wm * TM * 32 + lc;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  HALO_LOAD(0, As0);
  HALO_STORE(Xs0);
  __syncthreads();
  for (int st = 0; st < a.stages; ++st) {
    float* As = (st & 1) ? As1 : As0;
    float* Xs = (st & 1) ? Xs1 : Xs0;
    if (st + 1 < a.stages) HALO_LOAD(st + 1, (st & 1) ? As0 : As1);
#pragma unroll
    for (int cp = 0; cp < CH; ++cp) {
      const float* xb = Xs + cp * a.XPC;
#pragma unroll
      for (int ky = 0; ky < KS; ++ky) {
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) {
          const int step = (cp * KS + ky) * KS + kx;
          float av[TM], bv[TN];
#pragma unroll
          for (int i = 0; i < TM; ++i) av[i] = As[step * 2 * BM + aoff + i * 32];
          const int so = ky * a.RS + kx;
#pragma unroll
          for (int j = 0; j < TN; ++j) bv[j] = xb[boff[j] + so];
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
        }
      }
    }
    if (st + 1 < a.stages) HALO_STORE((st & 1) ? Xs0 : Xs1);
    // the next stage's A pieces were LDS-DMA'd by several waves: each drains its own
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

#undef HALO_LOAD
#undef HALO_STORE
  // ---- epilogue ----
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = (wn * TN + j) * 32 + lc;
    const int p = n / (a.TH * a.W);
    const int r = (n / a.W) % a.TH;
    const int c = n % a.W;
    const int q = plane0 + p, row = row0 + r;
    if (q >= a.P || row >= a.H) continue;
    const int b = q / a.T, t = q - (q / a.T) * a.T;
    const long pix = (long)row * a.W + c;
    const long obase = (long)b * a.ob + (long)t * a.ot + pix;
    const long rbase = (long)b * a.e.res_sb + (long)t * a.e.res_st + pix;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r16 = 0; r16 < 16; ++r16) {
        const int m = mtile * BM + (wm * TM + i) * 32 + (r16 & 3) + 8 * (r16 >> 2) + 4 * h;
        if (m >= a.Cout) continue;
        float v = acc[i][j][r16];
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

template <int KS, int BM, int CH, int BNP>
void launch(hipStream_t s, const HaloArgs& a, unsigned ntiles) {
  constexpr int AFL = CH * KS * KS * 2 * BM;
  const size_t lds = (size_t)2 * (AFL + 2 * CH * a.XPC) * sizeof(float);
  dim3 grid(ntiles, (a.Cout + BM - 1) / BM);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_halo_kernel<KS, BM, CH, BNP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((conv_halo_kernel<KS, BM, CH, BNP>), grid, dim3(256), lds, s, a);
}

}  // namespace

int halo_ch(int ks, int bm) {
  if (ks == 1) return 8;
  if (ks == 3) return bm == 128 ? 2 : 4;
  return 1;  // 7x7
}

bool conv_halo_forward(hipStream_t s, const View& out, const View& in0, const View* in1, const PackedW& w,
                       const ConvEpi& epi) {
  if (!w.wh || w.mode != MODE_CONV) return false;
  const int ks = w.KH;
  const int H = in0.H, W = in0.W;
  if (out.H != H || out.W != W || W > 128 || 128 % W != 0) return false;
  HaloArgs a{};
  const int P = out.B * out.T;
  const int bm = w.hbm;
  // small pixel counts (4x4 / 8x8 levels): 32-pixel tiles so the grid still fills 256 CUs
  int bnp = 128;
  {
    const int th = std::min(H, 128 / W), np = 128 / (th * W);
    const long blocks128 = (long)((P + np - 1) / np) * ((H + th - 1) / th) * ((out.C + bm - 1) / bm);
    if (bm == 128 && W <= 32 && blocks128 < 512) bnp = 32;
  }
  a.TH = std::min(H, bnp / W);
  a.NP = bnp / (a.TH * W);
  a.RS = W + ks - 1;
  a.XPC = a.NP * (a.TH + ks - 1) * a.RS;
  const int xmax = ks == 1 ? 128 : (ks == 3 ? 288 : 560);
  if (a.XPC > xmax) return false;
  a.in0 = in0.p; a.i0b = in0.sb; a.i0c = in0.sc; a.i0t = in0.st; a.C0 = in0.C;
  if (in1) { a.in1 = in1->p; a.i1b = in1->sb; a.i1c = in1->sc; a.i1t = in1->st; a.Cin = in0.C + in1->C; }
  else { a.in1 = in0.p; a.i1b = in0.sb; a.i1c = in0.sc; a.i1t = in0.st; a.Cin = in0.C; }
  a.H = H; a.W = W; a.T = out.T; a.P = P;
  a.w = w.wh; a.stages = w.hstages;
  a.out = out.p; a.ob = out.sb; a.oc = out.sc; a.ot = out.st; a.Cout = out.C;
  a.nrow_tiles = (H + a.TH - 1) / a.TH;
  a.e = epi;
  const unsigned ntiles = (unsigned)(((a.P + a.NP - 1) / a.NP) * a.nrow_tiles);
#define HALO_GO(K, BMv, CHv)                                                         \
  do {                                                                               \
    if (bnp == 32) launch<K, BMv, CHv, 32>(s, a, ntiles);                            \
    else launch<K, BMv, CHv, 128>(s, a, ntiles);                                     \
  } while (0)
  if (ks == 1) { if (bm == 128) HALO_GO(1, 128, 8); else launch<1, 64, 8, 128>(s, a, ntiles); }
  else if (ks == 3) { if (bm == 128) HALO_GO(3, 128, 2); else launch<3, 64, 4, 128>(s, a, ntiles); }
  else if (ks == 7) { if (bm == 128) HALO_GO(7, 128, 1); else launch<7, 64, 1, 128>(s, a, ntiles); }
#undef HALO_GO
  else return false;
  return true;
}

}  // namespace extdm
