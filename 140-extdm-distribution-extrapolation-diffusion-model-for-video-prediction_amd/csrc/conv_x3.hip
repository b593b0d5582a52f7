// Direct (1,k,k) stride-1 'same' convolution, k in {1, 3, 7}, on fp16 MFMA with
// a three-term split that keeps fp32 accuracy ("f16x3"): every fp32 operand is
// written as hi + lo with hi = fp16(v), lo = fp16(v - hi), and
//     sum_k a_k b_k  ~=  sum_k (a_lo b_hi + a_hi b_lo + a_hi b_hi)
// with every product exact in the fp32 accumulator (11 x 11 significant bits).
// The dropped a_lo*b_lo term and the representation error of hi + lo are
// ~2^-22 relative, below fp32 accumulation error at these K (K = Cin*k*k up to
// 25 088); the Unet eps matches the fp64 evaluation as closely as the fp32
// CPU reference does (tests/test_gpu_parity.py). Weights are
// pre-scaled per output channel by a power of two (exact) so their lo parts stay
// normal in fp16; activations must satisfy |v| < 65504, which the staging checks
// (g_x3_range is raised otherwise and the runtime reports it).
//
// Covers the same convs as conv_halo.hip (Block.proj u12:165, init_conv
// u12:913, the 1x1 projections) at 16x the MFMA rate of v_mfma_f32_32x32x2_f32
// per instruction (3 instructions per product => 5.3x).
//
// Tiling: a block owns BM output channels x BN output pixels (NP planes x TH
// rows x W cols) and loops over (channel block of CIB = 16*NG, ky). Per channel
// block the zero-haloed input tile is staged once, split into hi/lo fp16 in LDS
// as [hl][group][pos][16 channels] (one ds_read_b128 = the 8 channels of one
// lane's MFMA k-slice); per (channel block, ky) the packed weight slice
// [step = (g, kx)][m32][hl][lane][8] streams in by LDS-DMA. Both are double
// buffered; the next channel block's input is prefetched into registers while
// the KS ky-iterations of the current one run.
#include <algorithm>
#include <cstdlib>

#include "kernels.h"

// EXTDM_X3_LIN: the staged (fp32-input) X tile of the one-group tiles in the operand layout
// [hl][c8][pos][8] (a lane's k-slice = one 16-B record, consecutive positions = consecutive
// records: conflict-free ds_read_b128 with no swizzle, and a kx step is an immediate offset)
// instead of [hl][pos][16] with the bit-3 swizzle
// 1 = every one-group staged tile, 2 (default) = the k >= 5 tiles only (the 5x5 phase conv:
// -2.5 %; the 3x3 128-row tile's LDS then no longer fits two workgroups per CU: +30 %)
#ifndef EXTDM_X3_LIN
#define EXTDM_X3_LIN 2
#endif
// EXTDM_X3_BUFX: the staged X loads as buffer loads (the lane's pixel offset in VGPR, the
// channel's offset in soffset, a position outside the image past the extent so the load itself
// returns 0): no 64-bit address VALU per load and no store-time position mask
#ifndef EXTDM_X3_BUFX
#define EXTDM_X3_BUFX 1
#endif
// EXTDM_X3_EXP (diagnostic builds only, results invalid): bit 0 = the MFMAs replaced by one VALU
// per fragment pair (operand reads kept), bit 1 = no X global loads (zeros staged), bit 2 = the
// epilogue's output stores predicated off, bit 3 = no weight DMA
#ifndef EXTDM_X3_EXP
#define EXTDM_X3_EXP 0
#endif

namespace extdm {

__device__ int g_x3_range;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

struct X3Args {
  const float* in0; const float* in1;
  long i0b, i0c, i0t, i1b, i1c, i1t;
  int C0, Cin, H, W, T, P;
  const _Float16* w; const float* wscale; int ncgb;
  float* out; long ob, oc, ot; int Cout;
  int TH, NP, nrow_tiles, RS, XPOS;
  int out_bytes, res_bytes;  // extents of out / e.res (buffer descriptors of the epilogue)
  int stats_split;           // GroupNorm partial slots per (b, group) when e.stats is set
  // XOP: pre-split input operand (X3Op, kernels.h) copied by LDS-DMA instead of staged
  const _Float16* xop; long xop_cg, xop_hl;  // halves per channel group / per hi|lo half
  // split-K (SPL): fp32 partial accumulators [z][mtile][tile][TM*TN*16][NT], nsplit slices
  float* part; int nsplit;
  // PH: F's four edge lines [P][4 (top, bottom, left, right)][W][Cin] (fp32), written by the
  // m-tile-0 workgroups while staging (fea_x3.hip reads them); null: not written
  float* edge;
  int mfast;
  int in0_bytes, in1_bytes;  // BUFX: byte extents of the two sources (< 2^30), 0 = not usable
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

// One LDS-DMA piece (16 B per lane, wave-uniform LDS base) issued as inline asm, so that
// hipcc neither waits for it before the next ordinary global load nor drains it at the
// next use of one (it does both for __builtin_amdgcn_global_load_lds); the kernel
// retires it with its own counted vmcnt (cdna_hip_programming.md, LDS-DMA recipe).
__device__ __forceinline__ void glds16_asm(const void* gsrc, _Float16* lds) {
  const unsigned dst =
      __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(dst)
               : "memory");
}

// One buffer_load_dword ... lds: lane l's dword at byte offset voff of the resource lands at LDS
// byte lds + 4 l (an offset past the resource's extent loads 0); wave-uniform LDS base in M0.
// Asm like glds16_asm: hipcc neither waits for it nor counts it; the issuing wave's own vmcnt
// retires it.
__device__ __forceinline__ void bld4_asm(__amdgpu_buffer_rsrc_t rs, int voff, float* lds) {
  const unsigned dst =
      __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rs), "s"(dst)
               : "memory");
}

template <int KS, int BN> struct XMaxX3;
template <> struct XMaxX3<7, 256> { static constexpr int v = 560; };
template <> struct XMaxX3<3, 256> { static constexpr int v = 576; };
template <> struct XMaxX3<3, 128> { static constexpr int v = 288; };
template <> struct XMaxX3<1, 128> { static constexpr int v = 128; };
template <> struct XMaxX3<1, 256> { static constexpr int v = 256; };
template <> struct XMaxX3<7, 512> { static constexpr int v = 836; };
template <> struct XMaxX3<3, 512> { static constexpr int v = 800; };
template <> struct XMaxX3<5, 512> { static constexpr int v = 800; };
template <> struct XMaxX3<5, 256> { static constexpr int v = 400; };

// Stage barriers. SPAN = false: __syncthreads() per (channel block, ky) stage. While an
// A-slot LDS-DMA is in flight its fence waits vmcnt(0), which also drains the X prefetch
// loads issued in the same stage (65 % of the 1x1 / 52 % of the 3x3 wave cycles were
// parked there, profiles/r01_pmc_sq_convs_b64.json). SPAN = true: the X loads are issued
// with an exact count (16 per staging slot, unconditional clamped loads, the value masked
// by a multiply so hipcc cannot sink a load into a branch), after the stage's A DMA,
// and each stage ends with `s_waitcnt vmcnt(#X loads) lgkmcnt(0); s_barrier`: the DMA
// (older) is retired, the X loads (younger) stay in flight into the next stage.
// NS: staging slots per thread (ceil(XPOS * NG / threads), chosen at launch).
// KY: ky rows per A slot (stage). KY = KS makes a stage a whole channel block: one
// barrier per channel block instead of KS, and the X prefetch has all KS*KS*NG MFMA
// steps to land (the KS consecutive packed slices of a channel block are contiguous).
// XOP: the input is a pre-split operand (X3Op: hi / lo fp16 in (hl, c8) planes of
// zero-padded positions; written by groupnorm_silu_x3op): each channel block's halo tile
// is one contiguous run per plane, copied by LDS-DMA into the second X buffer during the
// block's first stage as [hl][c8][pos][8]: no staging registers, loads, conversions or
// LDS stores, and a lane's k-slice is 16 consecutive bytes (no swizzle needed).
// RGN: the residual is GroupNorm + SiLU-normalised in the epilogue (ConvEpi::res_aff; 1x1
// res_conv only — compiled out elsewhere: its live registers cost the 3x3 tiles their
// second wave per SIMD).
// SPL: split-K for launches with few workgroups (the small levels' long K loops were bound
// by the per-stage weight stream of too few CUs): 1 = slice blockIdx.z of the channel
// blocks, accumulators stored as fp32 partials; 2 = the partials summed in slice order
// (deterministic) and the normal epilogue.
// PH: phase output (the composed fea conv, conv_x3_phase_forward): m-tile = output phase
// (py, px) of a x2 upsampled map, row m - mtile * BM = output channel, tile pixel (row, col)
// stored at (2 row + py, 2 col + px) of the 2H x 2W output.
// WS: wave-specialised DMA queues. vmcnt counts one wave's memory operations in issue order,
// so with every wave issuing both the per-stage weight DMA and the channel block's X loads, the
// stage-end wait for the weight DMA also retired the X loads issued behind it: the X prefetch
// had one stage (~0.6 us) to cover an L2/HBM round trip (the X loads knocked out, the 5x5 phase
// conv ran 24 % faster, the level-0 3x3 31 %: EXTDM_X3_EXP builds). With WS the first half of
// the waves issues only the weight DMA and waits for it at each stage end; the second half
// issues only the X transfers (raw fp32 by buffer_load_dword ... lds into a [c][pos] tile, an
// out-of-image position past the extent so it loads 0; or the operand by LDS-DMA) for the next
// channel block at its first stage and waits for them at its last: STG stages of cover. The raw
// tile is split into the [hl][c8][pos][8] operand layout by all waves between channel blocks.
// BX: the buffer-load X staging (BUFX) known to apply at compile time (host: x3_bufx_ok). With the
// runtime choice both staging paths shared the channel-block loop, and merging them cost the loop
// register copies and 64-bit address arithmetic on the path taken (static count of the level-0
// 3x3 tile's loop: 1192 VALU + 521 SALU per 108 MFMAs; 249 + 218 with BX).
template <int KS, int KY, int BM, int BN, int NG, int WN, int NW, int XBUF, bool SPAN, int NS, bool XOP = false,
          bool RGN = false, int SPL = 0, bool PH = false, bool WS = false, bool BX = false>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW == 4 && KS == 5 ? 2 : 1))) void conv_x3_kernel(X3Args a) {
  constexpr int NT = NW * 64;
  constexpr int PAD = KS / 2;
  constexpr int CIB = 16 * NG;
  constexpr int MT32 = BM / 32;
  constexpr int STEPS = NG * KS;                // per A slot: (g, kx)
  constexpr int AH = STEPS * MT32 * 2 * 512;    // halves per ky slice
  constexpr int AHS = KY * AH;                  // halves per A slot (stage)
  constexpr int STG = KS / KY;                  // stages per channel block
  static_assert(KS % KY == 0, "KY must divide KS");
  constexpr int NSLOT = NS;
  constexpr int WM = NW / WN;
  constexpr int TM = BM / (32 * WM);
  constexpr int TN = BN / (32 * WN);
  static_assert(TM >= 1 && TN >= 1 && WM * WN == NW, "bad tile");
  static_assert(!XOP || (NG == 1 && XBUF == 2 && SPAN), "operand input: one group, two X buffers");

  extern __shared__ __attribute__((aligned(16))) _Float16 smx[];
  // halves from an X slot's hi block to its lo block (DMA mode: two c8 planes of whole
  // 1 KiB pieces each)
  static_assert(!WS || (NG == 1 && SPAN && SPL != 2 && NW % 2 == 0), "WS: one group, spanning barriers");
  constexpr bool WSR = WS && !XOP;  // WS with the raw fp32 tile
  constexpr bool LIN = WSR || ((EXTDM_X3_LIN == 1 || (EXTDM_X3_LIN == 2 && KS >= 5)) && NG == 1 && !XOP);
  // halves per (hl, c8) plane: DMA mode whole 1 KiB pieces; LIN one spare position past XPOS
  // (the target of unused staging slots)
  const int XPL = ((a.XPOS + (LIN ? 1 : 0) + 63) & ~63) * 8;
  const int XLO = (XOP || LIN) ? 2 * XPL : NG * a.XPOS * 16;
  const int XH = 2 * XLO;  // halves per X slot (hi + lo)
  constexpr int XB = WSR ? 1 : XBUF;  // WS raw: one split buffer, refilled between channel blocks
  const int RP = (a.XPOS + 63) & ~63;  // WS raw: positions per channel row of the raw tile
  _Float16* As0 = smx;
  _Float16* As1 = smx + AHS;
  _Float16* Xs0 = smx + 2 * AHS;
  _Float16* Xs1 = XB == 2 ? Xs0 + XH : Xs0;
  float* const Xr = reinterpret_cast<float*>(Xs0 + XB * XH);  // WS raw: [16 c][RP] fp32

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int h = lane >> 5, lc = lane & 31;
  // XCD-aware tile order for the k > 1 convs: workgroup w runs on XCD w mod 8 (the linear id
  // x + y X + z X Y has the residue of x when X % 8 == 0), so XCD k takes the contiguous tile
  // range [k X/8, (k+1) X/8) in dispatch order and the halo rows two row tiles of a plane
  // share are re-read from its L2, not HBM (round-robin put neighbouring tiles on different
  // XCDs). PMC at B = 64: 7x7 2326 -> 2062 MB, level-0 3x3 599 -> 546 MB per launch. The 1x1
  // tiles share nothing across tiles and ran 5 % slower remapped (HBM-bound: the round-robin
  // order spreads the 8 XCDs' concurrent reads over neighbouring addresses).
  // MFAST (1x1 with all m-tiles' weights within an XCD's L2, host: x3_mfast): the k-th
  // workgroup of XCD x takes m-tile k % MT of pixel tile x + 8 (k / MT), so a pixel tile's MT
  // m-tiles run back to back on one XCD and its input is read from HBM once (the default
  // order re-read it once per m-tile: the ups.3 Tmodulator 7 x 235 MB)
  int tile, mtile;
  if (KS == 1 && a.mfast) {
    const int lin = (int)(blockIdx.x + gridDim.x * blockIdx.y), MT = (int)gridDim.y;
    const int k = lin >> 3;
    mtile = k % MT;
    tile = (lin & 7) + 8 * (k / MT);
  } else {
    tile = (KS == 1 || (gridDim.x & 7)) ? (int)blockIdx.x
                                        : (int)((blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3));
    mtile = blockIdx.y;
  }
  const int plane0 = (tile / a.nrow_tiles) * a.NP;
  const int row0 = (tile % a.nrow_tiles) * a.TH;

  const int THK = a.TH + KS - 1;
  // first halo position of the tile in the operand's padded [P][H+KS-1][RS] planes
  const int tb = (plane0 * (a.H + KS - 1) + row0) * a.RS;
  const int c0 = SPL == 1 ? (int)blockIdx.z * a.ncgb / a.nsplit : 0;
  const int c1 = SPL == 1 ? ((int)blockIdx.z + 1) * a.ncgb / a.nsplit : a.ncgb;
  const int NIT = c1 * STG;
  const _Float16* wt = a.w + (long)mtile * a.ncgb * KS * AH;

  // ---- staging slots: (group, halo position), 16 channels each ----
  int sg[NSLOT], spos[NSLOT], soff0[NSLOT], soff1[NSLOT];
#pragma unroll
  for (int j = 0; j < NSLOT; ++j) {
    const int sl = tid + NT * j;
    sg[j] = -1; spos[j] = 0; soff0[j] = -1; soff1[j] = -1;
    if (sl < a.XPOS * NG) {
      const int g = sl / a.XPOS, pos = sl - g * a.XPOS;
      const int p = pos / (THK * a.RS);
      const int r2 = pos - p * THK * a.RS;
      const int rr = r2 / a.RS, cc = r2 - rr * a.RS;
      const int q = plane0 + p;
      const int iy = row0 + rr - PAD, ix = cc - PAD;
      sg[j] = g; spos[j] = pos;
      if (q < a.P && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) {
        const int b = q / a.T, t = q - b * a.T;
        soff0[j] = (int)((long)b * a.i0b + (long)t * a.i0t) + iy * a.W + ix;
        soff1[j] = (int)((long)b * a.i1b + (long)t * a.i1t) + iy * a.W + ix;
      }
    }
  }
  float xr[NSLOT][16];
  int range_bad = 0;

  // plain copies: selecting between fields of the by-value kernarg inside the lambdas
  // made hipcc spill the whole X3Args to scratch
  const float* const gin0 = a.in0;
  const float* const gin1 = a.in1;
  const long gi0c = a.i0c, gi1c = a.i1c;
  const int gC0 = a.C0, gCin = a.Cin;
  // channel groups never straddle the two sources nor run past Cin (wave-uniform)
  const bool whole = gC0 % 16 == 0 && gCin % CIB == 0;
  const bool bufx = BX || (EXTDM_X3_BUFX && whole && a.in0_bytes > 0);
  const auto rsx0 = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.in0), 0, a.in0_bytes, 0x00020000);
  const auto rsx1 = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.in1), 0, a.in1_bytes, 0x00020000);
  auto load_x_exact = [&](int cgb) __attribute__((always_inline)) {
#if EXTDM_X3_EXP & 2
#pragma unroll
    for (int j = 0; j < NSLOT; ++j)
#pragma unroll
      for (int c = 0; c < 16; ++c) xr[j][c] = 0.f;
    return;
#endif
    if (bufx) {
#pragma unroll
      for (int j = 0; j < NSLOT; ++j) {
        // the slot's channel group is wave-uniform (host: one group, or XPOS % 64 == 0)
        const int ci0 = __builtin_amdgcn_readfirstlane(cgb * CIB + (sg[j] < 0 ? 0 : sg[j]) * 16);
        const bool s1 = ci0 >= gC0;
        const int vo = soff0[j] >= 0 ? (s1 ? soff1[j] : soff0[j]) * 4 : 0x40000000;
        const int cb = s1 ? ci0 - gC0 : ci0;
        const int cs4 = (int)(s1 ? gi1c : gi0c) * 4;
#pragma unroll
        for (int c = 0; c < 16; ++c)
          xr[j][c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(s1 ? rsx1 : rsx0, vo, (cb + c) * cs4, 0));
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < NSLOT; ++j) {  // every slot loads (unused ones a masked dummy): 16 * NSLOT loads
      const bool pos_ok = soff0[j] >= 0;
      const int o0 = pos_ok ? soff0[j] : 0, o1 = pos_ok ? soff1[j] : 0;
      const int ci0 = cgb * CIB + (sg[j] < 0 ? 0 : sg[j]) * 16;
      // raw values only: any use of a load result here (even the mask) makes hipcc wait
      // vmcnt(0) while the stage's A DMA is in flight; store_x masks them
      if (whole) {
        const bool s1 = ci0 >= gC0;
        const float* bp = s1 ? gin1 + (long)(ci0 - gC0) * gi1c + o1 : gin0 + (long)ci0 * gi0c + o0;
        const long cs = s1 ? gi1c : gi0c;
#pragma unroll
        for (int c = 0; c < 16; ++c) xr[j][c] = bp[c * cs];
        continue;
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const int ci = ci0 + c;
        const bool s1 = ci >= gC0;
        int cc = s1 ? ci - gC0 : ci;
        const int cmax = s1 ? gCin - gC0 - 1 : gC0 - 1;
        cc = cc > cmax ? cmax : cc;
        const long off = s1 ? (long)cc * gi1c + o1 : (long)cc * gi0c + o0;
        xr[j][c] = (s1 ? gin1 : gin0)[off];
      }
    }
  };
  // store-time mask of an exact-count slot: halo position inside the image, channel < Cin
  auto xmask = [&](int j, int cgb, int c) __attribute__((always_inline)) {
    const int ci = cgb * CIB + (sg[j] < 0 ? 0 : sg[j]) * 16 + c;
    return (soff0[j] >= 0 && ci < gCin) ? 1.f : 0.f;
  };
  auto load_x = [&](int cgb) __attribute__((always_inline)) {
    if (SPAN) {
      load_x_exact(cgb);
      return;
    }
#pragma unroll
    for (int j = 0; j < NSLOT; ++j) {
      const int ci0 = cgb * CIB + sg[j] * 16;
      const bool src1 = ci0 >= a.C0;
      const float* base = src1 ? a.in1 + (long)(ci0 - a.C0) * a.i1c : a.in0 + (long)ci0 * a.i0c;
      const int cs = src1 ? (int)a.i1c : (int)a.i0c;
      const int off = src1 ? soff1[j] : soff0[j];
      const int cend = src1 ? a.Cin : a.C0;  // the group's source ends here
      if (off >= 0 && ci0 + 16 <= cend) {
#pragma unroll
        for (int c = 0; c < 16; ++c) xr[j][c] = base[off + c * cs];
      } else {
        // ragged group: the tail of a source (and the start of in1 when C0 % 16 != 0)
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const int ci = ci0 + c;
          float v = 0.f;
          if (soff0[j] >= 0 && ci < a.Cin)
            v = ci < a.C0 ? a.in0[(long)ci * a.i0c + soff0[j]] : a.in1[(long)(ci - a.C0) * a.i1c + soff1[j]];
          xr[j][c] = v;
        }
      }
    }
  };
  // 16-byte chunk h of position pos sits at chunk h ^ bit3(pos): conflict-free
  // ds_read_b128 for 32 consecutive positions (lane groups of 16, MI355X_MICROARCH §LDS)
  // An unused slot (SPAN) stores its zeros into a 64-byte dummy past the X buffers
  // instead of branching around the store: a lane-divergent skip leaves the X loads
  // pending on one path, and hipcc's path-insensitive wait analysis then drains vmcnt(0)
  // at the next channel block's X prefetch.
  _Float16* const xdummy = Xs0 + XB * XH + (WSR ? 2 * 16 * RP : 0);  // 32 halves, then the epilogue's scale/bias rows
  auto store_x = [&](_Float16* Xs, int cgb) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < NSLOT; ++j) {
      if (!SPAN && sg[j] < 0) continue;
      float v[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        float r = xr[j][c];
        if (SPAN) {
          // pinned here (volatile: not hoisted above the stage barriers of the 7x7
          // ky loop, where the first use of a load result would wait for the X loads)
          asm volatile("" : "+v"(r));
          if (!bufx) r *= xmask(j, cgb, c);  // bufx: outside positions already loaded as 0
        }
        v[c] = r;
      }
      unsigned hw[8], lw[8];
      float am = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        split2s(v[2 * c], v[2 * c + 1], hw[c], lw[c]);
        amax2(am, v[2 * c], v[2 * c + 1]);
      }
      range_bad |= am >= 65504.f;
      const h8 hi0 = __builtin_bit_cast(h8, u32x4{hw[0], hw[1], hw[2], hw[3]});
      const h8 hi1 = __builtin_bit_cast(h8, u32x4{hw[4], hw[5], hw[6], hw[7]});
      const h8 lo0 = __builtin_bit_cast(h8, u32x4{lw[0], lw[1], lw[2], lw[3]});
      const h8 lo1 = __builtin_bit_cast(h8, u32x4{lw[4], lw[5], lw[6], lw[7]});
      const bool used = sg[j] >= 0;
      if (LIN) {
        _Float16* d = Xs + (used ? spos[j] : XPL / 8 - 1) * 8;
        *reinterpret_cast<h8*>(d) = hi0;
        *reinterpret_cast<h8*>(d + XPL) = hi1;
        *reinterpret_cast<h8*>(d + 2 * XPL) = lo0;
        *reinterpret_cast<h8*>(d + 3 * XPL) = lo1;
        continue;
      }
      const int sw = (spos[j] >> 3) & 1;
      _Float16* dh = used ? Xs + ((long)sg[j] * a.XPOS + spos[j]) * 16 : xdummy;
      _Float16* dl = used ? dh + XLO : xdummy + 16;
      *reinterpret_cast<h8*>(dh + 8 * sw) = hi0;
      *reinterpret_cast<h8*>(dh + 8 * (sw ^ 1)) = hi1;
      *reinterpret_cast<h8*>(dl + 8 * sw) = lo0;
      *reinterpret_cast<h8*>(dl + 8 * (sw ^ 1)) = lo1;
    }
  };
  constexpr int NPIECE = AHS / 512;  // 1 KiB pieces
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  auto load_a = [&](int it, _Float16* As) {
#if EXTDM_X3_EXP & 8
    return;
#endif
    const _Float16* src = wt + (long)it * AHS;
    if (WS && wave_u >= NW / 2) return;  // WS: the weight waves only
    for (int pc = wave_u; pc < NPIECE; pc += (WS ? NW / 2 : NW)) {
      if (SPAN) glds16_asm(src + pc * 512 + lane * 8, As + pc * 512);
      else
        __builtin_amdgcn_global_load_lds((const void*)(src + pc * 512 + lane * 8), (lds_ptr_t)(As + pc * 512), 16, 0,
                                         0);
    }
  };

  // operand input: the channel block's tile, four (hl, c8) runs of XPOS 16-B records
  auto dma_x = [&](int cgb, _Float16* Xs) __attribute__((always_inline)) {
    const _Float16* src = a.xop + (long)cgb * a.xop_cg + (long)tb * 8;
    const int npc = (a.XPOS + 63) >> 6;  // 1 KiB pieces per plane
    if (WS && wave_u < NW / 2) return;  // WS: the X waves only
    for (int pc = WS ? wave_u - NW / 2 : wave_u; pc < 4 * npc; pc += (WS ? NW / 2 : NW)) {
      const int pl = pc / npc, k = pc - pl * npc;  // pl = 2 * hl + c8
      glds16_asm(src + (pl >> 1) * a.xop_hl + (pl & 1) * (a.xop_hl >> 1) + k * 512 + lane * 8,
                 Xs + pl * XPL + k * 512);
    }
  };

  // WS raw: the X waves' chunks of 64 positions of the tile (chunk k = xw + NW/2 i), each lane's
  // position offset in both sources (bytes; past the extent when outside the image)
  constexpr int NXW = NW / 2;
  constexpr int WCH = WSR ? (XMaxX3<KS, BN>::v + 64 * NXW - 1) / (64 * NXW) : 1;  // chunks per X wave
  int xo0[WCH], xo1[WCH];
  if (WSR) {
    const int xw = wave - NXW;
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int pos = (xw + NXW * i) * 64 + lane;
      xo0[i] = 0x40000000; xo1[i] = 0x40000000;
      if (xw >= 0 && pos < a.XPOS) {
        const int p = pos / (THK * a.RS), r2 = pos - p * THK * a.RS;
        const int rr = r2 / a.RS, cc = r2 - rr * a.RS;
        const int q = plane0 + p, iy = row0 + rr - PAD, ix = cc - PAD;
        if (q < a.P && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) {
          const int b = q / a.T, t = q - b * a.T;
          xo0[i] = (int)(((long)b * a.i0b + (long)t * a.i0t) + iy * a.W + ix) * 4;
          xo1[i] = (int)(((long)b * a.i1b + (long)t * a.i1t) + iy * a.W + ix) * 4;
        }
      }
    }
  }
  auto dma_raw = [&](int cgb) __attribute__((always_inline)) {
    if (!WSR || wave_u < NXW) return;
    const int xw = wave_u - NXW;
#pragma unroll 4
    for (int c = 0; c < 16; ++c) {
      const int ci = cgb * 16 + c;  // wave-uniform; host: channel blocks never straddle the sources
      const bool s1 = ci >= gC0;
      const int co = (int)((s1 ? ci - gC0 : ci) * (s1 ? gi1c : gi0c)) * 4;
#pragma unroll
      for (int i = 0; i < WCH; ++i) {
        const int k = xw + NXW * i;
        if (k * 64 < a.XPOS) bld4_asm(s1 ? rsx1 : rsx0, (s1 ? xo1[i] : xo0[i]) + co, Xr + c * RP + k * 64);
      }
    }
  };
  // raw [c][pos] fp32 -> the [hl][c8][pos][8] operand layout (every wave; range flag as store_x)
  auto split_raw = [&]() __attribute__((always_inline)) {
    for (int p = tid; p < a.XPOS; p += NT) {
      float v[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] = Xr[c * RP + p];
      unsigned hw[8], lw[8];
      float am = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        split2s(v[2 * c], v[2 * c + 1], hw[c], lw[c]);
        amax2(am, v[2 * c], v[2 * c + 1]);
      }
      range_bad |= am >= 65504.f;
      _Float16* d = Xs0 + p * 8;
      *reinterpret_cast<h8*>(d) = __builtin_bit_cast(h8, u32x4{hw[0], hw[1], hw[2], hw[3]});
      *reinterpret_cast<h8*>(d + XPL) = __builtin_bit_cast(h8, u32x4{hw[4], hw[5], hw[6], hw[7]});
      *reinterpret_cast<h8*>(d + 2 * XPL) = __builtin_bit_cast(h8, u32x4{lw[0], lw[1], lw[2], lw[3]});
      *reinterpret_cast<h8*>(d + 3 * XPL) = __builtin_bit_cast(h8, u32x4{lw[4], lw[5], lw[6], lw[7]});
    }
  };

  // ---- per-lane operand bases ----
  int bpos[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = (wn * TN + j) * 32 + lc;
    const int p = n / (a.TH * a.W);
    const int r = (n / a.W) % a.TH;
    const int c = n % a.W;
    bpos[j] = (p * THK + r) * a.RS + c;
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // per-row output scale and bias of this m-tile, staged for the epilogue
  float* const ep_sc = reinterpret_cast<float*>(xdummy + 32);
  float* const ep_bi = ep_sc + BM;
  if (tid < BM) {
    const int m = mtile * BM + tid;
    const int mc = m < a.Cout ? m : a.Cout - 1;
    ep_sc[tid] = a.wscale[mc];
    ep_bi[tid] = a.e.bias ? a.e.bias[mc] : 0.f;
  }
  if (SPL == 2) {
    // sum of the slices' partial accumulators, in slice order
    const long per = (long)TM * TN * 16 * NT;
    const float* pp = a.part + ((long)mtile * gridDim.x + tile) * per + tid;
    const long zs = (long)gridDim.y * gridDim.x * per;
    for (int z = 0; z < a.nsplit; ++z)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] += pp[z * zs + (long)((i * TN + j) * 16 + r) * NT];
    __syncthreads();  // ep_sc / ep_bi
  } else if (XOP) {
    dma_x(c0, Xs0);
    load_a(c0 * STG, As0);
  } else if (WSR) {
    dma_raw(c0);
    load_a(c0 * STG, As0);
  } else {
    load_x(c0);
    load_a(c0 * STG, As0);
    store_x(Xs0, c0);
  }
  if (SPL == 2) {
  } else if (SPAN) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");  // the asm DMA is invisible to __syncthreads
  else __syncthreads();
  if (WSR && SPL != 2) {
    split_raw();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // One (channel block, ky block) stage. `more` = a next channel block exists (its X is
  // prefetched at stage 0 and stored at stage STG - 1). The stages of a channel block are
  // issued as stage 0 peeled + the rest, and the last channel block is peeled with
  // more = false, so that hipcc sees the X prefetch and its store_x in one region with no
  // X load pending across a loop back edge (a path-insensitive pending load there made it
  // wait vmcnt(0) before re-loading the xr registers, right behind the stage's A DMA).
  // PH: F's edge lines from the staged tile of channel block cgb (m-tile 0 only): each edge
  // position's 16 channels as hi + lo' 2^-11 (exactly the operand the MFMAs use; the edge
  // kernels' own split of it gives back the same hi / lo'), into a.edge [P][4][W][Cin]. Issued
  // before the stage's A DMA, so the stage barrier's counted wait retires these stores too.
  auto export_edges = [&](const _Float16* Xs, int cgb) __attribute__((always_inline)) {
    const int nrec = a.NP * 4 * a.W;
    for (int r = tid; r < nrec; r += NT) {
      const int pp = r / (4 * a.W), rem = r - pp * 4 * a.W, line = rem / a.W, jj = rem - line * a.W;
      const int q = plane0 + pp;
      const int iy = line == 0 ? 0 : (line == 1 ? a.H - 1 : jj);
      const int ix = line == 2 ? 0 : (line == 3 ? a.W - 1 : jj);
      if (q >= a.P || iy < row0 || iy >= row0 + a.TH) continue;
      const int pos = (pp * THK + iy - row0 + PAD) * a.RS + ix + PAD;
      h8 h0, h1, l0, l1;
      if (LIN) {
        const _Float16* xh = Xs + (long)pos * 8;
        h0 = *reinterpret_cast<const h8*>(xh);
        h1 = *reinterpret_cast<const h8*>(xh + XPL);
        l0 = *reinterpret_cast<const h8*>(xh + 2 * XPL);
        l1 = *reinterpret_cast<const h8*>(xh + 3 * XPL);
      } else {
        const int sw = (pos >> 3) & 1;
        const _Float16* xh = Xs + (long)pos * 16;
        h0 = *reinterpret_cast<const h8*>(xh + 8 * sw);
        h1 = *reinterpret_cast<const h8*>(xh + 8 * (sw ^ 1));
        l0 = *reinterpret_cast<const h8*>(xh + XLO + 8 * sw);
        l1 = *reinterpret_cast<const h8*>(xh + XLO + 8 * (sw ^ 1));
      }
      float v[16];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        v[c] = (float)h0[c] + (float)l0[c] * (1.f / X3_LO_UP);
        v[8 + c] = (float)h1[c] + (float)l1[c] * (1.f / X3_LO_UP);
      }
      float4* d = reinterpret_cast<float4*>(a.edge + (((long)q * 4 + line) * a.W + jj) * a.Cin + cgb * CIB);
#pragma unroll
      for (int c = 0; c < 4; ++c) d[c] = make_float4(v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]);
    }
  };
  auto stage = [&](int cgb, int kb, bool more) __attribute__((always_inline)) {
    const int it = cgb * STG + kb;
    const int itr = it - c0 * STG, cr = cgb - c0;  // ring / buffer parity from the slice start
    const _Float16* Ast = (itr & 1) ? As1 : As0;
    const _Float16* Xs = (cr & 1) ? Xs1 : Xs0;  // WS raw: Xs1 == Xs0
    if (PH && !XOP && kb == 0 && a.edge && mtile == 0) export_edges(Xs, cgb);
    if (it + 1 < NIT) load_a(it + 1, (itr & 1) ? As0 : As1);
    const bool pre = (kb == 0) && more;
    if (SPAN) __builtin_amdgcn_sched_barrier(0);  // the X loads issue after the DMA (vmcnt order)
    if (pre) {
      if (XOP) dma_x(cgb + 1, (cr & 1) ? Xs0 : Xs1);
      else if (WSR) dma_raw(cgb + 1);
      else load_x(cgb + 1);
    }
#pragma unroll
    for (int kyl = 0; kyl < KY; ++kyl) {
    const int ky = kb * KY + kyl;
    const _Float16* As = Ast + kyl * AH;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        const int step = g * KS + kx;
        h8 ah[TM], al[TM], ad[TM], bh[TN], bl[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const _Float16* ap = As + ((step * MT32 + wm * TM + i) * 2) * 512 + lane * 8;
          ah[i] = *reinterpret_cast<const h8*>(ap);
          al[i] = *reinterpret_cast<const h8*>(ap + 512);
          ad[i] = lo_dn(ah[i]);  // pairs with the scaled activation lo (split2s, kernels.h)
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int pos = bpos[j] + ky * a.RS + kx;
          const _Float16* bp = (XOP || LIN) ? Xs + h * XPL + pos * 8
                                            : Xs + ((long)g * a.XPOS + pos) * 16 + 8 * (h ^ ((pos >> 3) & 1));
          bh[j] = *reinterpret_cast<const h8*>(bp);
          bl[j] = *reinterpret_cast<const h8*>(bp + XLO);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            // the scaled-lo product last: its lo_dn VALU is off the head of the chain (-3 %,
            // interleaved A/B at B = 64)
#if EXTDM_X3_EXP & 1
            acc[i][j][0] += (float)(al[i][0] * bh[j][0] + ah[i][1] * bh[j][1] + ad[i][2] * bl[j][2]);
#else
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ad[i], bl[j], acc[i][j], 0, 0, 0);
#endif
          }
      }
    }
    }
    if (WS) {
      // weight waves: this stage's DMA of the next stage's slot; X waves: the next channel
      // block's transfer at its last stage only (in flight across the other stage barriers)
      if (wave_u < NW / 2 || (kb == STG - 1 && more))
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (WSR && kb == STG - 1 && more) {
        split_raw();  // the split buffer's last reader (this stage) is past the barrier
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
      return;
    }
    if (!XOP && kb == STG - 1 && more) {
      if (XBUF == 1) {  // single X buffer: every wave is done with it
        if (SPAN) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else __syncthreads();
      }
      store_x((cr & 1) ? Xs0 : Xs1, cgb + 1);
    }
    if (SPAN) {
      // retire this stage's A DMA (issued before the X prefetch) and this wave's LDS
      // writes; the prefetch loads (16 per slot) may stay in flight across the barrier
      // (only at ky = 0: a later stage's DMA is younger than the X loads, and vmcnt
      // retires in issue order, so waiting for it is vmcnt(0))
      if (!XOP && pre && STG > 1) {
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(16 * NSLOT) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
    } else {
      __syncthreads();
    }
  };
  auto channel_block = [&](int cgb, bool more) __attribute__((always_inline)) {
    stage(cgb, 0, more);
    if (STG > 3) {
#pragma unroll 1
      for (int kb = 1; kb < STG; ++kb) stage(cgb, kb, more);
    } else {
#pragma unroll
      for (int kb = 1; kb < STG; ++kb) stage(cgb, kb, more);
    }
  };
  if (SPL != 2) {
    for (int cgb = c0; cgb + 1 < c1; ++cgb) channel_block(cgb, true);
    channel_block(c1 - 1, false);
  }
  if (range_bad) atomicOr(&g_x3_range, 1);
  if (SPL == 1) {
    const long per = (long)TM * TN * 16 * NT;
    float* pp = a.part + (((long)blockIdx.z * gridDim.y + mtile) * gridDim.x + tile) * per + tid;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) pp[(long)((i * TN + j) * 16 + r) * NT] = acc[i][j][r];
    return;
  }

  // ---- epilogue (C/D map: col = lane & 31, row = (r&3) + 8(r>>2) + 4h) ----
  // Every operand load of a row group is issued before its first use (clamped indices,
  // kernel-uniform branches only): per-element guarded loads made hipcc wait for each
  // one in turn, ~32 serial L2 round trips per wave at one workgroup per CU.
  const bool has_res = a.e.res != nullptr;
  const bool res_gn = RGN && has_res;
  const bool has_post = a.e.post_scale != nullptr, post_pc = a.e.post_per_channel != 0;
  const int act = a.e.act;
  // GroupNorm statistics of the stored values, per 8-row block (i, k) of the lane's rows
  // (r16 = 4k .. 4k + 3 on both halves h): fp32 within the lane, pairwise across lanes,
  // double across waves and into the (b, group) partial of this tile
  const bool do_stats = a.e.stats != nullptr;
  float* const red = reinterpret_cast<float*>(smx);  // [wave][TM * 4][2]; A / X staging is dead here
  const auto rs_out = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, a.out_bytes, 0x00020000);
  const auto rs_res = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.e.res), 0, a.res_bytes, 0x00020000);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int mrow[16];
    float scl[16], bia[16];
    float st_s[4] = {0.f, 0.f, 0.f, 0.f}, st_q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int ml = (wm * TM + i) * 32 + 8 * k + 4 * h;  // rows ml .. ml + 3 of the tile
      const float4 s4 = *reinterpret_cast<const float4*>(ep_sc + ml);
      const float4 b4 = *reinterpret_cast<const float4*>(ep_bi + ml);
      scl[4 * k] = s4.x; scl[4 * k + 1] = s4.y; scl[4 * k + 2] = s4.z; scl[4 * k + 3] = s4.w;
      bia[4 * k] = b4.x; bia[4 * k + 1] = b4.y; bia[4 * k + 2] = b4.z; bia[4 * k + 3] = b4.w;
    }
#pragma unroll
    for (int r16 = 0; r16 < 16; ++r16) {
      const int m = mtile * BM + (wm * TM + i) * 32 + (r16 & 3) + 8 * (r16 >> 2) + 4 * h;
      mrow[r16] = m < a.Cout ? m : a.Cout - 1;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = (wn * TN + j) * 32 + lc;
      const int p = n / (a.TH * a.W);
      const int r = (n / a.W) % a.TH;
      const int c = n % a.W;
      const int q0 = plane0 + p, row0q = row0 + r;
      const bool valid = q0 < a.P && row0q < a.H;
      const int q = valid ? q0 : 0, row = valid ? row0q : 0;
      const int b = q / a.T, t = q - b * a.T;
      // PH: the 64-row block's output phase (BM = 64: the m-tile; BM = 128: two phases of one
      // output row parity, one per wave row)
      const int ph = (mtile * BM + (wm * TM + i) * 32) / 64;
      const int pix = PH ? (2 * row + (ph >> 1)) * (2 * a.W) + 2 * c + (ph & 1) : row * a.W + c;
      float v[16];
#pragma unroll
      for (int r16 = 0; r16 < 16; ++r16) v[r16] = acc[i][j][r16] * scl[r16] + bia[r16];
      if (has_res) {
        const int rbase = (int)((long)b * a.e.res_sb + (long)t * a.e.res_st) + pix;
        float rv[16];
#pragma unroll
        for (int r16 = 0; r16 < 16; ++r16)
          rv[r16] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
              rs_res, (rbase + (PH ? mrow[r16] - ph * 64 : mrow[r16]) * (int)a.e.res_sc) * 4, 0, 0));
        if (res_gn) {  // the arithmetic of gn_apply_plane_kernel (norm.hip), no FiLM
#pragma unroll
          for (int r16 = 0; r16 < 16; ++r16) {
            const float2 ab = a.e.res_aff[b * a.Cout + mrow[r16]];
            const float w = rv[r16] * ab.x + ab.y;
            rv[r16] = w / (1.f + expf(-w));
          }
        }
#pragma unroll
        for (int r16 = 0; r16 < 16; ++r16) v[r16] += rv[r16];
      }
      if (has_post) {
        float ps[16], pt[16];
#pragma unroll
        for (int r16 = 0; r16 < 16; ++r16) {
          const int pi = post_pc ? mrow[r16] : b * a.Cout + mrow[r16];
          ps[r16] = a.e.post_scale[pi];
          pt[r16] = a.e.post_shift[pi];
        }
#pragma unroll
        for (int r16 = 0; r16 < 16; ++r16) v[r16] = v[r16] * ps[r16] + pt[r16];
      }
      if (act != ACT_NONE) {
#pragma unroll
        for (int r16 = 0; r16 < 16; ++r16) v[r16] = act_apply(v[r16], act);
      }
      // 32-bit byte offsets into a bounded descriptor; a lane outside the image or a row
      // past Cout stores to an offset past the extent, which the range check drops
      const int obase = (int)((long)b * a.ob + (long)t * a.ot) + pix;
#pragma unroll
      for (int r16 = 0; r16 < 16; ++r16) {
        const int m = mtile * BM + (wm * TM + i) * 32 + (r16 & 3) + 8 * (r16 >> 2) + 4 * h;
        const bool ok = valid && m < a.Cout;
        const int off = ok ? (obase + (PH ? m - ph * 64 : m) * (int)a.oc) * 4 : a.out_bytes;
#if EXTDM_X3_EXP & 4
        if (v[r16] == 12345.678f)
#endif
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[r16]), rs_out, off, 0, 0);
        if (do_stats) {
          const float x = ok ? v[r16] : 0.f;
          st_s[r16 >> 2] += x;
          st_q[r16 >> 2] += x * x;
        }
      }
    }
    if (do_stats) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float s_ = st_s[k], q_ = st_q[k];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
          s_ += __shfl_xor(s_, off);
          q_ += __shfl_xor(q_, off);
        }
        if (lane == 0) {
          red[(wave * TM * 4 + i * 4 + k) * 2] = s_;
          red[(wave * TM * 4 + i * 4 + k) * 2 + 1] = q_;
        }
      }
    }
  }
  if (do_stats) {
    __syncthreads();
    const int G = a.e.stats_groups, Cg = a.Cout / G;
    const int ngrp = BM / Cg;  // groups of this m-tile (host: Cg % 8 == 0, BM % Cg == 0)
    if (tid < ngrp) {
      const int g = mtile * ngrp + tid;
      if (g < G) {
        double s_ = 0.0, q_ = 0.0;
        for (int kb = tid * (Cg / 8); kb < (tid + 1) * (Cg / 8); ++kb) {  // 8-row blocks of the group
          const int wmk = kb / (TM * 4), ik = kb % (TM * 4);
          for (int wn_ = 0; wn_ < WN; ++wn_) {
            const int w_ = wmk * WN + wn_;
            s_ += (double)red[(w_ * TM * 4 + ik) * 2];
            q_ += (double)red[(w_ * TM * 4 + ik) * 2 + 1];
          }
        }
        const int bq = plane0 / a.T;  // the tile's sample (host: T % NP == 0)
        const int slot = ((plane0 % a.T) / a.NP) * a.nrow_tiles + tile % a.nrow_tiles;
        double* pp = a.e.stats + (((long)bq * G + g) * a.stats_split + slot) * 2;
        pp[0] = s_;
        pp[1] = q_;
      }
    }
  }
}

// the BX precondition: the kernel's bufx test (whole 16-channel groups in each source, extents set)
bool x3_bufx_ok(const X3Args& a, int cib) {
  static const bool off = [] { const char* v = getenv("EXTDM_X3_NO_BX"); return v && v[0] && v[0] != '0'; }();
  return !off && EXTDM_X3_BUFX && a.C0 % 16 == 0 && a.Cin % cib == 0 && a.in0_bytes > 0;
}

template <int KS, int KY, int BM, int BN, int NG, int WN, int NW, int XBUF, bool SPAN, int NS, bool XOP = false,
          bool RGN = false, int SPL = 0, bool PH = false, bool WS = false>
void launch_sp(hipStream_t s, const X3Args& a, unsigned ntiles) {
  constexpr int AH = KY * NG * KS * (BM / 32) * 2 * 512;
  constexpr bool WSR = WS && !XOP;
  constexpr bool LIN = WSR || ((EXTDM_X3_LIN == 1 || (EXTDM_X3_LIN == 2 && KS >= 5)) && NG == 1 && !XOP);
  const size_t xlo = XOP ? (size_t)((a.XPOS + 63) & ~63) * 16
                         : (LIN ? (size_t)((a.XPOS + 1 + 63) & ~63) * 16 : (size_t)a.XPOS * NG * 16);
  constexpr int XB = WSR ? 1 : XBUF;
  const size_t raw = WSR ? (size_t)2 * 16 * ((a.XPOS + 63) & ~63) : 0;  // halves of the [16][RP] fp32 tile
  // + 32 halves (unused-slot dummy) + 2 * BM floats (epilogue scale / bias)
  const size_t lds = ((size_t)2 * AH + (size_t)XB * 2 * xlo + raw + 32 + 4 * BM) * sizeof(_Float16);
  dim3 grid(ntiles, (a.Cout + BM - 1) / BM, SPL == 1 ? a.nsplit : 1);
  // BX only where the staging loads run (not the operand-input / WS-raw / split-K-sum tiles)
  constexpr bool BXV = !XOP && !WSR && SPL != 2 && SPAN;
  const bool bx = BXV && x3_bufx_ok(a, 16 * NG);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_x3_kernel<KS, KY, BM, BN, NG, WN, NW, XBUF, SPAN, NS, XOP, RGN, SPL, PH, WS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (BXV)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_x3_kernel<KS, KY, BM, BN, NG, WN, NW, XBUF, SPAN, NS, XOP, RGN, SPL, PH, WS, BXV>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  if (SPL != 2) {
    auto tf = [](bool v) { return v ? "true" : "false"; };
    note_kernel("conv_x3_kernel<%d, %d, %d, %d, %d, %d, %d, %d, %s, %d, %s, %s, %d, %s, %s, %s>", KS, KY, BM, BN, NG, WN,
                NW, XBUF, tf(SPAN), NS, tf(XOP), tf(RGN), SPL, tf(PH), tf(WS), tf(bx));
  }
  if (bx)
    hipLaunchKernelGGL((conv_x3_kernel<KS, KY, BM, BN, NG, WN, NW, XBUF, SPAN, NS, XOP, RGN, SPL, PH, WS, BXV>), grid, dim3(NW * 64), lds, s, a);
  else
    hipLaunchKernelGGL((conv_x3_kernel<KS, KY, BM, BN, NG, WN, NW, XBUF, SPAN, NS, XOP, RGN, SPL, PH, WS>), grid, dim3(NW * 64), lds, s, a);
}

template <int KS, int KY, int BM, int BN, int NG, int WN, int NW, int XBUF, bool SPAN>
void launch_ns(hipStream_t s, const X3Args& a, unsigned ntiles) {
  constexpr int XMAX = XMaxX3<KS, BN>::v;
  constexpr int NT = NW * 64;
  static_assert((XMAX * NG + NT - 1) / NT <= 3, "more than three staging slots");
  const int need = (a.XPOS * NG + NT - 1) / NT;
  if constexpr (XMAX * NG <= NT) launch_sp<KS, KY, BM, BN, NG, WN, NW, XBUF, SPAN, 1>(s, a, ntiles);
  else if constexpr (XMAX * NG <= 2 * NT) {
    if (need <= 1) launch_sp<KS, KY, BM, BN, NG, WN, NW, XBUF, SPAN, 1>(s, a, ntiles);
    else launch_sp<KS, KY, BM, BN, NG, WN, NW, XBUF, SPAN, 2>(s, a, ntiles);
  } else {
    if (need <= 1) launch_sp<KS, KY, BM, BN, NG, WN, NW, XBUF, SPAN, 1>(s, a, ntiles);
    else if (need == 2) launch_sp<KS, KY, BM, BN, NG, WN, NW, XBUF, SPAN, 2>(s, a, ntiles);
    else launch_sp<KS, KY, BM, BN, NG, WN, NW, XBUF, SPAN, 3>(s, a, ntiles);
  }
}

// Split-K for launches that leave CUs idle: the 3x3 128-row tile runs one workgroup per CU
// (84 KB of LDS), so it splits only below 128 workgroups and up to 256 in total (a second
// round of workgroups cost more than the shorter K loops saved: 70 -> 80 us at 256 x 2);
// the 1x1 128-row tile (several workgroups per CU) splits below 384, up to 512. Slices keep
// >= 2 channel blocks. The slice count is a function of the per-sample geometry only (the
// workgroup count at the reference batch 64), never of the batch: a clip's result must
// not depend on the shard it lands in (every output element sums the same slices in the same
// order whichever tile, and whichever tile-mates, it has). EXTDM_NO_SPLITK=1 turns it off (A/B).
// Long-K 256-row 1x1 convs (>= 128 channel blocks, K >= 4096: KTH's 7680 -> 5120 Tmodulators,
// 40 workgroups at its 16 clips per GPU): the slice count minimises a cost model at a reference
// batch of 16 clips (KTH's 64 on 4 GPUs) — ceil(S x workgroups / 256) rounds of ncgb / S channel
// blocks (1.74 us each on the 256 x 128 tile) plus S partial planes written and summed back (1.5 TB/s
// effective), both measured on KTH's level-2 Tmodulator (417 us unsplit, 364 us at S = 3) — a
// function of the per-sample geometry only, like the rule above. x3_bn256 keeps these convs
// on the 256 x 128 tile, so the split never depends on the launch's batch.
// EXTDM_X3_LONGK=0 turns it off (A/B).
constexpr int kLongKBlocks = 128;
int split_slices_longk(const X3Args& a) {
  static const bool on = [] { const char* v = getenv("EXTDM_X3_LONGK"); return !(v && v[0] == '0'); }();
  if (!on || a.ncgb < kLongKBlocks || a.P < 1) return 0;
  const long nwg16 = (16L * a.T + a.NP - 1) / a.NP * a.nrow_tiles * ((a.Cout + 255) / 256);
  const double blk_us = 1.74;
  const double part_us = (double)a.Cout * (16.0 * a.T * a.H * a.W) * 8.0 / 1.5e6;
  int best = 1;
  double bc = 1e300;
  for (int S = 1; S <= a.ncgb / 16; ++S) {
    const double c = (double)((nwg16 * S + 255) / 256) * ((a.ncgb + S - 1) / S) * blk_us + (S > 1 ? S * part_us : 0.0);
    if (c < bc * 0.999) { bc = c; best = S; }
  }
  return best >= 2 ? best : 0;
}

int split_slices(const X3Args& a, unsigned ntiles, long max_wg, long max_total, int bm = 128) {
  static const bool off = [] { const char* v = getenv("EXTDM_NO_SPLITK"); return v && v[0] && v[0] != '0'; }();
  (void)ntiles;
  if (off || a.ncgb < 4 || a.P < 1) return 0;
  if (bm == 256 && a.ncgb >= kLongKBlocks) return split_slices_longk(a);
  // workgroups of this conv at the reference batch 64 (a function of the per-sample geometry:
  // T frames per sample, NP planes and nrow_tiles row tiles per tile; single-frame views such as
  // the Tmodulator's '(T C)' GEMM put several samples in one tile, which is still batch-independent)
  const long nwg64 = (64L * a.T + a.NP - 1) / a.NP * a.nrow_tiles * ((a.Cout + bm - 1) / bm);
  if (nwg64 >= max_wg) return 0;
  const int S = (int)std::min<long>(a.ncgb / 2, max_total / nwg64);
  return S >= 2 ? S : 0;
}
size_t split_bytes(const X3Args& a, unsigned ntiles, int S) {
  return S ? (size_t)S * ntiles * ((a.Cout + 127) / 128) * 128 * 128 * sizeof(float) : 0;
}
// The 256-row 1x1 tile (one workgroup per CU) splits below 256 workgroups, into at most 256:
// the level-3 / mid Tmodulators ('(T C)' = 3584 input channels, 112 workgroups at B = 64).
// EXTDM_X3_SPLIT256=0 turns it off (A/B).
bool x3_split256() {
  static const bool on = [] { const char* v = getenv("EXTDM_X3_SPLIT256"); return !(v && v[0] == '0'); }();
  return on;
}
bool split_k(X3Args& a, unsigned ntiles, const ConvEpi& e, long max_wg, long max_total, int bm = 128) {
  const int S = split_slices(a, ntiles, max_wg, max_total, bm);
  if (!S || !e.split_ws || split_bytes(a, ntiles, S) > e.split_ws_bytes) return false;
  a.part = e.split_ws;
  a.nsplit = S;
  return true;
}

// EXTDM_X3_WS=<mask>: the wave-specialised staging (kernel note WS) per tile family --
// 1 the 5x5 phase conv, 2 the staged 64-row 3x3 tile, 4 the operand-input 64-row 3x3 tile,
// 8 the operand-input 128-row 3x3 tiles (unsplit)
enum { kWsPhase = 1, kWsStaged64 = 2, kWsOp64 = 4, kWsOp128 = 8 };
bool x3_ws(int fam) {
  static const int mask = [] { const char* v = getenv("EXTDM_X3_WS"); return v ? atoi(v) : 0; }();
  return (mask & fam) != 0;
}
// the raw path's preconditions: whole 16-channel blocks in each source, byte extents < 2^30
bool x3_ws_raw_ok(const X3Args& a, int fam) {
  return x3_ws(fam) && a.C0 % 16 == 0 && a.Cin % 16 == 0 && a.in0_bytes > 0;
}

int x3_v3() {
  static const int v3 = [] { const char* v = getenv("EXTDM_X3_V3"); return v ? atoi(v) : 0; }();
  return v3;
}

// 3x3 128 x 128 tile on 4 waves of 64 x 64 (12 MFMAs per 8 ds_read_b128, two workgroups per
// CU) when its LDS fits half a CU; else 8 waves of 32 x 64 at one workgroup per CU.
// EXTDM_X3_W128=8 keeps the 8-wave tile everywhere (A/B).
bool x3_w128_4(const X3Args& a, bool xop) {
  static const int w = [] { const char* v = getenv("EXTDM_X3_W128"); return v ? atoi(v) : 4; }();
  if (w == 8) return false;
  constexpr size_t AH = 3 * 4 * 2 * 512;
  const size_t xlo = xop ? (size_t)((a.XPOS + 63) & ~63) * 16
                         : (EXTDM_X3_LIN == 1 ? (size_t)((a.XPOS + 1 + 63) & ~63) * 16 : (size_t)a.XPOS * 16);
  return (2 * AH + 2 * 2 * xlo + 32 + 4 * 128) * sizeof(_Float16) <= 80 * 1024;
}
// split-K thresholds of the 3x3 128-row tile (launch_wg, total_wg): 8 waves at one workgroup
// per CU split below 128 workgroups, up to 256; the 4-wave tile (two per CU) below
// EXTDM_X3_SPLIT4 = "wg,total" (default 256,512)
void x3_split128(bool four, long& max_wg, long& max_total) {
  static const long* t4 = [] {
    static long v[2] = {256, 512};
    if (const char* e = getenv("EXTDM_X3_SPLIT4")) sscanf(e, "%ld,%ld", &v[0], &v[1]);
    return v;
  }();
  if (four) { max_wg = t4[0]; max_total = t4[1]; } else { max_wg = 128; max_total = 256; }
}

template <int KS, int KY, int BM, int BN, int NG, int WN, int NW, int XBUF>
void launch(hipStream_t s, const X3Args& a, unsigned ntiles) {
  // EXTDM_X3_NOSPAN=1: per-stage __syncthreads() (A/B against the spanning barriers)
  static const bool nospan = [] { const char* v = getenv("EXTDM_X3_NOSPAN"); return v && v[0] && v[0] != '0'; }();
  if (nospan) launch_ns<KS, KY, BM, BN, NG, WN, NW, XBUF, false>(s, a, ntiles);
  else launch_ns<KS, KY, BM, BN, NG, WN, NW, XBUF, true>(s, a, ntiles);
}

}  // namespace

X3Tile x3_tile(int ks, int cout) {
  X3Tile t{};
  // 7x7 (init_conv): 8 waves over 64 x 512 px tiles, one X buffer; 3x3: 8 waves
  if (ks == 7) {
    // EXTDM_X3_BN7=256: the 8-wave 64 x 256 tile (two X buffers) instead of 64 x 512
    static const int bn7 = [] { const char* v = getenv("EXTDM_X3_BN7"); return v ? atoi(v) : 512; }();
    t.bm = 64; t.bn = bn7 == 256 ? 256 : 512; t.ng = 1;
  }
  else if (ks == 5) {
    // the phase-composed fea conv (conv_x3_phase_forward): 128-row m-tiles holding both column
    // phases of one output row parity over 256 px, so each output line is written by one
    // workgroup and F is staged twice instead of four times (2172 -> 2026 us at B = 64, whole
    // step -0.45 %); EXTDM_FEA_BM=64: one 64-row m-tile per phase over 512 px
    static const int bm5 = [] { const char* v = getenv("EXTDM_FEA_BM"); return v ? atoi(v) : 128; }();
    if (bm5 == 128) { t.bm = 128; t.bn = 256; } else { t.bm = 64; t.bn = 512; }
    t.ng = 1;
  }
  else if (ks == 3) {
    // EXTDM_X3_BN3: pixel tile of the Cout <= 64 3x3 convs (256 or 512)
    static const int bn3 = [] { const char* v = getenv("EXTDM_X3_BN3"); return v ? atoi(v) : 256; }();
    if (cout <= 64) { t.bm = 64; t.bn = bn3 == 512 ? 512 : 256; } else { t.bm = 128; t.bn = 128; }
    t.ng = 1;
  }
  else if (ks == 1) {
    // Cout a multiple of 256: one 256-row m-tile (8 waves), so each pixel tile's input is
    // staged once instead of once per 128 rows. EXTDM_X3_BM1=128 restores 128-row tiles.
    static const int bm1 = [] { const char* v = getenv("EXTDM_X3_BM1"); return v ? atoi(v) : 256; }();
    t.bm = cout <= 64 ? 64 : ((bm1 == 256 && cout % 256 == 0) ? 256 : 128);
    // (the 256-row convs may run on 256 x 256 tiles instead: x3_bn256, chosen per launch)
    t.bn = 128; t.ng = 2;
  }
  return t;
}

namespace {

// Tile geometry, operands and epilogue of one conv_x3 launch; false if not covered.
bool x3_setup(const View& out, const View& in0, const View* in1, const PackedW& w, const ConvEpi& epi, X3Args& a,
              unsigned& ntiles, int* stats_slots) {
  if (stats_slots) *stats_slots = 0;
  if (!w.wx || w.mode != MODE_CONV) return false;
  const int ks = w.KH;
  const int H = in0.H, W = in0.W;
  const X3Tile tl{w.xbm, w.xbn, w.xng};
  if (out.H != H || out.W != W || W > tl.bn || tl.bn % W != 0) return false;
  // 32-bit in-plane offsets in the staging
  if ((long)in0.B * in0.sb > (1L << 31) || (in1 && (long)in1->B * in1->sb > (1L << 31))) return false;
  a = X3Args{};
  a.TH = std::min(H, tl.bn / W);
  if (tl.bn % (a.TH * W) != 0) return false;
  a.NP = tl.bn / (a.TH * W);
  a.RS = W + ks - 1;
  a.XPOS = a.NP * (a.TH + ks - 1) * a.RS;
  const int xmax = tl.bn == 512 ? (ks == 7 ? 836 : 800)
                                 : (ks == 7 ? 560 : (ks == 5 ? 400 : (ks == 3 ? (tl.bn == 256 ? 576 : 288) : (tl.bn == 256 ? 256 : 128))));
  if (a.XPOS > xmax) return false;
  a.in0 = in0.p; a.i0b = in0.sb; a.i0c = in0.sc; a.i0t = in0.st; a.C0 = in0.C;
  if (in1) { a.in1 = in1->p; a.i1b = in1->sb; a.i1c = in1->sc; a.i1t = in1->st; a.Cin = in0.C + in1->C; }
  else { a.in1 = in0.p; a.i1b = in0.sb; a.i1c = in0.sc; a.i1t = in0.st; a.Cin = in0.C; }
  a.H = H; a.W = W; a.T = out.T; a.P = out.B * out.T;
  a.w = reinterpret_cast<const _Float16*>(w.wx); a.wscale = w.xscale; a.ncgb = w.xncgb;
  a.out = out.p; a.ob = out.sb; a.oc = out.sc; a.ot = out.st; a.Cout = out.C;
  a.nrow_tiles = (H + a.TH - 1) / a.TH;
  a.e = epi;
  // the epilogue addresses out / res with 32-bit byte offsets (buffer descriptors)
  auto extent = [&](long sb, long sc, long st, int C) {
    return ((long)(out.B - 1) * sb + (long)(C - 1) * sc + (long)(out.T - 1) * st + (long)H * W) * 4;
  };
  const long ob = extent(out.sb, out.sc, out.st, out.C);
  const long rb = epi.res ? extent(epi.res_sb, epi.res_sc, epi.res_st, out.C) : 0;
  if (ob >= (1L << 31) - 4 || rb >= (1L << 31) - 4) return false;
  a.out_bytes = (int)ob;
  a.res_bytes = (int)rb;
  ntiles = (unsigned)(((a.P + a.NP - 1) / a.NP) * a.nrow_tiles);
  // BUFX: both sources' byte extents below 2^30 (the out-of-image offset 2^30 then reads 0)
  // and the staging slots' channel group wave-uniform
  {
    auto ext_in = [&](const View& v) {
      return ((long)(v.B - 1) * v.sb + (long)(v.C - 1) * v.sc + (long)(v.T - 1) * v.st + (long)v.H * v.W) * 4;
    };
    const long e0 = ext_in(in0), e1 = in1 ? ext_in(*in1) : e0;
    const bool ok = e0 < (1L << 30) && e1 < (1L << 30) && (tl.ng == 1 || a.XPOS % 64 == 0);
    a.in0_bytes = ok ? (int)e0 : 0;
    a.in1_bytes = ok ? (int)e1 : 0;
  }
  // GroupNorm partials in the epilogue: whole tiles inside one sample, groups of whole
  // 8-row blocks inside one m-tile, at most 64 slots (the runtime's partials buffer)
  if (epi.stats) {
    const int G = epi.stats_groups, Cg = G > 0 ? out.C / G : 0;
    const int split = (out.T / std::max(a.NP, 1)) * a.nrow_tiles;
    const bool ok = G > 0 && out.C % G == 0 && Cg % 8 == 0 && tl.bm % Cg == 0 && out.T % a.NP == 0 &&
                    split >= 1 && split <= 64;
    if (ok) {
      a.stats_split = split;
      if (stats_slots) *stats_slots = split;
    } else {
      a.e.stats = nullptr;
    }
  }
  return true;
}

}  // namespace

// 1x1: the m-tile-fast XCD order (kernel note MFAST) when the whole weight (every m-tile, hi +
// lo) fits comfortably in one XCD's 4 MiB L2 and there is more than one m-tile.
// EXTDM_X3_NO_MFAST=1 turns it off (A/B).
bool x3_mfast(const X3Args& a, const X3Tile& tl, unsigned ntiles) {
  static const bool off = [] { const char* v = getenv("EXTDM_X3_NO_MFAST"); return v && v[0] && v[0] != '0'; }();
  static const long cap = [] { const char* v = getenv("EXTDM_X3_MFAST_KB"); return (v ? atol(v) : 3584L) * 1024; }();
  const long mt = (a.Cout + tl.bm - 1) / tl.bm;
  return !off && mt > 1 && ntiles % 8 == 0 && mt * tl.bm * (long)a.Cin * 4 <= cap;
}

// 1x1 256-row convs on 256 x 256 tiles (twice the MFMAs per staged weight fragment) when that
// tiling still fills >= 3/4 of the CUs in one round at this launch's batch (round 6; it was the
// reference batch 64, which left KTH's 16-clip Tmodulator 7680 -> 5120 on 80 workgroups). Both
// tilings sum K in the same order, so the choice may depend on the batch: a clip's result is
// bitwise the same either way (tests/test_gpu_parity.py batch-slice test). The level-2 Tmodulator
// 460 -> 353 us at B = 64; the level-3 / mid ones (56 workgroups at 256 px) keep 256 x 128 + split-K.
// EXTDM_X3_BN1=128 keeps 256 x 128 everywhere, EXTDM_X3_BN1=64 restores the batch-64 rule (A/B).
bool x3_bn256(const View& out, const PackedW& w, const ConvEpi& epi) {
  static const int bn1 = [] { const char* v = getenv("EXTDM_X3_BN1"); return v ? atoi(v) : 256; }();
  if ((bn1 != 256 && bn1 != 64) || w.KH != 1 || w.xbm != 256 || w.xbn != 128 || epi.res_aff) return false;
  // long-K convs stay on the 256 x 128 tile and its batch-independent split-K (split_slices_longk)
  static const bool longk = [] { const char* v = getenv("EXTDM_X3_LONGK"); return !(v && v[0] == '0'); }();
  if (longk && w.xncgb >= kLongKBlocks) return false;
  const int H = out.H, W = out.W;
  if (W > 256 || 256 % W != 0) return false;
  const int TH = std::min(H, 256 / W);
  if (256 % (TH * W) != 0) return false;
  const long NP = 256 / (TH * W), nrow = (H + TH - 1) / TH;
  const long Bref = bn1 == 64 ? 64L : (long)out.B;
  const long nwg = (Bref * out.T + NP - 1) / NP * nrow * ((out.C + 255) / 256);
  return nwg >= 192;
}

bool conv_x3_forward(hipStream_t s, const View& out, const View& in0, const View* in1, const PackedW& w0,
                     const ConvEpi& epi, int* stats_slots) {
  PackedW wt = w0;
  if (x3_bn256(out, w0, epi)) wt.xbn = 256;
  const PackedW& w = wt;
  X3Args a;
  unsigned ntiles = 0;
  if (!x3_setup(out, in0, in1, w, epi, a, ntiles, stats_slots)) return false;
  const int ks = w.KH;
  const X3Tile tl{w.xbm, w.xbn, w.xng};
  if (ks == 1) a.mfast = x3_mfast(a, tl, ntiles);
  if (epi.res_aff) {  // residual GroupNorm: the 1x1 tiles only
    if (ks != 1 || !epi.res || tl.bn != 128) return false;
    if (tl.bm == 64) launch_sp<1, 1, 64, 128, 2, 4, 4, 2, true, 1, false, true>(s, a, ntiles);
    else if (tl.bm == 128) launch_sp<1, 1, 128, 128, 2, 2, 4, 2, true, 1, false, true>(s, a, ntiles);
    else if (tl.bm == 256) launch_sp<1, 1, 256, 128, 2, 2, 8, 2, true, 1, false, true>(s, a, ntiles);
    else return false;
    return true;
  }
  if (tl.bn == 512) {
    // 7x7 64 x 512 tile: 8 waves of 64 x 64 (two per SIMD, 256 registers, no scratch):
    // 4.02 -> 3.80 ms at B = 64 against 16 waves of 32 x 64 (128 registers, 132-148 B of
    // scratch per lane); EXTDM_X3_NW7=16 restores the 16-wave tile (A/B)
    static const int nw7 = [] { const char* v = getenv("EXTDM_X3_NW7"); return v ? atoi(v) : 8; }();
    if (ks == 7 && tl.bm == 64 && nw7 != 16) launch<7, 1, 64, 512, 1, 8, 8, 1>(s, a, ntiles);
    else if (ks == 7 && tl.bm == 64) launch<7, 1, 64, 512, 1, 8, 16, 1>(s, a, ntiles);
    else if (ks == 3 && tl.bm == 64) launch<3, 1, 64, 512, 1, 8, 16, 1>(s, a, ntiles);
    else return false;
    return true;
  }
  if (ks == 7 && tl.bm == 64) launch<7, 1, 64, 256, 1, 4, 8, 2>(s, a, ntiles);
  else if (ks == 3 && tl.bm == 64) {
    // EXTDM_X3_V3=1: the 8-wave tile (32 x 64 per wave, whole-channel-block stages, one
    // workgroup per CU at 117 KB of LDS). Default: 4 waves of 64 x 64 (12 MFMAs per 8
    // ds_read_b128 instead of 6 per 6) at 68 KB, two independent workgroups per CU,
    // 12 % faster on the level-0 64 -> 64 conv at B = 64.
    if (x3_v3() == 1) launch<3, 3, 64, 256, 1, 4, 8, 2>(s, a, ntiles);
    else if (x3_ws_raw_ok(a, kWsStaged64)) launch_sp<3, 1, 64, 256, 1, 4, 4, 2, true, 1, false, false, 0, false, true>(s, a, ntiles);
    else launch<3, 1, 64, 256, 1, 4, 4, 2>(s, a, ntiles);
  }
  else if (ks == 3 && tl.bm == 128) {
    const bool four = x3_w128_4(a, false);
    long mw, mt;
    x3_split128(four, mw, mt);
    if (four && split_k(a, ntiles, epi, mw, mt)) {
      launch_sp<3, 1, 128, 128, 1, 2, 4, 2, true, 1, false, false, 1>(s, a, ntiles);
      launch_sp<3, 1, 128, 128, 1, 2, 4, 2, true, 1, false, false, 2>(s, a, ntiles);
    } else if (!four && split_k(a, ntiles, epi, mw, mt)) {
      launch_sp<3, 1, 128, 128, 1, 2, 8, 2, true, 1, false, false, 1>(s, a, ntiles);
      launch_sp<3, 1, 128, 128, 1, 2, 8, 2, true, 1, false, false, 2>(s, a, ntiles);
    } else if (four) {
      launch<3, 1, 128, 128, 1, 2, 4, 2>(s, a, ntiles);
    } else {
      launch<3, 1, 128, 128, 1, 2, 8, 2>(s, a, ntiles);
    }
  }
  else if (ks == 1 && tl.bm == 64) launch<1, 1, 64, 128, 2, 4, 4, 2>(s, a, ntiles);
  else if (ks == 1 && tl.bm == 256 && tl.bn == 256) launch<1, 1, 256, 256, 2, 2, 8, 2>(s, a, ntiles);
  else if (ks == 1 && tl.bm == 256) {
    if (x3_split256() && split_k(a, ntiles, epi, 256, 256, 256)) {
      launch_sp<1, 1, 256, 128, 2, 2, 8, 2, true, 1, false, false, 1>(s, a, ntiles);
      launch_sp<1, 1, 256, 128, 2, 2, 8, 2, true, 1, false, false, 2>(s, a, ntiles);
    } else {
      launch<1, 1, 256, 128, 2, 2, 8, 2>(s, a, ntiles);
    }
  }
  else if (ks == 1 && tl.bm == 128) {
    if (split_k(a, ntiles, epi, 384, 512)) {
      launch_sp<1, 1, 128, 128, 2, 2, 4, 2, true, 1, false, false, 1>(s, a, ntiles);
      launch_sp<1, 1, 128, 128, 2, 2, 4, 2, true, 1, false, false, 2>(s, a, ntiles);
    } else {
      launch<1, 1, 128, 128, 2, 2, 4, 2>(s, a, ntiles);
    }
  }
  else return false;
  return true;
}

// The cond_fea half of init_conv over a bilinear x2 upsample of F, phase-composed
// (runtime.cpp Pfea_phase): the 7x7 over the 2H x 2W upsampled map equals, per output phase
// (py, px), a 5x5 over the zero-padded H x W map F plus edge corrections (fea_x3.hip). This
// launch is the 5x5 part: Cout = 4 phases x C rows, out [B][C][T][2H][2W] (+= epi.res).
// EXTDM_FEA_XBUF=1: one X buffer (A/B; default two). dry: return whether the launch is covered
// (every check above, no launch).
bool conv_x3_phase_forward(hipStream_t s, const View& out, const View& in, const PackedW& w, const ConvEpi& epi,
                           float* edge, bool dry) {
  if (!w.wx || w.mode != MODE_CONV || w.KH != 5 || !((w.xbm == 64 && w.xbn == 512) || (w.xbm == 128 && w.xbn == 256)) ||
      w.M != 4 * out.C || out.C != 64)
    return false;
  if (out.H != 2 * in.H || out.W != 2 * in.W || out.B != in.B || out.T != in.T || in.C * 25 != w.K) return false;
  View og = out;  // the kernel's tile geometry: the input planes, 4C rows
  og.H = in.H; og.W = in.W; og.C = w.M;
  X3Args a;
  unsigned ntiles = 0;
  ConvEpi e = epi;
  e.stats = nullptr;
  // EXTDM_FEA_TILE=256: 64 x 256 px on 4 waves with one X buffer (66 KB of LDS: two workgroups
  // per CU); default 64 x 512 on 8 waves
  static const int bn = [] { const char* v = getenv("EXTDM_FEA_TILE"); return v ? atoi(v) : 512; }();
  PackedW wt = w;
  if (w.xbm == 64) wt.xbn = bn == 256 ? 256 : 512;
  if (!x3_setup(og, in, nullptr, wt, e, a, ntiles, nullptr)) return false;
  auto extent = [&](long sb, long sc, long st) {
    return ((long)(out.B - 1) * sb + (long)(out.C - 1) * sc + (long)(out.T - 1) * st + (long)out.H * out.W) * 4;
  };
  const long ob = extent(out.sb, out.sc, out.st);
  const long rb = e.res ? extent(e.res_sb, e.res_sc, e.res_st) : 0;
  if (ob >= (1L << 31) - 4 || rb >= (1L << 31) - 4) return false;
  a.out_bytes = (int)ob;
  a.res_bytes = (int)rb;
  if (edge && (in.H != in.W || in.C % 16 != 0 || w.xng != 1)) return false;
  a.edge = edge;
  if (dry) return true;  // coverage only (runtime.cpp fea_phase_on)
  static const int xbuf = [] { const char* v = getenv("EXTDM_FEA_XBUF"); return v ? atoi(v) : 2; }();
  if (wt.xbm == 128) launch_sp<5, 1, 128, 256, 1, 4, 8, 2, true, 1, false, false, 0, true>(s, a, ntiles);
  else if (wt.xbn == 512 && x3_ws_raw_ok(a, kWsPhase)) launch_sp<5, 1, 64, 512, 1, 8, 8, 2, true, 2, false, false, 0, true, true>(s, a, ntiles);
  else if (wt.xbn == 256) launch_sp<5, 1, 64, 256, 1, 4, 4, 1, true, 2, false, false, 0, true>(s, a, ntiles);
  else if (xbuf == 1) launch_sp<5, 1, 64, 512, 1, 8, 8, 1, true, 2, false, false, 0, true>(s, a, ntiles);
  else launch_sp<5, 1, 64, 512, 1, 8, 8, 2, true, 2, false, false, 0, true>(s, a, ntiles);
  return true;
}

bool conv_x3_covers(const View& out, const View& in0, const View* in1, const PackedW& w) {
  if (w.mode != MODE_CONV || w.KH != w.KW) return false;
  X3Args a;
  unsigned ntiles = 0;
  const int ks = w.KH;
  const bool tile_ok = (w.xbn == 512 && w.xbm == 64 && (ks == 7 || ks == 3)) ||
                       (w.xbn != 512 && ((ks == 7 && w.xbm == 64) || (ks == 3 && (w.xbm == 64 || w.xbm == 128)) ||
                                         (ks == 1 && (w.xbm == 64 || w.xbm == 128 || w.xbm == 256))));
  return tile_ok && x3_setup(out, in0, in1, w, ConvEpi{}, a, ntiles, nullptr);
}

static size_t conv_x3_split_bytes_256(const X3Args& a, unsigned ntiles) {
  return x3_split256() ? split_bytes(a, ntiles, split_slices(a, ntiles, 256, 256, 256)) : 0;
}

size_t conv_x3_split_bytes(const View& out, const View& in0, const View* in1, const PackedW& w) {
  X3Args a;
  unsigned ntiles = 0;
  if (w.mode != MODE_CONV || w.KH != w.KW || !x3_setup(out, in0, in1, w, ConvEpi{}, a, ntiles, nullptr)) return 0;
  if (w.xbn == 512 || (w.xbm != 128 && !(w.xbm == 256 && w.KH == 1))) return 0;
  if (w.xbm == 256) return conv_x3_split_bytes_256(a, ntiles);
  if (w.KH == 3) {
    long mw, mt;
    x3_split128(x3_w128_4(a, false), mw, mt);
    return split_bytes(a, ntiles, split_slices(a, ntiles, mw, mt));
  }
  if (w.KH == 1) return split_bytes(a, ntiles, split_slices(a, ntiles, 384, 512));
  return 0;
}

size_t conv_x3_op_split_bytes(const View& out, const PackedW& w, int C) {
  if (!conv_x3_op_supported(out, w, C, 1) || w.xbm != 128) return 0;
  X3Args a;
  unsigned ntiles = 0;
  const View g = cf_view(nullptr, out.B, C, out.T, out.H, out.W);
  if (!x3_setup(out, g, nullptr, w, ConvEpi{}, a, ntiles, nullptr)) return 0;
  long mw, mt;
  x3_split128(x3_w128_4(a, true), mw, mt);
  return split_bytes(a, ntiles, split_slices(a, ntiles, mw, mt));
}

size_t x3op_halves(int B, int C, int T, int H, int W, int pad) {
  // + one plane and 1 KiB of slack: the last tile's DMA pieces read past the last position
  const size_t plane = (size_t)(H + 2 * pad) * (W + 2 * pad) * 16;
  return 2 * (size_t)(C / 16) * B * T * plane + plane + 512;
}

bool conv_x3_op_supported(const View& out, const PackedW& w, int C, int pad) {
  if (!w.wx || w.mode != MODE_CONV || w.KH != 3 || w.KW != 3 || pad != 1 || w.xng != 1 || C % 16 != 0) return false;
  // EXTDM_NO_X3OP=1: the producer writes fp32 and the conv stages it (A/B)
  static const bool off = [] {
    auto on = [](const char* n) { const char* v = getenv(n); return v && v[0] && v[0] != '0'; };
    return on("EXTDM_X3_NOSPAN") || on("EXTDM_NO_X3OP");
  }();
  if (off) return false;
  const int H = out.H, W = out.W, bn = w.xbn;
  if (W > bn || bn % W != 0) return false;
  const int TH = std::min(H, bn / W);
  if (bn % (TH * W) != 0 || H % TH != 0) return false;
  const int NP = bn / (TH * W);
  if ((out.B * out.T) % NP != 0) return false;
  return w.xbm == 64 ? bn == 256 : (w.xbm == 128 && bn == 128);
}

bool conv_x3_forward_op(hipStream_t s, const View& out, const X3Op& in, const PackedW& w, const ConvEpi& epi,
                        int* stats_slots) {
  if (stats_slots) *stats_slots = 0;
  if (!conv_x3_op_supported(out, w, in.C, in.pad) || in.H != out.H || in.W != out.W || in.B != out.B ||
      in.T != out.T)
    return false;
  // geometry from a channel-first stand-in of the operand's activation (no staging reads)
  const View g = cf_view(nullptr, in.B, in.C, in.T, in.H, in.W);
  X3Args a;
  unsigned ntiles = 0;
  if (!x3_setup(out, g, nullptr, w, epi, a, ntiles, stats_slots)) return false;
  const size_t plane = (size_t)(in.H + 2 * in.pad) * (in.W + 2 * in.pad) * 8;  // one (hl, c8) plane
  a.xop = in.p;
  a.xop_cg = (long)((size_t)in.B * in.T * plane);
  a.xop_hl = 2 * (long)((size_t)(in.C / 16) * in.B * in.T * plane);
  if (w.xbm == 64) {
    if (x3_v3() == 1) launch_sp<3, 3, 64, 256, 1, 4, 8, 2, true, 1, true>(s, a, ntiles);
    else if (x3_ws(kWsOp64)) launch_sp<3, 1, 64, 256, 1, 4, 4, 2, true, 1, true, false, 0, false, true>(s, a, ntiles);
    else launch_sp<3, 1, 64, 256, 1, 4, 4, 2, true, 1, true>(s, a, ntiles);
    return true;
  }
  const bool four = x3_w128_4(a, true);
  long mw, mt;
  x3_split128(four, mw, mt);
  if (four && split_k(a, ntiles, epi, mw, mt)) {
    launch_sp<3, 1, 128, 128, 1, 2, 4, 2, true, 1, true, false, 1>(s, a, ntiles);
    launch_sp<3, 1, 128, 128, 1, 2, 4, 2, true, 1, true, false, 2>(s, a, ntiles);
  } else if (!four && split_k(a, ntiles, epi, mw, mt)) {
    launch_sp<3, 1, 128, 128, 1, 2, 8, 2, true, 1, true, false, 1>(s, a, ntiles);
    launch_sp<3, 1, 128, 128, 1, 2, 8, 2, true, 1, true, false, 2>(s, a, ntiles);
  } else if (four) {
    if (x3_ws(kWsOp128)) launch_sp<3, 1, 128, 128, 1, 2, 4, 2, true, 1, true, false, 0, false, true>(s, a, ntiles);
    else launch_sp<3, 1, 128, 128, 1, 2, 4, 2, true, 1, true>(s, a, ntiles);
  } else {
    if (x3_ws(kWsOp128)) launch_sp<3, 1, 128, 128, 1, 2, 8, 2, true, 1, true, false, 0, false, true>(s, a, ntiles);
    else launch_sp<3, 1, 128, 128, 1, 2, 8, 2, true, 1, true>(s, a, ntiles);
  }
  return true;
}

int* x3_range_ptr() {
  static thread_local int dev = -1;
  static thread_local int* ptr = nullptr;
  int d = 0;
  (void)hipGetDevice(&d);
  if (d != dev) {
    void* p = nullptr;
    (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_x3_range));
    ptr = reinterpret_cast<int*>(p);
    dev = d;
  }
  return ptr;
}

void x3_range_reset(hipStream_t s) {
  void* p = nullptr;
  (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_x3_range));
  (void)hipMemsetAsync(p, 0, sizeof(int), s);
}

int x3_range_read(hipStream_t s) {
  void* p = nullptr;
  int v = 0;
  (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_x3_range));
  (void)hipMemcpyAsync(&v, p, sizeof(int), hipMemcpyDeviceToHost, s);
  (void)hipStreamSynchronize(s);
  return v;
}

}  // namespace extdm
