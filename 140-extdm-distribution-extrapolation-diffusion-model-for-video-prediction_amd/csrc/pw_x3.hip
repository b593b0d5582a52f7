// Pointwise (1x1) 256 -> 256 f16x3 conv with the weights held in registers: TrajWarp's
// linear_q / linear_o per step and linear_k / linear_v per sampling call (u12:806-821 via
// MultiHeadAttentionOp), each 2 x 235 MB of fp32 activations per launch at the BAIR bench shape
// (B = 64, tp = 14, 16 x 16): HBM-bound, 3 FLOP-equivalents of MFMA per byte moved. (The fuser,
// u12:826, is 512 -> 256: its weights do not fit the register file and it stays on conv_x3.)
//
// Why not conv_x3's 1x1 tile: it streams the packed weights through LDS by DMA once per
// workgroup, and a 256-row weight matrix (256 KB of hi / lo halves) is twice the bytes of the
// 128-pixel input tile it multiplies, so each stage waited on an L2 round trip of weights (0.24
// of HBM). Here the 256 x 256 matrix lives in the register file for the whole launch: wave w of
// the 8 owns rows [32 w, 32 w + 32) for all 16 k-steps, 128 VGPRs of hi / lo fragments, loaded
// once. The workgroups are persistent (one per CU, 2 waves per SIMD) and loop over 64-pixel
// tiles of one frame; per tile the 256 input channels arrive as four 64-channel chunks through
// a ring of four LDS slots [hl][k8][px][8] (a lane's MFMA k-slice = one conflict-free 16-B
// record). Wave w fetches channels 8 w .. 8 w + 7 of each chunk by LDS-DMA into a raw fp32 ring
// (64 consecutive pixels per wave instruction: 256-B coalesced), four chunks ahead of the one
// being multiplied (48 KB in flight per CU), each lane reads its pixel's 8 values back after a
// counted vmcnt, splits them into hi / lo' fp16 (split2s) into the slot, and one barrier per
// chunk publishes it. Operands, products and accumulation order are conv_x3's (al bh, ah bh,
// ah 2^-11 bl' per k-step in k order; acc * wscale + bias): the BAIR forward through either
// path is bit-identical (tests/test_gpu_pw.py asserts it; round 5, library 374380dd94696d56).
#include <algorithm>
#include <cstdlib>

#include "kernels.h"

// EXTDM_PW_EXP (diagnostic builds only, results invalid): bit 0 = output stores predicated off,
// bit 1 = no input loads (zeros staged)
#ifndef EXTDM_PW_EXP
#define EXTDM_PW_EXP 0
#endif
// EXTDM_PW_MANUAL: the chunk loads as LDS-DMA (buffer_load_dword ... lds, inline asm) into a raw
// fp32 ring retired by counted waits of this kernel's own; 0 = plain buffer loads to registers
// with hipcc's waits (it counted only the loads younger than the awaited chunk, so with the
// previous tile's 32 output stores also younger it drained the prefetch at every tile start;
// and register-destination asm loads are unsafe: hipcc may copy a register before the wait)
#ifndef EXTDM_PW_MANUAL
#define EXTDM_PW_MANUAL 0
#endif
// EXTDM_PW_LOADFIRST: issue the next tile's chunk before waiting for chunk g + 1 (four chunks in
// flight at the wait instead of three)
#ifndef EXTDM_PW_LOADFIRST
#define EXTDM_PW_LOADFIRST 0
#endif

namespace extdm {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

constexpr int PW_M = 256, PW_K = 256;
constexpr int PW_NPX = 64;                         // pixels per tile (two n32 tiles)
constexpr int PW_KC = 64;                          // channels per chunk (4 k-steps)
constexpr int PW_NKC = PW_K / PW_KC;               // chunks per tile
constexpr int PW_KS = PW_K / 16;                   // k-steps
constexpr int PW_SLOT = 2 * (PW_KC / 8) * PW_NPX * 8;  // halves per slot: [hl][k8][px][8]

struct PwArgs {
  const float* x; long xb, xc, xt;  // input view strides (elements)
  int T, tpf, ntiles, x_bytes;      // tiles per frame (HW / 64), tiles, input extent
  const _Float16* w;                // conv_x3's packed 1x1 layout (xbm 256, xng 2), m-tile 0
  const float* wscale; const float* bias;
  float* out; long ob, oc, ot; int out_bytes;
  int act;
  int* range;
};

// one buffer_load_dword ... lds: lane l's dword at byte voff + soff of the resource lands at LDS
// byte lds + 4 l (wave-uniform LDS base in M0); retired by the issuing wave's own vmcnt
__device__ __forceinline__ void pw_dma(__amdgpu_buffer_rsrc_t rs, int voff, int soff, float* lds) {
  const unsigned dst =
      __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_dword %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rs), "s"(soff), "s"(dst)
               : "memory");
}

__global__ __launch_bounds__(512) void pw_x3_kernel(PwArgs a) {
  extern __shared__ __attribute__((aligned(16))) _Float16 sm[];
  float* const esb = reinterpret_cast<float*>(sm + PW_NKC * PW_SLOT);  // [scale 256][bias 256]
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, lc = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // the wave's weight rows for every k-step (conv_x3 packing: [(cb, g) = k-step][m32][hl][lane][8])
  h8 ah[PW_KS], al[PW_KS];
#pragma unroll
  for (int s = 0; s < PW_KS; ++s) {
    const _Float16* wp = a.w + ((long)(s * 8 + wave) * 2) * 512 + lane * 8;
    ah[s] = *reinterpret_cast<const h8*>(wp);
    al[s] = *reinterpret_cast<const h8*>(wp + 512);
  }
  // retired here, before any chunk load: a weight load still pending in hipcc's count at its
  // first MFMA use inside the tile loop put a static vmcnt wait there that, with the chunk
  // loads outside that count, drained the prefetch on every pass
#pragma unroll
  for (int s = 0; s < PW_KS; ++s) asm volatile("" ::"v"(ah[s]), "v"(al[s]));
  if (tid < PW_M) {
    esb[tid] = a.wscale[tid];
    esb[PW_M + tid] = a.bias ? a.bias[tid] : 0.f;
  }

  // staging role: pixel `lane` of the tile, channels 8 wave .. 8 wave + 7 of each chunk
  const auto rsx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x), 0, a.x_bytes, 0x00020000);
  const int cs4 = (int)a.xc * 4;
  const int T = a.T, tpf = a.tpf, ntiles = a.ntiles, G = (int)gridDim.x;
  auto tile_base = [&](int tile) __attribute__((always_inline)) {  // element offset of pixel `lane`
    tile = tile < ntiles ? tile : ntiles - 1;  // past the last tile: a harmless re-read
    const int f = tile / tpf, p0 = (tile - f * tpf) * PW_NPX;
    const int b = f / T, t = f - b * T;
    return (int)((long)b * a.xb + (long)t * a.xt) + p0 + lane;
  };
#if EXTDM_PW_MANUAL
  // raw fp32 ring [chunk slot][64 channels][64 px] after the split slots; a wave DMAs and later
  // reads back only its own 8 channel rows, so its own vmcnt orders the two (no barrier)
  float* const raw = reinterpret_cast<float*>(esb + 2 * PW_M);
  auto load_chunk = [&](int slot, int base) __attribute__((always_inline)) {
#if EXTDM_PW_EXP & 2
    return;
#endif
    const int c0 = slot * PW_KC + wave * 8;
    float* const r = raw + (slot * PW_KC + wave * 8) * PW_NPX;
#pragma unroll
    for (int e = 0; e < 8; ++e) pw_dma(rsx, base * 4, (c0 + e) * cs4, r + e * PW_NPX);
  };
#else
  float xr[PW_NKC][8];
  auto load_chunk = [&](int slot, int base) __attribute__((always_inline)) {
    const int c0 = slot * PW_KC + wave * 8;
#if EXTDM_PW_EXP & 2
#pragma unroll
    for (int e = 0; e < 8; ++e) xr[slot][e] = 0.f;
    return;
#endif
#pragma unroll
    for (int e = 0; e < 8; ++e)
      xr[slot][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsx, base * 4, (c0 + e) * cs4, 0));
  };
#endif
  float am = 0.f;
  // `younger`: vector-memory operations this wave issued after the chunk's loads (loads, stores and
  // LDS-DMA retire in issue order, MI355X_MICROARCH.md vmcnt), so vmcnt(younger) retires exactly
  // the chunk; a smaller count only waits longer. Pinned here (volatile, ordered with the
  // barriers): otherwise the scheduler hoists the chunk's split / range VALU right behind its loads.
  auto store_chunk = [&](int slot, int younger) __attribute__((always_inline)) {
    float x[8];
#if EXTDM_PW_MANUAL
    if (younger >= 63) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
    else if (younger >= 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
    else if (younger >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    const float* r = raw + (slot * PW_KC + wave * 8) * PW_NPX + lane;
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = r[e * PW_NPX];
#else
    (void)younger;
    asm volatile("" : "+v"(xr[slot][0]), "+v"(xr[slot][1]), "+v"(xr[slot][2]), "+v"(xr[slot][3]), "+v"(xr[slot][4]),
                 "+v"(xr[slot][5]), "+v"(xr[slot][6]), "+v"(xr[slot][7]));
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = xr[slot][e];
#endif
    unsigned hw[4], lw[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      split2s(x[2 * c], x[2 * c + 1], hw[c], lw[c]);
      amax2(am, x[2 * c], x[2 * c + 1]);
    }
    _Float16* d = sm + slot * PW_SLOT + (wave * PW_NPX + lane) * 8;
    *reinterpret_cast<h8*>(d) = __builtin_bit_cast(h8, u32x4{hw[0], hw[1], hw[2], hw[3]});
    *reinterpret_cast<h8*>(d + PW_SLOT / 2) = __builtin_bit_cast(h8, u32x4{lw[0], lw[1], lw[2], lw[3]});
  };

  f32x16 acc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  const int t0 = blockIdx.x;
  const int nit = t0 < ntiles ? (ntiles - t0 + G - 1) / G : 0;
  const int base_cur = tile_base(t0);
  int base_next = tile_base(t0 + G);
#pragma unroll
  for (int kc = 0; kc < PW_NKC; ++kc) load_chunk(kc, base_cur);
  store_chunk(0, 24);

  const auto rs_out = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, a.out_bytes, 0x00020000);
  const bool relu = a.act == ACT_RELU;
  const int oc = (int)a.oc;
  const int epi_ops = 32;  // the epilogue's vector-memory operations per tile (stores)
  for (int it = 0; it < nit; ++it) {
#pragma unroll
    for (int kc = 0; kc < PW_NKC; ++kc) {
      // chunk g + 1 into its slot, then chunk g + 4 (the next tile's chunk kc) into the registers
      // chunk g freed: three chunks in flight, each with three chunk-times of cover
      // younger than chunk g + 1: the two chunks loaded after it, and for kc < 3 the previous
      // tile's epilogue (none before the first tile)
#if EXTDM_PW_LOADFIRST
      load_chunk(kc, base_next);
      store_chunk((kc + 1) & 3, 24 + (kc < 3 && it > 0 ? epi_ops : 0));
#else
      store_chunk((kc + 1) & 3, 16 + (kc < 3 && it > 0 ? epi_ops : 0));
      load_chunk(kc, base_next);
#endif
      // slot g + 1 published; slot g (written one chunk earlier) readable by every wave
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      const _Float16* sl = sm + kc * PW_SLOT;
#pragma unroll
      for (int ks = 0; ks < PW_KC / 16; ++ks) {
        const int s = kc * (PW_KC / 16) + ks;
        h8 bh[2], bl[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const _Float16* bp = sl + ((2 * ks + h) * PW_NPX + 32 * j + lc) * 8;
          bh[j] = *reinterpret_cast<const h8*>(bp);
          bl[j] = *reinterpret_cast<const h8*>(bp + PW_SLOT / 2);
        }
        // opaque per tile: hoisted out of the tile loop, the 16 lo_dn products would take 64 more
        // VGPRs than the register file has left (scratch spills)
        asm volatile("" : "+v"(ah[s]));
        const h8 ad = lo_dn(ah[s]);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[s], bh[j], acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s], bh[j], acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ad, bl[j], acc[j], 0, 0, 0);
        }
      }
    }
    // ---- epilogue of tile t0 + it G (C/D map: col = lane & 31, row = (r&3) + 8(r>>2) + 4h) ----
    const int tile = t0 + it * G;
    const int f = tile / tpf, p0 = (tile - f * tpf) * PW_NPX;
    const int b = f / T, t = f - b * T;
    const int obase = (int)((long)b * a.ob + (long)t * a.ot) + p0 + lc;
    // four rows at a time (scale / bias from LDS): the 128 weight VGPRs stay live throughout
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int m0 = wave * 32 + 8 * k + 4 * h;
      const float4 s4 = *reinterpret_cast<const float4*>(esb + m0);
      const float4 b4 = *reinterpret_cast<const float4*>(esb + PW_M + m0);
      const float sc[4] = {s4.x, s4.y, s4.z, s4.w}, bi[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = acc[j][4 * k + q] * sc[q] + bi[q];
        if (relu) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = v[q] > 0.f ? v[q] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          // the row's wave-uniform part in soffset: no per-row VGPR offsets to keep live
#if EXTDM_PW_EXP & 1
          if (v[q] == 12345.678f)
#endif
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[q]), rs_out, (obase + 32 * j + 4 * h * oc) * 4,
                                                (wave * 32 + 8 * k + q) * oc * 4, 0);
          acc[j][4 * k + q] = 0.f;
        }
      }
    }
    base_next = tile_base(t0 + (it + 2) * G);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the prefetches past the last tile
  if (am >= 65504.f) atomicOr(a.range, 1);
}

int pw_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t p;
    n = hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0 ? p.multiProcessorCount : 256;
  }
  return n;
}

// extent in bytes of a view's addressed range (0 if it does not fit a 32-bit buffer offset)
int view_bytes(const View& v) {
  const long last = (long)(v.B - 1) * v.sb + (long)(v.C - 1) * v.sc + (long)(v.T - 1) * v.st + (long)v.H * v.W;
  return last * 4 < (1L << 31) ? (int)(last * 4) : 0;
}

}  // namespace

// read per launch decision (not cached): tests compare both paths in one process
bool pw_x3_enabled() {
  const char* v = getenv("EXTDM_NO_PW");
  return !(v && v[0] && v[0] != '0');
}

bool pw_x3_forward(hipStream_t s, const View& out, const View& in, const PackedW& w, const ConvEpi& e) {
  if (!pw_x3_enabled() || !w.wx || w.KH != 1 || w.KW != 1 || w.xbm != PW_M || w.xng != 2 || w.xncgb != PW_K / 32)
    return false;
  if (in.C != PW_K || out.C != PW_M || in.B != out.B || in.T != out.T || in.H != out.H || in.W != out.W)
    return false;
  const int HW = in.H * in.W;
  if (HW % PW_NPX != 0 || e.res || e.stats || e.post_scale || e.res_aff) return false;
  if (e.act != ACT_NONE && e.act != ACT_RELU) return false;
  PwArgs a{};
  a.x = in.p; a.xb = in.sb; a.xc = in.sc; a.xt = in.st;
  a.T = in.T; a.tpf = HW / PW_NPX; a.ntiles = in.B * in.T * a.tpf;
  a.x_bytes = view_bytes(in);
  a.w = reinterpret_cast<const _Float16*>(w.wx); a.wscale = w.xscale; a.bias = e.bias;
  a.out = out.p; a.ob = out.sb; a.oc = out.sc; a.ot = out.st; a.out_bytes = view_bytes(out);
  a.act = e.act; a.range = x3_range_ptr();
  if (!a.x_bytes || !a.out_bytes) return false;
  const unsigned grid = (unsigned)std::min(a.ntiles, pw_cus());
  const size_t lds = (size_t)PW_NKC * PW_SLOT * 2 + 2 * PW_M * 4 + (EXTDM_PW_MANUAL ? (size_t)PW_NKC * PW_KC * PW_NPX * 4 : 0);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&pw_x3_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(pw_x3_kernel, dim3(grid), dim3(512), lds, s, a);
  return true;
}

}  // namespace extdm
