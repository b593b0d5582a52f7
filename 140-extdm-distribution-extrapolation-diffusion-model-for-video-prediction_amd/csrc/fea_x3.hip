// Edge corrections of the phase-composed init_conv cond_fea branch (u12:1034-1041; ada the
// same through fup): r += Wb * pad(up2(F)), Wb the last fea_ch input channels of init_conv
// (1,7,7), up2 = F.interpolate(..., size = 2H x 2W, mode='bilinear') (align_corners=False).
//
// Per axis, the upsampled row r of F is U(r) = sum_k U[r][k] F[k] with
//   U[r][k] = the clamped bilinear weights for r in [0, 2H), 0 outside (the conv's zero pad).
// Write U = Uinf + D, where Uinf is the unclamped, unpadded interpolation of the zero-padded F
// (2j: .75 F[j] + .25 F[j-1], 2j+1: .75 F[j] + .25 F[j+1], any integer r). Uinf is shift-
// invariant in the output phase, so the 7x7 over Uinf F Uinf^T is, per output phase (py, px),
// a 5x5 over the zero-padded H x W map: conv_x3_phase_forward (conv_x3.hip), 25 taps instead
// of 49 and a quarter of the input pixels. D has four entries: -.25 / +.25 at rows -1 / 0 of
// column 0 and +.25 / -.25 at rows 2H-1 / 2H of column H-1, so
//   7x7(U F U^T) = 7x7(Uinf F Uinf^T) + [D F Uinf^T] + [Uinf F D^T] + [D F D^T]
// and the three corrections touch only the 4-pixel border ring of the output:
//   fea_side_x3_kernel  the edge lines: [D F Uinf^T] for output rows 0-3 / 2H-4..2H-1 from F's
//                       rows 0 / H-1, [Uinf F D^T] for the columns likewise; per (d, py, px, c)
//                       a 5-tap 1-D conv of the line (an f16x3 GEMM, K = 5 * Cin)
//   fea_corner_kernel   [D F D^T]: the 4 x 4 corner pixels from F's corner value, K = Cin, fp32
// Both add into the output (read-modify-write; the top/bottom launch, the left/right launch
// and the corner launch run in sequence, so a corner pixel's three additions keep one order).
// Weights are composed in fp64 at first use (runtime.cpp Pfea_phase).
#include <cstdlib>

#include "kernels.h"

namespace extdm {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int SBM = 128;   // rows per m-tile
constexpr int SBN = 256;   // line positions per column tile (whole lines)
constexpr int SNW = 8;     // waves: 2 (rows) x 4 (columns), 64 x 64 each
constexpr int STAPS = 5;

// One (line pair, m-tile, column tile): C[m][n] = sum_{ci, l} W[m][ci][l] line[n + l - 2][ci].
// Rows m = c * 8 + (d * 2 + py) * 2 + px (d = depth from the edge): a lane's accumulator rows
// (r & 3) + 8 (r >> 2) + 4h are, per channel, the four (py, px) of one depth, so its epilogue
// reads and writes 8-B pairs of neighbouring pixels. Columns n = (frame, j).
// LDS: A per 16-channel block [tap][m32][hl][lane][8] by LDS-DMA (two slots), X [hl][pos][16]
// with pos = frame * (L + 4) + j + 2 (zero halo of 2 on each side of a line), two buffers.
__global__ __launch_bounds__(SNW * 64) void fea_side_x3_kernel(FeaSideArgs a) {
  constexpr int TM = 2, TN = 2, WN = 4;
  constexpr int AH = STAPS * (SBM / 32) * 2 * 512;  // halves per A slot
  extern __shared__ __attribute__((aligned(16))) _Float16 sm[];
  const int L = a.L, LP = L + 4, NFT = SBN / L;
  const int XPOS = NFT * LP;
  const int XH = XPOS * 16;  // halves per (hl) half of an X buffer
  _Float16* As0 = sm;
  _Float16* As1 = sm + AH;
  _Float16* Xs0 = sm + 2 * AH;
  _Float16* Xs1 = Xs0 + 2 * XH;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int h = lane >> 5, lc = lane & 31;
  const int side = blockIdx.z, mtile = blockIdx.y;
  const int q0 = blockIdx.x * NFT;  // first frame (b * T + t) of the tile
  const int line = 2 * a.pair + side;  // top, bottom, left, right
  const int ncb = a.C / 16;
  const _Float16* wt = a.w + ((long)side * gridDim.y + mtile) * ncb * AH;

  // staging slot: one (frame, position) of the tile, 16 channels
  const bool sl_ok = tid < XPOS;
  const int sf = sl_ok ? tid / LP : 0, sj = sl_ok ? tid % LP - 2 : 0;
  const int sq = q0 + sf;
  const bool in_ok = sl_ok && sq < a.P && sj >= 0 && sj < L;
  const long soff = in_ok ? (((long)sq * 4 + line) * L + sj) * a.C : 0;
  float xr[16];
  float am = 0.f;
  auto load_x = [&](int cb) __attribute__((always_inline)) {
    const float4* p = reinterpret_cast<const float4*>(a.e + soff + cb * 16);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float4 v = in_ok ? p[c] : make_float4(0.f, 0.f, 0.f, 0.f);
      xr[4 * c] = v.x; xr[4 * c + 1] = v.y; xr[4 * c + 2] = v.z; xr[4 * c + 3] = v.w;
    }
  };
  auto store_x = [&](_Float16* Xs) __attribute__((always_inline)) {
    if (!sl_ok) return;
    unsigned hw[8], lw[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      split2s(xr[2 * c], xr[2 * c + 1], hw[c], lw[c]);
      amax2(am, xr[2 * c], xr[2 * c + 1]);
    }
    const int sw = (tid >> 3) & 1;
    _Float16* dh = Xs + tid * 16;
    *reinterpret_cast<h8*>(dh + 8 * sw) = __builtin_bit_cast(h8, u32x4{hw[0], hw[1], hw[2], hw[3]});
    *reinterpret_cast<h8*>(dh + 8 * (sw ^ 1)) = __builtin_bit_cast(h8, u32x4{hw[4], hw[5], hw[6], hw[7]});
    *reinterpret_cast<h8*>(dh + XH + 8 * sw) = __builtin_bit_cast(h8, u32x4{lw[0], lw[1], lw[2], lw[3]});
    *reinterpret_cast<h8*>(dh + XH + 8 * (sw ^ 1)) = __builtin_bit_cast(h8, u32x4{lw[4], lw[5], lw[6], lw[7]});
  };
  auto load_a = [&](int cb, _Float16* As) __attribute__((always_inline)) {
    const _Float16* src = wt + (long)cb * AH;
    for (int pc = wave; pc < AH / 512; pc += SNW)
      __builtin_amdgcn_global_load_lds((const void*)(src + pc * 512 + lane * 8), (lds_ptr_t)(As + pc * 512), 16, 0, 0);
  };

  // per-lane B positions (tap 0)
  int bpos[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = (wn * TN + j) * 32 + lc;
    bpos[j] = (n / L) * LP + n % L;
  }
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  load_x(0);
  load_a(0, As0);
  store_x(Xs0);
  __syncthreads();
  for (int cb = 0; cb < ncb; ++cb) {
    const _Float16* As = (cb & 1) ? As1 : As0;
    const _Float16* Xs = (cb & 1) ? Xs1 : Xs0;
    const bool more = cb + 1 < ncb;
    if (more) {
      load_a(cb + 1, (cb & 1) ? As0 : As1);
      load_x(cb + 1);
    }
#pragma unroll
    for (int l = 0; l < STAPS; ++l) {
      h8 ah[TM], al[TM], ad[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const _Float16* ap = As + ((l * (SBM / 32) + wm * TM + i) * 2) * 512 + lane * 8;
        ah[i] = *reinterpret_cast<const h8*>(ap);
        al[i] = *reinterpret_cast<const h8*>(ap + 512);
        ad[i] = lo_dn(ah[i]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int pos = bpos[j] + l;
        const _Float16* bp = Xs + pos * 16 + 8 * (h ^ ((pos >> 3) & 1));
        bh[j] = *reinterpret_cast<const h8*>(bp);
        bl[j] = *reinterpret_cast<const h8*>(bp + XH);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ad[i], bl[j], acc[i][j], 0, 0, 0);
        }
    }
    if (more) store_x((cb & 1) ? Xs0 : Xs1);
    __syncthreads();
  }
  if (am >= 65504.f) atomicOr(a.range, 1);

  // ---- epilogue: out[b][c][t][y][x] += acc * wscale (C/D map: col = lane & 31, row = (r&3) + 8(r>>2) + 4h)
  const float* wsc = a.wscale + (long)side * gridDim.y * SBM;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, a.out_bytes, 0x00020000);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = (wn * TN + j) * 32 + lc;
    const int fl = n / L, jj = n % L;
    const int q = q0 + fl;
    const bool valid = q < a.P && fl < NFT;
    const int qq = valid ? q : 0;
    const int b = qq / a.T, t = qq - b * a.T;
    const int base = (int)((long)b * a.ob + (long)t * a.ot);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      // rows of this lane: channel c = m >> 3 for r >> 2 = 0..3, phase (d = h, py, px) = r & 3
      if (a.pair == 0) {
        // rows y = base + 2h + py: a lane owns the pixel pair x = 2jj, 2jj + 1 (8 B; the 32 lanes
        // of a half cover 256 contiguous bytes of the row)
        int off[8];
        float2 rv[8];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = (mtile * SBM + (wm * TM + i) * 32 + 8 * g) >> 3;
#pragma unroll
          for (int py = 0; py < 2; ++py) {
            const int k = 2 * g + py;
            const int y = (side ? a.OH - 4 : 0) + 2 * h + py, x = 2 * jj;
            off[k] = valid && c < a.Co ? (base + (int)(c * a.oc) + y * a.OW + x) * 4 : a.out_bytes;
            const u32x2 ld = __builtin_amdgcn_raw_buffer_load_b64(rs, off[k], 0, 0);
            rv[k] = make_float2(__uint_as_float(ld.x), __uint_as_float(ld.y));
          }
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int m0 = mtile * SBM + (wm * TM + i) * 32 + 8 * g + 4 * h;
#pragma unroll
          for (int py = 0; py < 2; ++py) {
            const int k = 2 * g + py, r = 4 * g + 2 * py;  // acc rows r (px = 0), r + 1 (px = 1)
            const float v0 = rv[k].x + acc[i][j][r] * wsc[m0 + 2 * py];
            const float v1 = rv[k].y + acc[i][j][r + 1] * wsc[m0 + 2 * py + 1];
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, make_float2(v0, v1)), rs, off[k], 0, 0);
          }
        }
      } else {
        // columns x = base + 2h + px of rows y = 2jj + py: lane h = 0 holds x = base, base + 1
        // and lane h = 1 x = base + 2, base + 3 of the same two rows; one exchange across the
        // halves gives lane h the whole 16-B row piece of row y = 2jj + h
        int off[4];
        float4 rv[4];
        const int x0 = side ? a.OW - 4 : 0;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = (mtile * SBM + (wm * TM + i) * 32 + 8 * g) >> 3;
          const int y = 2 * jj + h;
          off[g] = valid && c < a.Co ? (base + (int)(c * a.oc) + y * a.OW + x0) * 4 : a.out_bytes;
          const u32x4 ld = __builtin_amdgcn_raw_buffer_load_b128(rs, off[g], 0, 0);
          rv[g] = make_float4(__uint_as_float(ld.x), __uint_as_float(ld.y), __uint_as_float(ld.z),
                              __uint_as_float(ld.w));
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int m0 = mtile * SBM + (wm * TM + i) * 32 + 8 * g + 4 * h;
          // this lane's products: (py, px) = r & 3 at x = base + 2h + px, y = 2jj + py
          float p00 = acc[i][j][4 * g] * wsc[m0], p01 = acc[i][j][4 * g + 1] * wsc[m0 + 1];
          float p10 = acc[i][j][4 * g + 2] * wsc[m0 + 2], p11 = acc[i][j][4 * g + 3] * wsc[m0 + 3];
          // send the row this lane does not store (py = 1 - h) to the partner lane (lane ^ 32)
          const float s0 = h ? p00 : p10, s1 = h ? p01 : p11;
          const float r0 = __shfl_xor(s0, 32), r1 = __shfl_xor(s1, 32);
          // row y = 2jj + h: x = base .. base + 3 = (h = 0: own px 0, 1 | partner's) (h = 1: partner's | own)
          const float k0 = h ? p10 : p00, k1 = h ? p11 : p01;
          const float4 add = h ? make_float4(r0, r1, k0, k1) : make_float4(k0, k1, r0, r1);
          const float4 v = make_float4(rv[g].x + add.x, rv[g].y + add.y, rv[g].z + add.z, rv[g].w + add.w);
          __builtin_amdgcn_raw_buffer_store_b128(
              u32x4{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)}, rs,
              off[g], 0, 0);
        }
      }
    }
  }
}

// [D F D^T]: out[b][c][t][y][x] += sum_ci Dw[corner][p][ci][c] F[b][ci][t][ky][kx] for the 16
// pixels p = (yy, xx) of each corner block (y = yy or 2H-4+yy, x likewise), fp32. A block owns
// one corner, 16 frames and 16 output channels: thread = (pixel, channel) with the 16 frames'
// sums; F's corner values in LDS (broadcast float4 reads), one weight load per input channel.
__global__ __launch_bounds__(256) void fea_corner_kernel(FeaCornerArgs a) {
  __shared__ __attribute__((aligned(16))) float fc[512 * 16];  // [ci][16 frames], Cin <= 512
  const int corner = blockIdx.y, q0 = blockIdx.x * 16;
  // F's corner value: top (0) / bottom (1) line, position 0 / L - 1
  const int eline = corner >> 1, epos = (corner & 1) ? a.L - 1 : 0;
  for (int i = threadIdx.x; i < a.C * 16; i += blockDim.x) {
    const int f = i / a.C, ci = i % a.C, q = q0 + f;
    fc[ci * 16 + f] = q < a.P ? a.e[(((long)q * 4 + eline) * a.L + epos) * a.C + ci] : 0.f;
  }
  __syncthreads();
  const int p = threadIdx.x & 15, c = blockIdx.z * 16 + (threadIdx.x >> 4);  // p fastest: 16-B row pieces
  if (c >= a.Co) return;
  float acc[16];
#pragma unroll
  for (int f = 0; f < 16; ++f) acc[f] = 0.f;
  // weights [corner][ci][c][p]: a wave's 64 lanes (4 channels x 16 pixels) read 256 contiguous bytes
  const float* wp = a.dw + ((long)corner * a.C * a.Co + c) * 16 + p;
#pragma unroll 4
  for (int ci = 0; ci < a.C; ++ci) {
    const float w = wp[(long)ci * a.Co * 16];
    const float4* fv = reinterpret_cast<const float4*>(fc + ci * 16);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 v = fv[k];
      acc[4 * k] = fmaf(w, v.x, acc[4 * k]);
      acc[4 * k + 1] = fmaf(w, v.y, acc[4 * k + 1]);
      acc[4 * k + 2] = fmaf(w, v.z, acc[4 * k + 2]);
      acc[4 * k + 3] = fmaf(w, v.w, acc[4 * k + 3]);
    }
  }
  const int yy = p >> 2, xx = p & 3;
  const int y = ((corner >> 1) ? a.OH - 4 : 0) + yy, x = ((corner & 1) ? a.OW - 4 : 0) + xx;
#pragma unroll
  for (int f = 0; f < 16; ++f) {
    const int q = q0 + f;
    if (q >= a.P) break;
    const int b = q / a.T, t = q - b * a.T;
    a.out[(long)b * a.ob + (long)t * a.ot + (long)c * a.oc + (long)y * a.OW + x] += acc[f];
  }
}

}  // namespace

bool fea_edges_supported(int C, int Co, int L) {
  return C % 16 == 0 && C <= 512 && Co % 16 == 0 && Co <= 64 && L >= 4 && SBN % L == 0 && (SBN / L) * (L + 4) <= SNW * 64;
}

bool fea_edges_forward(hipStream_t s, const View& out, const float* edge, int C, const void* side_w,
                       const float* side_scale, const float* corner_w, bool dry) {
  const int L = out.H / 2, Co = out.C;
  if (out.W != out.H || out.H % 2 != 0 || !fea_edges_supported(C, Co, L)) return false;
  const long ext = ((long)(out.B - 1) * out.sb + (long)(Co - 1) * out.sc + (long)(out.T - 1) * out.st + 4L * L * L) * 4;
  if (ext >= (1L << 31) - 4) return false;
  if (dry) return true;
  FeaSideArgs a{};
  a.e = edge;
  a.C = C; a.L = L; a.T = out.T; a.P = out.B * out.T;
  a.out = out.p; a.ob = out.sb; a.oc = out.sc; a.ot = out.st; a.OH = out.H; a.OW = out.W; a.Co = Co;
  a.out_bytes = (int)ext;
  a.range = x3_range_ptr();
  const int mt = (8 * Co + SBM - 1) / SBM, nft = SBN / L;
  const size_t ah = (size_t)STAPS * (SBM / 32) * 2 * 512;
  const size_t lds = (2 * ah + 2 * 2 * (size_t)nft * (L + 4) * 16) * sizeof(_Float16);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&fea_side_x3_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const dim3 grid((unsigned)((a.P + nft - 1) / nft), (unsigned)mt, 2);
  const size_t per_pair = (size_t)2 * mt * (C / 16) * ah;
  for (int pair = 0; pair < 2; ++pair) {
    FeaSideArgs b = a;
    b.pair = pair;
    b.w = reinterpret_cast<const _Float16*>(side_w) + pair * per_pair;
    b.wscale = side_scale + (size_t)pair * 2 * mt * SBM;
    hipLaunchKernelGGL(fea_side_x3_kernel, grid, dim3(SNW * 64), lds, s, b);
  }
  FeaCornerArgs c{};
  c.e = edge;
  c.C = C; c.L = L; c.T = out.T; c.P = out.B * out.T;
  c.out = out.p; c.ob = out.sb; c.oc = out.sc; c.ot = out.st; c.OH = out.H; c.OW = out.W; c.Co = Co;
  c.dw = corner_w;
  hipLaunchKernelGGL(fea_corner_kernel, dim3((unsigned)((c.P + 15) / 16), 4, (unsigned)((Co + 15) / 16)), dim3(256), 0, s,
                     c);
  return true;
}

}  // namespace extdm
