// init_conv's x-branch folded with init_noise_conv (u12:913-914, 1029-1041; ada the
// same), f16x3 MFMA.
//
// The reference computes
//     r = init_conv(cat(init_noise_conv(x), fu))              (1,7,7) convs, pad 3
// i.e. r = Wa * pad(x0) + Wb * pad(fu) + b with x0 = Wn * pad(x) + bn (3 -> 256 ch)
// and Wa the first 256 input channels of init_conv. Both branches are linear, so
// Wa * pad(x0) is ONE 13x13 convolution of the 3-channel x with the composed
// kernel Wa o Wn, except that pad(x0) is zero outside the latent: the intermediate
// positions q = p + (a-3, b-3) that fall outside [0, L) drop out. Which ones do
// depends only on how close p is to each border, so there are 7 classes per axis
// (0, 1, 2, interior, L-3, L-2, L-1) and 49 composed kernels
//     K_c[m][ci][dy][dx] = sum_{(a,b) valid for c} sum_c' Wa[m][c'][a][b] Wn[c'][ci][dy-a][dx-b]
// plus the per-class constant sum_{(a,b) valid} sum_c' Wa[m][c'][a][b] bn[c'] + b[m]
// (built in fp64 at extdm_finalize, runtime.cpp pack_xpath). That is 3*169 MACs per
// output channel instead of 256*49 (the x-branch was half of init_conv's FLOPs).
//
// The kernel is an implicit GEMM per class: M = Cout (32 * M32), K = 3 ch x 13 rows x
// 16 columns (13 used), N = the class's pixels over all frames (a class's pixel set
// is rows(cy) x cols(cx) of every frame). One wave owns 32 NT pixels (NT n32 tiles) and
// all output channels; A (the class's packed weights, [kstep][m32][hl][lane][8]) is
// read straight from L2, B is gathered from the pre-split copy of x (8 consecutive columns per
// lane and k-step, already hi / lo'). No LDS, no barriers.
#include <algorithm>
#include <cstdlib>

#include "kernels.h"

// EXTDM_XP_EXP (diagnostic builds only, results invalid): bit 0 = xpath's output stores predicated off
#ifndef EXTDM_XP_EXP
#define EXTDM_XP_EXP 0
#endif

namespace extdm {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

constexpr int KSTEPS = 3 * 13;  // (ci, dy); 16 dx columns per step

__device__ __forceinline__ f32x16 mma3(const h8& ah, const h8& al, const h8& bh, const h8& bl, f32x16 c) {
  // the scaled-lo product last, so its lo_dn VALU is off the head of the chain
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(lo_dn(ah), bl, c, 0, 0, 0);  // scaled x lo (xpad_kernel)
  return c;
}

// hi / lo' fragments of 8 consecutive positions of a row of the zero-padded, pre-split copy of x
// (xpad_kernel: one dword per position, hi in the low half, lo' = fp16((v - hi) 2^11) in the
// high half): two 16-B loads (dword alignment suffices for global_load_dwordx4) and 8 v_perm_b32,
// no index, clamp, mask or split VALU in the k-loop (the round-3 fp32 copy split every gathered
// value again in each of the 13 k-steps that read it: 8.8 VALU per MFMA in xpath's k-loop,
// profiles/r04_sq_layers.txt). Columns the composed kernels do not use (dx >= 13, noise_pool's
// 8th column) are read from the padding or the next columns and meet zero weights: the values
// are finite, so their products are exact zeros.
__device__ __forceinline__ void gather8p(const unsigned* p, h8& bh, h8& bl) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint4 w = *reinterpret_cast<const uint4*>(p + 4);
  const unsigned v[8] = {u.x, u.y, u.z, u.w, w.x, w.y, w.z, w.w};
  unsigned hi[4], lo[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    hi[e] = __builtin_amdgcn_perm(v[2 * e + 1], v[2 * e], 0x05040100u);  // low halves
    lo[e] = __builtin_amdgcn_perm(v[2 * e + 1], v[2 * e], 0x07060302u);  // high halves
  }
  bh = __builtin_bit_cast(h8, u32x4{hi[0], hi[1], hi[2], hi[3]});
  bl = __builtin_bit_cast(h8, u32x4{lo[0], lo[1], lo[2], lo[3]});
}

// x [B][3][T][L][L] -> xpad [B][3][T][LP][LP] with x at (6, 6) and zeros around (LP >= L + 16:
// xpath reads rows py - 6 .. py + 6 and columns px - 6 .. px + 9, noise_pool rows 2yp - 3 ..
// 2yp + 5 and columns lc - 3 .. lc + 4), each position split once into the f16x3 pair
// (hi | lo' << 16; lo' = fp16(fma(hi, -2^11, 2^11 v)): v * 2^11 exact, the fma exact, one
// rounding) and range-checked here for both consumers
__global__ __launch_bounds__(256) void xpad_kernel(const float* __restrict__ x, long xb, long xc, long xt,
                                                   unsigned* __restrict__ xp, int T, int L, int LP, long n,
                                                   int* range) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int col = (int)(i % LP), row = (int)((i / LP) % LP);
  const long pl = i / ((long)LP * LP);  // (b, ci, t)
  const int t = (int)(pl % T), ci = (int)((pl / T) % 3);
  const long b = pl / (3L * T);
  const int y = row - 6, xx = col - 6;
  const float v = split_src((y >= 0 && y < L && xx >= 0 && xx < L) ? x[b * xb + ci * xc + t * xt + (long)y * L + xx] : 0.f);
  if (fabsf(v) >= 65504.f) atomicOr(range, 1);
  const _Float16 hi = (_Float16)v;
  const float up = split_src(X3_LO_UP);
  const _Float16 lo = (_Float16)__builtin_fmaf((float)hi, -up, v * up);
  xp[i] = (unsigned)__builtin_bit_cast(unsigned short, hi) | ((unsigned)__builtin_bit_cast(unsigned short, lo) << 16);
}

__device__ __forceinline__ void class_span(int c, int L, int& start, int& count) {
  if (c < 3) { start = c; count = 1; }
  else if (c == 3) { start = 3; count = L - 6; }
  else { start = L - 7 + c; count = 1; }
}

// Tile order (round 5): frame groups of FG frames, and within a group every class's tiles
// consecutively, the groups laid out XCD-contiguously (workgroup j runs on XCD j mod 8 and takes
// logical slot (j mod 8) nwg / 8 + j / 8). An output line of a border row or column is written by
// up to four classes (a border column class, the interior, the row class); in the class-major
// order those writes came hundreds of workgroups apart, after the first partial line had left L2,
// so each line reached HBM two or three times (PMC WRITE 648 MB for 235 MB of output). Now all
// classes of a group's frames run back to back on one XCD and the partial writes of a line merge in
// its L2 before the write-back.
// NT: n32 tiles (32-pixel columns) per wave sharing each A fragment load: 2 (64 px) or 4 (128 px:
// half the per-pixel weight reads from L2, twice the accumulators)
template <int M32, int NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void xpath_x3_kernel(XPathArgs a) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lc = lane & 31, h = lane >> 5;
  const int nwg = (int)gridDim.x;
  const int q = a.xcd ? (int)(blockIdx.x & 7) * (nwg >> 3) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  const int tile = q * 4 + wave;
  const int total = (a.ngroups - 1) * a.gtiles + a.tile_last[49];
  if (tile >= total) return;
  const int g = min(tile / a.gtiles, a.ngroups - 1);
  const bool lastg = g == a.ngroups - 1;
  const int lt = tile - g * a.gtiles;
  int cls = 0, cstart = 0;  // static indices: a dynamic index into the kernarg array spills it to scratch
#pragma unroll
  for (int c = 1; c < 49; ++c) {
    const int st = lastg ? a.tile_last[c] : a.tile_start[c];
    if (lt >= st) { cls = c; cstart = st; }
  }
  const int L = a.L;
  int y0, ry, x0, rx;
  class_span(cls / 7, L, y0, ry);
  class_span(cls % 7, L, x0, rx);
  const int fg = lastg ? a.F - g * a.FG : a.FG;
  const int per = ry * rx, npx = fg * per;
  const int base = (lt - cstart) * (32 * NT);

  int py[NT], px[NT];
  long xoff[NT], ooff[NT], aoff[NT];
  bool ok[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int idx = base + nt * 32 + lc;
    ok[nt] = idx < npx;
    const int i = ok[nt] ? idx : 0;
    const int f = g * a.FG + i / per, rem = i - (i / per) * per;
    const int iy = rem / rx, ix = rem - iy * rx;
    const int b = f / a.T, t = f - b * a.T;
    py[nt] = y0 + iy;
    px[nt] = x0 + ix;
    xoff[nt] = (long)b * a.xb + (long)t * a.xt + (long)py[nt] * a.LP + px[nt];  // padded: row py + dy, col px + 8h
    ooff[nt] = (long)b * a.ob + (long)t * a.ot + (long)py[nt] * L + px[nt];
    aoff[nt] = (long)b * a.ab + (long)t * a.at + (long)py[nt] * L + px[nt];
  }

  f32x16 acc[M32][NT];
#pragma unroll
  for (int m = 0; m < M32; ++m)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][nt][r] = 0.f;

  const _Float16* wc = a.w + (long)cls * KSTEPS * M32 * 1024 + lane * 8;
  const unsigned* const xu = reinterpret_cast<const unsigned*>(a.x);
  for (int ci = 0; ci < 3; ++ci) {
    const unsigned* xc = xu + (long)ci * a.xc + 8 * h;
    // whole rows unrolled: the next k-steps' x / weight loads issue ahead of this one's MFMAs
#pragma unroll
    for (int dy = 0; dy < 13; ++dy) {
      const int ks = ci * 13 + dy;
      h8 ah[M32], al[M32];
#pragma unroll
      for (int m = 0; m < M32; ++m) {
        const _Float16* ap = wc + (long)(ks * M32 + m) * 1024;
        ah[m] = *reinterpret_cast<const h8*>(ap);
        al[m] = *reinterpret_cast<const h8*>(ap + 512);
      }
      h8 bh[NT], bl[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) gather8p(xc + xoff[nt] + dy * a.LP, bh[nt], bl[nt]);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int m = 0; m < M32; ++m) acc[m][nt] = mma3(ah[m], al[m], bh[nt], bl[nt], acc[m][nt]);
    }
  }
  // ---- epilogue (C/D map: col = lane & 31, row = (r&3) + 8(r>>2) + 4h) ----
  const float* rs = a.rscale + (long)cls * M32 * 32;
  const float* cb = a.cbias + (long)cls * M32 * 32;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    if (!ok[nt]) continue;
#pragma unroll
    for (int m = 0; m < M32; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
#if EXTDM_XP_EXP & 1
        if (acc[m][nt][r] == 12345.678f)
#endif
        if (row < a.Cout) {
          float v = acc[m][nt][r] * rs[row] + cb[row];
          if (a.add) v += a.add[aoff[nt] + (long)row * a.ac];
          a.out[ooff[nt] + (long)row * a.oc] = v;
        }
      }
  }
}

// TrajWarp's input maxpool(init_noise_conv(x)) (u12:913, 811): the 3 -> C (1,7,7) conv on
// f16x3 MFMA with the (1,2,2) max pool in the epilogue, so the full-resolution
// init_noise_conv output never reaches HBM (the composed init_conv no longer reads it).
// A wave owns two rows 2yp, 2yp+1 of one frame (n-tile nt = row, lane = column, L <= 32)
// and 4 m32 tiles (128 output channels); K = 3 ch x 4 row pairs x 8 columns (7 used):
// lane half h takes row 2*dyp + h of the pair. Pool: rows within the lane (nt), columns
// with the partner lane (lane ^ 1, same rows of the accumulator).
constexpr int NP_MW = 2;
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void noise_pool_x3_kernel(NoisePoolArgs a) {
  // m32 tiles per wave: 2 (64 rows), so accumulators + operands fit two waves per SIMD
  // (MW = 4 took 158 VGPRs + 128 AGPRs: one wave per SIMD, every k-step's L2 loads exposed)
  constexpr int MW = NP_MW;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lc = lane & 31, h = lane >> 5;
  const int L = a.L, Lh = L / 2;
  const int nrp = a.F * Lh;
  const int unit = blockIdx.x * 4 + wave;  // (row pair, m-quarter)
  const int nmq = (a.Cout + 32 * MW - 1) / (32 * MW);
  if (unit >= nrp * nmq) return;
  const int rp = unit / nmq, mq = unit - rp * nmq;
  const int f = rp / Lh, yp = rp - f * Lh;
  const int b = f / a.T, t = f - b * a.T;
  const bool ok = lc < L;
  // padded copy: row 2yp + nt + dy + 3, column lc + 3 (+ e)
  const unsigned* xf =
      reinterpret_cast<const unsigned*>(a.x) + (long)b * a.xb + (long)t * a.xt + (long)(2 * yp + 3) * a.LP + (ok ? lc : 0) + 3;

  f32x16 acc[MW][2];
#pragma unroll
  for (int m = 0; m < MW; ++m)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][nt][r] = 0.f;
  const _Float16* wq = a.w + (long)mq * MW * 1024 + lane * 8;
  const int M32 = (a.Cout + 31) / 32;
#pragma unroll 2
  for (int ks = 0; ks < 12; ++ks) {
    const int ci = ks / 4, dy = 2 * (ks % 4) + h;
    h8 ah[MW], al[MW];
#pragma unroll
    for (int m = 0; m < MW; ++m) {
      const _Float16* ap = wq + (long)(ks * M32 + m) * 1024;
      ah[m] = *reinterpret_cast<const h8*>(ap);
      al[m] = *reinterpret_cast<const h8*>(ap + 512);
    }
    h8 bh[2], bl[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) gather8p(xf + (long)ci * a.xc + (nt + dy) * a.LP, bh[nt], bl[nt]);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int m = 0; m < MW; ++m) acc[m][nt] = mma3(ah[m], al[m], bh[nt], bl[nt], acc[m][nt]);
  }
  float* of = a.out + (long)b * a.ob + (long)t * a.ot + (long)yp * Lh + (lc >> 1);
#pragma unroll
  for (int m = 0; m < MW; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (mq * MW + m) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      float v = fmaxf(acc[m][0][r], acc[m][1][r]);
      v = fmaxf(v, __shfl_xor(v, 1));
      if (ok && !(lc & 1) && row < a.Cout) of[(long)row * a.oc] = v * a.rscale[row] + a.bias[row];
    }
}

// A plain (1,7,7) conv of the 3-channel x (ada_u22 / wo_ref init_conv x-branch; the reference
// convolves cat(x, cond_fea) at once, ada_u22:1188-1190, wo_ref:911-921, and the cond_fea half is
// hoisted out of the step into `add`): noise_pool's k-loop (K = 3 ch x 4 row pairs x 8 columns, 7
// used; lane half h takes row 2 dyp + h) over 32-column tiles, no pool. A wave owns two output
// rows x 32 columns of one frame and 64 output channels; each store instruction writes two whole
// 128-B row segments (columns of one channel row, lanes 0-31 and 32-63 four channels apart).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void conv7c3_x3_kernel(NoisePoolArgs a) {
  constexpr int MW = 2;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lc = lane & 31, h = lane >> 5;
  const int L = a.L, nct = L / 32, Lh = L / 2;
  const int nmq = a.Cout / (32 * MW);
  const int unit = blockIdx.x * 4 + wave;  // (frame, row pair, column tile, m-group)
  if (unit >= a.F * Lh * nct * nmq) return;
  const int mq = unit % nmq, u2 = unit / nmq;
  const int ct = u2 % nct, rp = u2 / nct;
  const int f = rp / Lh, yp = rp - f * Lh;
  const int b = f / a.T, t = f - b * a.T;
  const int col = ct * 32 + lc;
  // padded copy (x at (6, 6)): output (y, c) reads rows y + 3 .. y + 9, columns c + 3 .. c + 10
  const unsigned* xf = reinterpret_cast<const unsigned*>(a.x) + (long)b * a.xb + (long)t * a.xt +
                       (long)(2 * yp + 3) * a.LP + col + 3;
  f32x16 acc[MW][2];
#pragma unroll
  for (int m = 0; m < MW; ++m)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][nt][r] = 0.f;
  const _Float16* wq = a.w + (long)mq * MW * 1024 + lane * 8;
  const int M32 = a.Cout / 32;
#pragma unroll 2
  for (int ks = 0; ks < 12; ++ks) {
    const int ci = ks / 4, dy = 2 * (ks % 4) + h;
    h8 ah[MW], al[MW];
#pragma unroll
    for (int m = 0; m < MW; ++m) {
      const _Float16* ap = wq + (long)(ks * M32 + m) * 1024;
      ah[m] = *reinterpret_cast<const h8*>(ap);
      al[m] = *reinterpret_cast<const h8*>(ap + 512);
    }
    h8 bh[2], bl[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) gather8p(xf + (long)ci * a.xc + (nt + dy) * a.LP, bh[nt], bl[nt]);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int m = 0; m < MW; ++m) acc[m][nt] = mma3(ah[m], al[m], bh[nt], bl[nt], acc[m][nt]);
  }
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const long pix = (long)(2 * yp + nt) * L + col;
    float* of = a.out + (long)b * a.ob + (long)t * a.ot + pix;
    const float* ad = a.add ? a.add + (long)b * a.ab + (long)t * a.at + pix : nullptr;
#pragma unroll
    for (int m = 0; m < MW; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (mq * MW + m) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        float v = acc[m][nt][r] * a.rscale[row];
        if (a.bias) v += a.bias[row];
        if (ad) v += ad[(long)row * a.ac];
        of[(long)row * a.oc] = v;
      }
  }
}

}  // namespace

int xpad_size(int L) { return (L + 16 + 7) & ~7; }

// x: the zero-padded copy (xpad_forward; LP = x.W, the latent L = out.H)
bool conv7c3_x3_forward(hipStream_t s, const View& out, const View& x, const void* w, const float* rscale,
                        const float* bias, const View* add) {
  const int L = out.H;
  if (x.C != 3 || x.W != x.H || x.W != xpad_size(L) || x.st != (long)x.W * x.H || out.W != L || L % 32 != 0 ||
      out.T != x.T || out.B != x.B || out.C % 64 != 0)
    return false;
  if (add && (add->B != out.B || add->C != out.C || add->T != out.T || add->H != L || add->W != L)) return false;
  NoisePoolArgs a{};
  a.x = x.p; a.xb = x.sb; a.xc = x.sc; a.xt = x.st; a.LP = x.W;
  a.T = x.T; a.L = L; a.F = x.B * x.T;
  a.out = out.p; a.ob = out.sb; a.oc = out.sc; a.ot = out.st; a.Cout = out.C;
  a.w = reinterpret_cast<const _Float16*>(w); a.rscale = rscale; a.bias = bias;
  if (add) { a.add = add->p; a.ab = add->sb; a.ac = add->sc; a.at = add->st; }
  const long units = (long)a.F * (L / 2) * (L / 32) * (out.C / 64);
  note_kernel("conv7c3_x3_kernel");
  hipLaunchKernelGGL(conv7c3_x3_kernel, dim3((unsigned)((units + 3) / 4)), dim3(256), 0, s, a);
  return true;
}

void xpad_forward(hipStream_t s, const View& xpad, const View& x) {
  const long n = (long)x.B * 3 * x.T * xpad.H * xpad.W;
  hipLaunchKernelGGL(xpad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x.p, x.sb, x.sc, x.st,
                     reinterpret_cast<unsigned*>(xpad.p), x.T, x.H, xpad.W, n, x3_range_ptr());
}

// x: the zero-padded copy (xpad_forward; LP = x.W, the latent L = out.H * 2)
bool noise_pool_x3_forward(hipStream_t s, const View& out, const View& x, const void* w, const float* rscale,
                           const float* bias) {
  const int L = out.H * 2;
  if (x.C != 3 || x.W != x.H || x.W != xpad_size(L) || x.st != (long)x.W * x.H || L > 32 || out.W != L / 2 ||
      out.T != x.T || out.B != x.B || out.C % 128 != 0)
    return false;
  NoisePoolArgs a{};
  a.x = x.p; a.xb = x.sb; a.xc = x.sc; a.xt = x.st; a.LP = x.W;
  a.T = x.T; a.L = L; a.F = x.B * x.T;
  a.out = out.p; a.ob = out.sb; a.oc = out.sc; a.ot = out.st; a.Cout = out.C;
  a.w = reinterpret_cast<const _Float16*>(w); a.rscale = rscale; a.bias = bias;
  const long units = (long)a.F * (L / 2) * ((out.C + 32 * NP_MW - 1) / (32 * NP_MW));
  hipLaunchKernelGGL(noise_pool_x3_kernel, dim3((unsigned)((units + 3) / 4)), dim3(256), 0, s, a);
  return true;
}

// x: the zero-padded copy (xpad_forward; LP = x.W, the latent L = out.H)
bool xpath_x3_forward(hipStream_t s, const View& out, const View& x, const void* w, const float* rscale,
                      const float* cbias, const View* add) {
  const int L = out.H;
  if (x.C != 3 || x.W != x.H || x.W != xpad_size(L) || x.st != (long)x.W * x.H || out.W != L || L < 7 ||
      out.C > 64 || out.T != x.T || out.B != x.B)
    return false;
  if (add && (add->B != out.B || add->C != out.C || add->T != out.T || add->H != L || add->W != L)) return false;
  XPathArgs a{};
  a.x = x.p; a.xb = x.sb; a.xc = x.sc; a.xt = x.st; a.LP = x.W;
  a.T = x.T; a.L = L; a.F = x.B * x.T;
  a.out = out.p; a.ob = out.sb; a.oc = out.sc; a.ot = out.st; a.Cout = out.C;
  a.w = reinterpret_cast<const _Float16*>(w); a.rscale = rscale; a.cbias = cbias;
  if (add) { a.add = add->p; a.ab = add->sb; a.ac = add->sc; a.at = add->st; }
  // FG = 32 frames (measured sweep at BAIR B = 64, layer 9: 4 / 8 / 16 / 32 / 64 / 112 frames ->
  // 610 / 515 / 450 / 442 / 432-444 / 502 us, class-major 546 us): smaller groups waste the corner
  // classes' tiles (one pixel per frame: 32 of a tile's 64 columns at FG = 32) and re-read every
  // class's weight slice per group; larger ones lose the L2 merge. EXTDM_XP_FG overrides (A/B;
  // 0 = the class-major order over all frames).
  static const int fgv = [] { const char* v = getenv("EXTDM_XP_FG"); return v ? atoi(v) : 32; }();
  a.FG = fgv > 0 ? std::min(fgv, a.F) : a.F;
  a.ngroups = (a.F + a.FG - 1) / a.FG;
  // EXTDM_XP_NT: pixels per wave = 32 NT (2: 64 px, 4: 128 px)
  static const int ntv = [] { const char* v = getenv("EXTDM_XP_NT"); return v && atoi(v) == 4 ? 4 : 2; }();
  const int TPX = 32 * ntv;
  auto prefix = [&](int fg, int* ts) {
    ts[0] = 0;
    for (int c = 0; c < 49; ++c) {
      const int cy = c / 7, cx = c % 7;
      const long n = (long)fg * (cy == 3 ? L - 6 : 1) * (cx == 3 ? L - 6 : 1);
      ts[c + 1] = ts[c] + (int)((n + TPX - 1) / TPX);
    }
  };
  prefix(a.FG, a.tile_start);
  prefix(a.F - (a.ngroups - 1) * a.FG, a.tile_last);
  a.gtiles = a.tile_start[49];
  const long total = (long)(a.ngroups - 1) * a.gtiles + a.tile_last[49];
  unsigned blocks = (unsigned)((total + 3) / 4);
  a.xcd = fgv > 0 && blocks >= 64;
  if (a.xcd) blocks = (blocks + 7) & ~7u;
  if (ntv == 4) {
    note_kernel("xpath_x3_kernel<%d, 4>", out.C > 32 ? 2 : 1);
    if (out.C > 32) hipLaunchKernelGGL((xpath_x3_kernel<2, 4>), dim3(blocks), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((xpath_x3_kernel<1, 4>), dim3(blocks), dim3(256), 0, s, a);
  } else {
    note_kernel("xpath_x3_kernel<%d, 2>", out.C > 32 ? 2 : 1);
    if (out.C > 32) hipLaunchKernelGGL((xpath_x3_kernel<2, 2>), dim3(blocks), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((xpath_x3_kernel<1, 2>), dim3(blocks), dim3(256), 0, s, a);
  }
  return true;
}

}  // namespace extdm
