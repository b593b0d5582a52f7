// Fused sampler step (one workgroup of 1024 threads per sample):
//   x0  = sqrt(1/acp[t]) x - sqrt(1/acp[t]-1) eps            (Diffusion.py:130-134)
//   s   = max(1, quantile(|x0|, 0.9))  — exact order statistics by an MSB-first
//         radix select on the fp32 bit patterns (|x0| >= 0 so bits are monotone),
//         then torch.quantile's linear interpolation            (Diffusion.py:150-163)
//   x0  = clamp(x0, -s, s) / s
//   DDPM: x = c1 x0 + c2 x + sigma * noise                     (Diffusion.py:136-177)
//   DDIM: x = sqrt(a_next) x0 + c eps + sigma * noise          (Diffusion.py:220-255)
// Coefficients come from a per-step table the host fills in fp32 with the
// reference's own expressions; the current step index lives in device memory so
// a captured hipGraph of one denoising step can be replayed for the whole loop.
// Noise is either injected (parity with the reference's host RNG stream) or a
// counter-based Philox4x32-10 + Box-Muller stream keyed by (seed, global sample
// index) with counter (element, step, round): results do not depend on how the
// batch is sharded over ranks.
#include "kernels.h"

// EXTDM_SAMPLER_DEBUG (diagnostic builds only): the multi-workgroup update records every chunk
// workgroup's threshold, thresh_out[(step B + b) nch + chunk]
#ifndef EXTDM_SAMPLER_DEBUG
#define EXTDM_SAMPLER_DEBUG 0
#endif

namespace extdm {

namespace {

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const unsigned lo0 = c.x * 0xD2511F53u, hi0 = __umulhi(c.x, 0xD2511F53u);
    const unsigned lo1 = c.z * 0xCD9E8D57u, hi1 = __umulhi(c.z, 0xCD9E8D57u);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ float philox_normal(uint64_t seed, int sample, int round, int step, long e) {
  const uint4 ctr = make_uint4((unsigned)(e >> 2), (unsigned)step, (unsigned)round, 0x5EEDu);
  const uint2 key = make_uint2((unsigned)seed ^ (unsigned)sample * 0x85EBCA6Bu, (unsigned)(seed >> 32) + (unsigned)sample);
  const uint4 r = philox4x32_10(ctr, key);
  const int lane = (int)(e & 3);
  const unsigned a = (lane < 2) ? r.x : r.z;
  const unsigned b2 = (lane < 2) ? r.y : r.w;
  const float u1 = ((float)a + 1.0f) * 2.3283064365386963e-10f;  // (0, 1]
  const float u2 = (float)b2 * 2.3283064365386963e-10f;
  const float rad = sqrtf(-2.0f * logf(u1));
  float sn, cs;
  sincosf(6.283185307179586f * u2, &sn, &cs);
  return (lane & 1) ? rad * sn : rad * cs;
}

// the four normals of one Philox block (e0 % 4 == 0): exactly philox_normal(e0 + i), i = 0..3 —
// one Philox call and two Box-Muller pairs instead of four calls and four pairs
__device__ __forceinline__ void philox_normal4(uint64_t seed, int sample, int round, int step, long e0, float z[4]) {
  const uint4 ctr = make_uint4((unsigned)(e0 >> 2), (unsigned)step, (unsigned)round, 0x5EEDu);
  const uint2 key = make_uint2((unsigned)seed ^ (unsigned)sample * 0x85EBCA6Bu, (unsigned)(seed >> 32) + (unsigned)sample);
  const uint4 r = philox4x32_10(ctr, key);
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const unsigned a = p ? r.z : r.x, b2 = p ? r.w : r.y;
    const float u1 = ((float)a + 1.0f) * 2.3283064365386963e-10f;  // (0, 1]
    const float u2 = (float)b2 * 2.3283064365386963e-10f;
    const float rad = sqrtf(-2.0f * logf(u1));
    float sn, cs;
    sincosf(6.283185307179586f * u2, &sn, &cs);
    z[2 * p] = rad * cs;
    z[2 * p + 1] = rad * sn;
  }
}

// |x0| bit pattern of element e (recomputed from x and eps on every pass: the
// sample's 2 x 4n bytes stay L2-resident, so nothing is held in registers).
__device__ __forceinline__ unsigned x0_bits(const float* xb, const float* eb, const StepCoef& c, int e) {
  return __float_as_uint(fabsf(c.sra * xb[e] - c.srm1 * eb[e]));
}

__device__ float radix_select(const float* xb, const float* eb, const StepCoef& c, int n, int rank,
                              unsigned* hist, unsigned* sh) {
  unsigned prefix = 0, mask = 0;
  int r = rank;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int e = threadIdx.x; e < n; e += blockDim.x) {
      const unsigned u = x0_bits(xb, eb, c, e);
      if ((u & mask) == prefix) atomicAdd(&hist[(u >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      // wave-parallel scan of the 256 bins: lane owns bins 4l..4l+3
      const unsigned h0 = hist[4 * threadIdx.x], h1 = hist[4 * threadIdx.x + 1];
      const unsigned h2 = hist[4 * threadIdx.x + 2], h3 = hist[4 * threadIdx.x + 3];
      const unsigned tot = h0 + h1 + h2 + h3;
      unsigned incl = tot;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned v = __shfl_up(incl, o);
        if ((int)threadIdx.x >= o) incl += v;
      }
      const unsigned excl = incl - tot;
      const unsigned ur = (unsigned)r;
      if (ur >= excl && ur < incl) {
        unsigned cum = excl;
        int d = 4 * threadIdx.x;
        if (ur >= cum + h0) { cum += h0; ++d;
          if (ur >= cum + h1) { cum += h1; ++d;
            if (ur >= cum + h2) { cum += h2; ++d; } } }
        sh[0] = (unsigned)d;
        sh[1] = ur - cum;
      }
    }
    __syncthreads();
    prefix |= sh[0] << shift;
    mask |= 255u << shift;
    r = (int)sh[1];
    __syncthreads();
  }
  return __uint_as_float(prefix);
}

__global__ __launch_bounds__(1024) void sampler_step_kernel(float* x, const float* eps, int n,
                                                            const StepCoef* coefs, const int* step_ctr,
                                                            const float* noise, int B, uint64_t seed,
                                                            int sample_base, int round, int k_lo, int k_hi,
                                                            float q_w, float* thresh_out) {
  __shared__ unsigned hist[256];
  __shared__ unsigned sh[2];
  const int b = blockIdx.x;
  const int step = *step_ctr;
  const StepCoef c = coefs[step];
  float* xb = x + (long)b * n;
  const float* eb = eps + (long)b * n;
  const float vlo = radix_select(xb, eb, c, n, k_lo, hist, sh);
  const float vhi = k_hi == k_lo ? vlo : radix_select(xb, eb, c, n, k_hi, hist, sh);
  // torch lerp (CPU): w < 0.5 ? a + w (b - a) : b - (b - a)(1 - w)
  float s = q_w < 0.5f ? vlo + q_w * (vhi - vlo) : vhi - (vhi - vlo) * (1.f - q_w);
  if (s < 1.f) s = 1.f;
  if (thresh_out && threadIdx.x == 0) thresh_out[(size_t)step * B + b] = s;
  const float* nb = noise ? noise + ((long)step * B + b) * n : nullptr;
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    const float xv = xb[e], ev = eb[e];
    const float x0 = c.sra * xv - c.srm1 * ev;
    const float xc = fminf(fmaxf(x0, -s), s) / s;
    float out;
    if (c.kind == 0) out = c.c1 * xc + c.c2 * xv;
    else out = xc * c.c1 + c.c2 * ev;
    if (c.use_noise) {
      const float z = nb ? nb[e] : philox_normal(seed, sample_base + b, round, step, e);
      out = out + c.sigma * z;
    }
    xb[e] = out;
  }
}

// ---- multi-workgroup form: the same step over (chunk, sample) workgroups ----
// The one-workgroup-per-sample kernel above runs 4 radix passes x up to 2 selections over the whole
// sample in one workgroup: 4 of 256 CUs busy at UCF's B = 4 (2.6 ms per step) and 64 at BAIR's 64
// (168 us). Here every pass is a launch over SCH-element chunks x samples. Each workgroup counts its
// chunk's |x0| bytes (filtered by the prefix chosen so far) into LDS bins and STORES the chunk's
// 256-bin histogram to its own slot hist[pass][b][chunk][sel][256] — no global atomics, no zeroing:
// every slot is overwritten whole by one workgroup on every step. The next launch's workgroups sum
// the sample's chunk histograms of the previous pass in a fixed order (integer sums: exact, so the
// order statistics are those of the one-workgroup kernel whatever the workgroup order and placement)
// and take the next radix digit. Chunk 0's workgroup of pass p stores the (prefix, mask, rank) state
// after p digits for pass p + 1. The only cross-workgroup hand-offs are plain stores read by plain
// loads in a LATER launch of the same stream — the kernel-boundary visibility every other producer /
// consumer pair of the forward relies on. The final launch derives the two order
// statistics and the threshold and updates its chunk; a one-workgroup launch then writes the next
// step's t and increments the step counter (sampler_advance_kernel).
constexpr int SCH = 4096;       // elements per workgroup
constexpr int SNT = 256;        // threads per workgroup

struct SelLayout {
  int B, nch;
  __host__ __device__ size_t hist_words() const { return (size_t)4 * B * nch * 2 * 256; }
  // histogram of (pass, sample, chunk, selection)
  __host__ __device__ size_t hist(int p, int b, int ch, int sl) const {
    return (((size_t)p * B + b) * nch + ch) * 512 + (size_t)sl * 256;
  }
  // (prefix, mask, rank, -) after `p` digits (p = 1..3) of (sample, selection)
  __host__ __device__ size_t state(int p, int b, int sl) const {
    return hist_words() + (((size_t)p * B + b) * 2 + sl) * 4;
  }
  __host__ __device__ size_t words() const { return hist_words() + (size_t)4 * B * 2 * 4; }
};

// One radix digit of selection `sl` of sample b: the sum over the sample's chunks of pass `p`'s
// histograms (fixed chunk order; lane l owns bins 4l..4l+3), then the bin holding residual rank
// `rank`. Called by one whole wave; returns wave-uniform (digit, residual rank).
__device__ void next_digit(const unsigned* ws, const SelLayout& L, int p, int b, int sl, unsigned rank,
                           unsigned& digit, unsigned& nrank) {
  const int l = threadIdx.x & 63;
  uint4 s = make_uint4(0u, 0u, 0u, 0u);
  for (int ch = 0; ch < L.nch; ++ch) {
    const uint4 v = *reinterpret_cast<const uint4*>(ws + L.hist(p, b, ch, sl) + 4 * l);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  const unsigned tot = s.x + s.y + s.z + s.w;
  unsigned incl = tot;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned v = __shfl_up(incl, o);
    if (l >= o) incl += v;
  }
  const unsigned excl = incl - tot;
  const bool mine = rank >= excl && rank < incl;
  unsigned d = 4 * l, cum = excl;
  if (rank >= cum + s.x) { cum += s.x; ++d;
    if (rank >= cum + s.y) { cum += s.y; ++d;
      if (rank >= cum + s.z) { cum += s.z; ++d; } } }
  const unsigned long long bal = __ballot(mine);
  const int src = bal ? __ffsll((long long)bal) - 1 : 0;
  digit = __shfl(d, src);
  nrank = __shfl(rank - cum, src);
}

// (prefix, mask, residual rank) of selection sl after PASS digits: from the stored state after
// PASS - 1 digits (written by the previous launch's chunk-0 workgroup) and pass PASS - 1's chunk
// histograms. Whole wave; chunk 0's lane 0 stores it for the next launch when `store`.
template <int PASS>
__device__ void sel_state(unsigned* ws, const SelLayout& L, int b, int sl, unsigned rank0, bool store,
                          unsigned& prefix, unsigned& mask, unsigned& rank) {
  if (PASS == 0) { prefix = 0; mask = 0; rank = rank0; return; }
  unsigned pp = 0, pm = 0, pr = rank0;
  if (PASS > 1) {
    const uint4 st = *reinterpret_cast<const uint4*>(ws + L.state(PASS - 1, b, sl));
    pp = st.x; pm = st.y; pr = st.z;
  }
  unsigned d, nr;
  next_digit(ws, L, PASS - 1, b, sl, pr, d, nr);
  constexpr int shift = 24 - 8 * (PASS - 1);
  prefix = pp | (d << shift);
  mask = pm | (255u << shift);
  rank = nr;
  if (store && PASS < 4 && (threadIdx.x & 63) == 0)
    *reinterpret_cast<uint4*>(ws + L.state(PASS, b, sl)) = make_uint4(prefix, mask, rank, 0u);
}

template <int PASS>
__global__ __launch_bounds__(SNT) void radix_count_kernel(const float* x, const float* eps, int n,
                                                          const StepCoef* coefs, const int* step_ctr,
                                                          unsigned* ws, int k_lo, int k_hi) {
  __shared__ unsigned lh[2][256];
  __shared__ unsigned st[2][2];  // [sel][prefix, mask]
  const SelLayout L{(int)gridDim.y, (int)gridDim.x};
  const int b = blockIdx.y, ch = blockIdx.x;
  const int step = *step_ctr;
  const StepCoef c = coefs[step];
  const int nsel = k_hi == k_lo ? 1 : 2;
  for (int i = threadIdx.x; i < 512; i += SNT) lh[i >> 8][i & 255] = 0;
  if (threadIdx.x < 64 * nsel) {
    const int sl = threadIdx.x >> 6;
    unsigned pf, mk, rk;
    sel_state<PASS>(ws, L, b, sl, (unsigned)(sl ? k_hi : k_lo), ch == 0, pf, mk, rk);
    if ((threadIdx.x & 63) == 0) { st[sl][0] = pf; st[sl][1] = mk; }
  }
  __syncthreads();
  const unsigned p0 = st[0][0], m0 = st[0][1];
  const unsigned p1 = nsel > 1 ? st[1][0] : 0, m1 = nsel > 1 ? st[1][1] : 0;
  constexpr int shift = 24 - 8 * PASS;
  const float* xb = x + (long)b * n;
  const float* eb = eps + (long)b * n;
  const int e0 = ch * SCH, e1 = min(n, e0 + SCH);
  for (int e = e0 + threadIdx.x; e < e1; e += SNT) {
    const unsigned u = x0_bits(xb, eb, c, e);
    if ((u & m0) == p0) atomicAdd(&lh[0][(u >> shift) & 255u], 1u);
    if (nsel > 1 && (u & m1) == p1) atomicAdd(&lh[1][(u >> shift) & 255u], 1u);
  }
  __syncthreads();
  // the chunk's histograms, stored whole (zero bins included): 16 B per thread
  for (int i = 4 * threadIdx.x; i < 256 * nsel; i += 4 * SNT) {
    const int sl = i >> 8, j = i & 255;
    *reinterpret_cast<uint4*>(ws + L.hist(PASS, b, ch, sl) + j) =
        make_uint4(lh[sl][j], lh[sl][j + 1], lh[sl][j + 2], lh[sl][j + 3]);
  }
}

__global__ __launch_bounds__(SNT) void sampler_final_kernel(float* x, const float* eps, int n, const StepCoef* coefs,
                                                            const int* step_ctr, const float* noise, int B,
                                                            uint64_t seed, int sample_base, int round, int k_lo,
                                                            int k_hi, float q_w, float* thresh_out, unsigned* ws) {
  __shared__ float vs[2];
  const SelLayout L{(int)gridDim.y, (int)gridDim.x};
  const int b = blockIdx.y;
  const int step = *step_ctr;
  const StepCoef c = coefs[step];
  const int nsel = k_hi == k_lo ? 1 : 2;
  if (threadIdx.x < 64 * nsel) {
    const int sl = threadIdx.x >> 6;
    unsigned pf, mk, rk;
    sel_state<4>(ws, L, b, sl, (unsigned)(sl ? k_hi : k_lo), false, pf, mk, rk);
    if ((threadIdx.x & 63) == 0) vs[sl] = __uint_as_float(pf);
  }
  __syncthreads();
  const float vlo = vs[0], vhi = nsel > 1 ? vs[1] : vs[0];
  // torch lerp (CPU): w < 0.5 ? a + w (b - a) : b - (b - a)(1 - w)
  float s = q_w < 0.5f ? vlo + q_w * (vhi - vlo) : vhi - (vhi - vlo) * (1.f - q_w);
  if (s < 1.f) s = 1.f;
#if EXTDM_SAMPLER_DEBUG
  if (thresh_out && threadIdx.x == 0) thresh_out[((size_t)step * B + b) * gridDim.x + blockIdx.x] = s;
#else
  if (thresh_out && blockIdx.x == 0 && threadIdx.x == 0) thresh_out[(size_t)step * B + b] = s;
#endif
  float* xb = x + (long)b * n;
  const float* eb = eps + (long)b * n;
  const float* nb = noise ? noise + ((long)step * B + b) * n : nullptr;
  const int e0 = blockIdx.x * SCH, e1 = min(n, e0 + SCH);
  auto update = [&](float xv, float ev, float z) __attribute__((always_inline)) {
    const float x0 = c.sra * xv - c.srm1 * ev;
    const float xc = fminf(fmaxf(x0, -s), s) / s;
    float out;
    if (c.kind == 0) out = c.c1 * xc + c.c2 * xv;
    else out = xc * c.c1 + c.c2 * ev;
    if (c.use_noise) out = out + c.sigma * z;
    return out;
  };
  if ((n & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(eps) & 15) == 0 &&
      (!nb || (reinterpret_cast<uintptr_t>(noise) & 15) == 0)) {
    // four consecutive elements per thread (16-B loads and stores; one Philox block per four)
    for (int e = e0 + 4 * threadIdx.x; e < e1; e += 4 * SNT) {
      const float4 x4 = *reinterpret_cast<const float4*>(xb + e), e4 = *reinterpret_cast<const float4*>(eb + e);
      float z[4] = {0.f, 0.f, 0.f, 0.f};
      if (c.use_noise) {
        if (nb) {
          const float4 n4 = *reinterpret_cast<const float4*>(nb + e);
          z[0] = n4.x; z[1] = n4.y; z[2] = n4.z; z[3] = n4.w;
        } else {
          philox_normal4(seed, sample_base + b, round, step, e, z);
        }
      }
      float4 o;
      o.x = update(x4.x, e4.x, z[0]);
      o.y = update(x4.y, e4.y, z[1]);
      o.z = update(x4.z, e4.z, z[2]);
      o.w = update(x4.w, e4.w, z[3]);
      *reinterpret_cast<float4*>(xb + e) = o;
    }
  } else {
    for (int e = e0 + threadIdx.x; e < e1; e += SNT) {
      const float z = c.use_noise ? (nb ? nb[e] : philox_normal(seed, sample_base + b, round, step, e)) : 0.f;
      xb[e] = update(xb[e], eb[e], z);
    }
  }
}

// t and the step counter for the next step (one workgroup, after the update launch: every
// workgroup of this step has read the counter before it changes).
__global__ __launch_bounds__(256) void sampler_advance_kernel(int* step_ctr, const StepCoef* coefs, int* t_next, int B,
                                                              int nsteps) {
  const int step = *step_ctr;
  if (step + 1 < nsteps)
    for (int i = threadIdx.x; i < B; i += 256) t_next[i] = coefs[step + 1].t;
  __syncthreads();  // every thread has read the counter
  if (threadIdx.x == 0) *step_ctr = step + 1;
}

__global__ void fill_normal_kernel(float* x, int n, uint64_t seed, int sample_base, int round, int stream_id) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (e >= n) return;
  x[(long)b * n + e] = philox_normal(seed, sample_base + b, round, stream_id, e);
}

__global__ void set_t_kernel(int* t_batch, int B, const StepCoef* coefs, const int* step_ctr) {
  const int i = threadIdx.x;
  if (i < B) t_batch[i] = coefs[*step_ctr].t;
}
__global__ void incr_kernel(int* c) { c[0] += 1; }
__global__ void t_to_int_kernel(const int64_t* t, int* tb, int B) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < B) tb[i] = (int)t[i];
}

// ---- LFAE decoder without occlusion: prediction == deformed ----
__device__ __forceinline__ void lin_idx(int o, int in, int out, int& i0, int& i1, float& l0, float& l1) {
  const float scale = (float)in / (float)out;
  float src = scale * ((float)o + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = src - (float)i0;
  l0 = 1.f - l1;
}

__global__ __launch_bounds__(256) void warp_kernel(float* out, const float* src, const float* flow, int C, int T,
                                                   int S, int fh, int fw, long osb, long osc, long ost) {
  const int pix = blockIdx.x * 256 + threadIdx.x;
  const int t = blockIdx.y, b = blockIdx.z;
  if (pix >= S * S) return;
  const int y = pix / S, xq = pix % S;
  // bilinear resize of the flow (Generator.deform_input, generator.py:63-71)
  int y0, y1, x0, x1;
  float ly0, ly1, lx0, lx1;
  lin_idx(y, fh, S, y0, y1, ly0, ly1);
  lin_idx(xq, fw, S, x0, x1, lx0, lx1);
  const float* fx = flow + (((long)b * 2 + 0) * T + t) * fh * fw;
  const float* fy = flow + (((long)b * 2 + 1) * T + t) * fh * fw;
  const float gx = ly0 * (lx0 * fx[y0 * fw + x0] + lx1 * fx[y0 * fw + x1]) +
                   ly1 * (lx0 * fx[y1 * fw + x0] + lx1 * fx[y1 * fw + x1]);
  const float gy = ly0 * (lx0 * fy[y0 * fw + x0] + lx1 * fy[y0 * fw + x1]) +
                   ly1 * (lx0 * fy[y1 * fw + x0] + lx1 * fy[y1 * fw + x1]);
  // grid_sample bilinear, zeros padding, align_corners=True
  const float sf = (float)(S - 1) / 2.0f;
  const float ix = (gx + 1.f) * sf, iy = (gy + 1.f) * sf;
  const float ixw = floorf(ix), iyn = floorf(iy);
  const float w = ix - ixw, e = 1.f - w;
  const float nn = iy - iyn, ss = 1.f - nn;
  const int xw = (int)ixw, yn = (int)iyn;
  const float nw = ss * e, ne = ss * w, sw = nn * e, se = nn * w;
  const bool vxw = xw >= 0 && xw < S, vxe = xw + 1 >= 0 && xw + 1 < S;
  const bool vyn = yn >= 0 && yn < S, vys = yn + 1 >= 0 && yn + 1 < S;
  for (int c = 0; c < C; ++c) {
    const float* p = src + ((long)b * C + c) * S * S;
    const float vnw = (vxw && vyn) ? p[yn * S + xw] : 0.f;
    const float vne = (vxe && vyn) ? p[yn * S + xw + 1] : 0.f;
    const float vsw = (vxw && vys) ? p[(yn + 1) * S + xw] : 0.f;
    const float vse = (vxe && vys) ? p[(yn + 1) * S + xw + 1] : 0.f;
    out[(long)b * osb + (long)c * osc + (long)t * ost + pix] = vnw * nw + vne * ne + vsw * sw + vse * se;
  }
}

}  // namespace

void sampler_step(hipStream_t s, float* x, const float* eps, int B, int n, const StepCoef* coefs,
                  const int* step_ctr, const float* noise, uint64_t seed, int sample_base, int round, int k_lo,
                  int k_hi, float q_w, float* thresh_out) {
  hipLaunchKernelGGL(sampler_step_kernel, dim3(B), dim3(1024), 0, s, x, eps, n, coefs, step_ctr, noise, B, seed,
                     sample_base, round, k_lo, k_hi, q_w, thresh_out);
}

size_t sampler_sel_bytes(int B, int n) {
  return SelLayout{B, (n + SCH - 1) / SCH}.words() * sizeof(unsigned);
}

void sampler_step_mw(hipStream_t s, float* x, const float* eps, int B, int n, const StepCoef* coefs, int* step_ctr,
                     const float* noise, uint64_t seed, int sample_base, int round, int k_lo, int k_hi, float q_w,
                     float* thresh_out, unsigned* ws, int* t_next, int nsteps) {
  const dim3 grid((n + SCH - 1) / SCH, B);
  hipLaunchKernelGGL(radix_count_kernel<0>, grid, dim3(SNT), 0, s, x, eps, n, coefs, step_ctr, ws, k_lo, k_hi);
  hipLaunchKernelGGL(radix_count_kernel<1>, grid, dim3(SNT), 0, s, x, eps, n, coefs, step_ctr, ws, k_lo, k_hi);
  hipLaunchKernelGGL(radix_count_kernel<2>, grid, dim3(SNT), 0, s, x, eps, n, coefs, step_ctr, ws, k_lo, k_hi);
  hipLaunchKernelGGL(radix_count_kernel<3>, grid, dim3(SNT), 0, s, x, eps, n, coefs, step_ctr, ws, k_lo, k_hi);
  hipLaunchKernelGGL(sampler_final_kernel, grid, dim3(SNT), 0, s, x, eps, n, coefs, step_ctr, noise, B, seed,
                     sample_base, round, k_lo, k_hi, q_w, thresh_out, ws);
  if (t_next) hipLaunchKernelGGL(sampler_advance_kernel, dim3(1), dim3(256), 0, s, step_ctr, coefs, t_next, B, nsteps);
}

void fill_normal(hipStream_t s, float* x, int B, int n, uint64_t seed, int sample_base, int round, int stream_id) {
  hipLaunchKernelGGL(fill_normal_kernel, dim3((n + 255) / 256, B), dim3(256), 0, s, x, n, seed, sample_base, round,
                     stream_id);
}

void set_t_from_step(hipStream_t s, int* t_batch, int B, const StepCoef* coefs, const int* step_ctr) {
  hipLaunchKernelGGL(set_t_kernel, dim3(1), dim3(1024), 0, s, t_batch, B, coefs, step_ctr);
}
void incr_counter(hipStream_t s, int* ctr) { hipLaunchKernelGGL(incr_kernel, dim3(1), dim3(1), 0, s, ctr); }
void t_to_int(hipStream_t s, const int64_t* t, int* t_batch, int B) {
  hipLaunchKernelGGL(t_to_int_kernel, dim3((B + 255) / 256), dim3(256), 0, s, t, t_batch, B);
}

void warp_frames(hipStream_t s, float* out, const float* src, const float* flow, int B, int C, int T, int S, int fh,
                 int fw, long out_sb, long out_sc, long out_st) {
  hipLaunchKernelGGL(warp_kernel, dim3((S * S + 255) / 256, T, B), dim3(256), 0, s, out, src, flow, C, T, S, fh, fw,
                     out_sb, out_sc, out_st);
}

}  // namespace extdm
