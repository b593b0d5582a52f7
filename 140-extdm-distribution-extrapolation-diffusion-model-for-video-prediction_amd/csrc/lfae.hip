// LFAE encoder kernels: the memory-bound / per-region pieces of
// RegionPredictor, BGMotionPredictor and PixelwiseFlowPredictor. Their
// convolutions (Hourglass down/up blocks, the 7x7 heads) run on the conv kernels
// with BatchNorm(eval)+ReLU folded into the epilogues; what is here:
//   aa_down        AntiAliasInterpolation2d: depthwise Gaussian + stride (util.py:224-264)
//   region_stats   spatial softmax(logits / T) -> shift, covariance, 2x2 SVD (sgesdd
//                  sign convention), affine = U sqrt(S)   (region_predictor.py:62-150)
//   bg_head        mean over space + Linear -> 3x3 background transform
//                  (bg_motion_predictor.py:47-64)
//   sparse_motion  per (image, region, pixel): region / background motion, the
//                  Gaussian heatmap difference and the deformed source, written
//                  straight into the Hourglass input layout (pixelwise_flow_predictor.py:45-104)
//   flow_combine   softmax over the R+1 mask logits, flow = sum_k mask_k motion_k (:135-143)
#include "kernels.h"

namespace extdm {

namespace {

// make_coordinate_grid (util.py:50-66): 2 * (i / (n - 1)) - 1 in fp32
__device__ __forceinline__ float coord(int i, int n) { return 2.f * ((float)i / (float)(n - 1)) - 1.f; }

__device__ __forceinline__ float fsign(float a, float b) { return b >= 0.f ? fabsf(a) : -fabsf(a); }

// LAPACK slasv2 (2x2 upper-triangular SVD); returns the left rotation (csl, snl)
// and the signed singular values.
__device__ void slasv2(float F, float G, float H, float& ssmin, float& ssmax, float& snl, float& csl) {
  float ft = F, fa = fabsf(ft), ht = H, ha = fabsf(H);
  int pmax = 1;
  const bool swap = ha > fa;
  if (swap) {
    pmax = 3;
    float t = ft; ft = ht; ht = t;
    t = fa; fa = ha; ha = t;
  }
  const float gt = G, ga = fabsf(gt);
  float clt, crt, slt, srt;
  const float eps = 5.9604645e-08f;
  if (ga == 0.f) {
    ssmin = ha; ssmax = fa; clt = 1.f; crt = 1.f; slt = 0.f; srt = 0.f;
  } else {
    bool gasmal = true;
    if (ga > fa) {
      pmax = 2;
      if (fa / ga < eps) {
        gasmal = false;
        ssmax = ga;
        ssmin = ha > 1.f ? fa / (ga / ha) : (fa / ga) * ha;
        clt = 1.f; slt = ht / gt; srt = 1.f; crt = ft / gt;
      }
    }
    if (gasmal) {
      const float d = fa - ha;
      float l = d == fa ? 1.f : d / fa;
      const float m = gt / ft;
      float t = 2.f - l;
      const float mm = m * m, tt = t * t;
      const float s = sqrtf(tt + mm);
      const float r = l == 0.f ? fabsf(m) : sqrtf(l * l + mm);
      const float a = 0.5f * (s + r);
      ssmin = ha / a;
      ssmax = fa * a;
      if (mm == 0.f) {
        t = l == 0.f ? fsign(2.f, ft) * fsign(1.f, gt) : gt / fsign(d, ft) + m / t;
      } else {
        t = (m / (s + t) + m / (r + l)) * (1.f + a);
      }
      l = sqrtf(t * t + 4.f);
      crt = 2.f / l;
      srt = t / l;
      clt = (crt + srt * m) / a;
      slt = (ht / ft) * srt / a;
    }
  }
  float csr, snr;
  if (swap) { csl = srt; snl = crt; csr = slt; snr = clt; }
  else { csl = clt; snl = slt; csr = crt; snr = srt; }
  float tsign;
  if (pmax == 1) tsign = fsign(1.f, csr) * fsign(1.f, csl) * fsign(1.f, F);
  else if (pmax == 2) tsign = fsign(1.f, snr) * fsign(1.f, csl) * fsign(1.f, G);
  else tsign = fsign(1.f, snr) * fsign(1.f, snl) * fsign(1.f, H);
  ssmax = fsign(ssmax, tsign);
  ssmin = fsign(ssmin, tsign * fsign(1.f, F) * fsign(1.f, H));
}

// torch.svd of a 2x2 matrix m (row-major) as LAPACK sgesdd computes it on CPU:
// slarfg bidiagonalisation, sbdsqr (split test + slasv2, sign fix, sort), sormbr.
__device__ void svd2(const float m[4], float u[4], float sv[2]) {
  const float a = m[0], b = m[2], c = m[1], d = m[3];  // column 1 = (a, b), column 2 = (c, d)
  float tau = 0.f, beta = a, v = 0.f;
  if (b != 0.f) {
    beta = -fsign(sqrtf(a * a + b * b), a);
    tau = (beta - a) / beta;
    v = b * (1.f / (a - beta));
  }
  const float w = c + v * d;
  const float c2 = c - tau * w, d2 = d - tau * v * w;
  const float tol = 10.f * 5.9604645e-08f;
  float sminoa = fabsf(beta);
  if (sminoa != 0.f) {
    const float mu = fabsf(d2) * (sminoa / (sminoa + fabsf(c2)));
    sminoa = fminf(sminoa, mu);
  }
  sminoa = sminoa / sqrtf(2.f);
  float ub[4], s0, s1;
  if (fabsf(c2) <= tol * sminoa) {
    ub[0] = 1.f; ub[1] = 0.f; ub[2] = 0.f; ub[3] = 1.f;
    s0 = fabsf(beta); s1 = fabsf(d2);
  } else {
    float smn, smx, snl, csl;
    slasv2(beta, c2, d2, smn, smx, snl, csl);
    ub[0] = csl; ub[1] = -snl; ub[2] = snl; ub[3] = csl;
    s0 = fabsf(smx); s1 = fabsf(smn);
  }
  if (s1 > s0) {
    float t = ub[0]; ub[0] = ub[1]; ub[1] = t;
    t = ub[2]; ub[2] = ub[3]; ub[3] = t;
    t = s0; s0 = s1; s1 = t;
  }
  // U = H ub, H = I - tau [1 v]^T [1 v]
  const float h00 = 1.f - tau, h01 = -tau * v, h11 = 1.f - tau * v * v;
  u[0] = h00 * ub[0] + h01 * ub[2];
  u[1] = h00 * ub[1] + h01 * ub[3];
  u[2] = h01 * ub[0] + h11 * ub[2];
  u[3] = h01 * ub[1] + h11 * ub[3];
  sv[0] = s0;
  sv[1] = s1;
}

__global__ __launch_bounds__(256) void aa_down_kernel(float* out, const float* in, const float* w, int C, int H,
                                                      int W, int k, int ka, int step, int Ho, int Wo, long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % Wo);
  long r = i / Wo;
  const int y = (int)(r % Ho);
  r /= Ho;
  const int c = (int)(r % C);
  const float* p = in + r * (long)H * W;
  const float* wk = w + (long)c * k * k;
  float acc = 0.f;
  for (int dy = 0; dy < k; ++dy) {
    const int iy = y * step + dy - ka;
    if (iy < 0 || iy >= H) continue;
    for (int dx = 0; dx < k; ++dx) {
      const int ix = x * step + dx - ka;
      if (ix < 0 || ix >= W) continue;
      acc += wk[dy * k + dx] * p[(long)iy * W + ix];
    }
  }
  out[i] = acc;
}

// One block per (image, region): softmax over the h*w logits / temperature, then
// the first and second moments over the coordinate grid and the 2x2 SVD.
__global__ __launch_bounds__(256) void region_stats_kernel(const float* logits, int h, int w, float temp,
                                                           float* heat, float* shift, float* covar, float* affine,
                                                           float* uout, float* svout) {
  __shared__ double sh[6][8];
  const long base = (long)blockIdx.x * h * w;
  const int n = h * w, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // max of logits / T (softmax of x / T, F.softmax(region / temperature))
  float mx = -INFINITY;
  for (int i = tid; i < n; i += 256) mx = fmaxf(mx, logits[base + i] / temp);
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  __shared__ float smx[4];
  if (lane == 0) smx[wave] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(smx[0], smx[1]), fmaxf(smx[2], smx[3]));
  double se = 0.0;
  for (int i = tid; i < n; i += 256) se += (double)expf(logits[base + i] / temp - mx);
  for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o);
  __shared__ double ssum[4];
  if (lane == 0) ssum[wave] = se;
  __syncthreads();
  const float sum = (float)(ssum[0] + ssum[1] + ssum[2] + ssum[3]);
  // moments: E[g], then E[(g - m)(g - m)^T] (two passes, as region2affine)
  double mxs = 0.0, mys = 0.0;
  for (int i = tid; i < n; i += 256) {
    const float p = expf(logits[base + i] / temp - mx) / sum;
    if (heat) heat[base + i] = p;
    const float gx = coord(i % w, w), gy = coord(i / w, h);
    mxs += (double)(p * gx);
    mys += (double)(p * gy);
  }
  for (int o = 32; o > 0; o >>= 1) { mxs += __shfl_xor(mxs, o); mys += __shfl_xor(mys, o); }
  if (lane == 0) { sh[0][wave] = mxs; sh[1][wave] = mys; }
  __syncthreads();
  const float m0 = (float)(sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3]);
  const float m1 = (float)(sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3]);
  double cxx = 0.0, cxy = 0.0, cyy = 0.0;
  for (int i = tid; i < n; i += 256) {
    const float p = expf(logits[base + i] / temp - mx) / sum;
    const float dx = coord(i % w, w) - m0, dy = coord(i / w, h) - m1;
    cxx += (double)((dx * dx) * p);
    cxy += (double)((dx * dy) * p);
    cyy += (double)((dy * dy) * p);
  }
  for (int o = 32; o > 0; o >>= 1) {
    cxx += __shfl_xor(cxx, o);
    cxy += __shfl_xor(cxy, o);
    cyy += __shfl_xor(cyy, o);
  }
  __syncthreads();
  if (lane == 0) { sh[2][wave] = cxx; sh[3][wave] = cxy; sh[4][wave] = cyy; }
  __syncthreads();
  if (tid == 0) {
    const long r = blockIdx.x;
    float cv[4];
    cv[0] = (float)(sh[2][0] + sh[2][1] + sh[2][2] + sh[2][3]);
    cv[1] = (float)(sh[3][0] + sh[3][1] + sh[3][2] + sh[3][3]);
    cv[2] = cv[1];
    cv[3] = (float)(sh[4][0] + sh[4][1] + sh[4][2] + sh[4][3]);
    shift[r * 2 + 0] = m0;
    shift[r * 2 + 1] = m1;
    for (int j = 0; j < 4; ++j) covar[r * 4 + j] = cv[j];
    float u[4], sv[2];
    svd2(cv, u, sv);
    const float q0 = sqrtf(sv[0]), q1 = sqrtf(sv[1]);  // s ** 0.5
    affine[r * 4 + 0] = u[0] * q0;
    affine[r * 4 + 1] = u[1] * q1;
    affine[r * 4 + 2] = u[2] * q0;
    affine[r * 4 + 3] = u[3] * q1;
    if (uout) for (int j = 0; j < 4; ++j) uout[r * 4 + j] = u[j];
    if (svout) { svout[r * 2 + 0] = q0; svout[r * 2 + 1] = q1; }
  }
}

// One block per image: mean over HW of Cin channels, then the fc layer (nout rows).
__global__ __launch_bounds__(256) void bg_head_kernel(const float* feat, int Cin, int HW, const float* fw,
                                                      const float* fb, int nout, int bg_type, float* out) {
  __shared__ float mean[2048];
  const int n = blockIdx.x, tid = threadIdx.x;
  const float* f = feat + (long)n * Cin * HW;
  for (int c = tid; c < Cin; c += 256) {
    float s = 0.f;
    for (int i = 0; i < HW; ++i) s += f[(long)c * HW + i];
    mean[c] = s / (float)HW;
  }
  __syncthreads();
  __shared__ float pr[8];
  const int wave = tid >> 6, lane = tid & 63;
  for (int o = wave; o < nout; o += 4) {
    double acc = 0.0;
    for (int c = lane; c < Cin; c += 64) acc += (double)(fw[(long)o * Cin + c] * mean[c]);
    for (int k = 32; k > 0; k >>= 1) acc += __shfl_xor(acc, k);
    if (lane == 0) pr[o] = (float)acc + fb[o];
  }
  __syncthreads();
  if (tid == 0) {
    float* m = out + (long)n * 9;
    for (int j = 0; j < 9; ++j) m[j] = (j % 4 == 0) ? 1.f : 0.f;
    if (bg_type == 1) { m[2] = pr[0]; m[5] = pr[1]; }
    else if (bg_type >= 2) {
      for (int j = 0; j < 6; ++j) m[j] = pr[j];
      if (bg_type == 3) { m[6] = pr[6]; m[7] = pr[7]; }
    }
  }
}

__device__ __forceinline__ void inv2(const float* a, float* r) {
  const float det = a[0] * a[3] - a[1] * a[2];
  r[0] = a[3] / det;
  r[1] = -a[1] / det;
  r[2] = -a[2] / det;
  r[3] = a[0] / det;
}

// grid_sample(align_corners=True, zeros) of one channel plane at grid point (gx, gy)
__device__ __forceinline__ float sample_zero(const float* p, int h, int w, float gx, float gy) {
  const float ix = (gx + 1.f) * (float)(w - 1) / 2.f, iy = (gy + 1.f) * (float)(h - 1) / 2.f;
  const float fx = floorf(ix), fy = floorf(iy);
  const int x0 = (int)fx, y0 = (int)fy;
  const float wx = ix - fx, wy = iy - fy;
  const bool vx0 = x0 >= 0 && x0 < w, vx1 = x0 + 1 >= 0 && x0 + 1 < w;
  const bool vy0 = y0 >= 0 && y0 < h, vy1 = y0 + 1 >= 0 && y0 + 1 < h;
  const float nw = (vx0 && vy0) ? p[(long)y0 * w + x0] : 0.f;
  const float ne = (vx1 && vy0) ? p[(long)y0 * w + x0 + 1] : 0.f;
  const float sw = (vx0 && vy1) ? p[(long)(y0 + 1) * w + x0] : 0.f;
  const float se = (vx1 && vy1) ? p[(long)(y0 + 1) * w + x0 + 1] : 0.f;
  return nw * ((1.f - wx) * (1.f - wy)) + ne * (wx * (1.f - wy)) + sw * ((1.f - wx) * wy) + se * (wx * wy);
}

__device__ __forceinline__ float gauss(float mx, float my, const float* cov, float gx, float gy, int use_cov,
                                       float var) {
  const float dx = gx - mx, dy = gy - my;
  if (!use_cov) return expf(-0.5f * (dx * dx + dy * dy) / var);
  float iv[4];
  inv2(cov, iv);
  const float q = (dx * iv[0] + dy * iv[2]) * dx + (dx * iv[1] + dy * iv[3]) * dy;
  return expf(-0.5f * q);
}

struct MotionArgs {
  const float* src;      // [N][C][h][w] (downsampled source)
  const float* dshift;   // [N][R][2]
  const float* dcov;     // [N][R][4]
  const float* daff;     // [N][R][4]
  const float* sshift;
  const float* scov;
  const float* saff;
  const float* bg;       // [N][9] or null
  float* motion;         // [N][R+1][h][w][2]
  float* pin;            // [N][(R+1)*(C*use_def+1)][h][w]
  int N, R, C, h, w;
  int use_cov, use_def, revert;
  float var;
};

__global__ __launch_bounds__(256) void sparse_motion_kernel(MotionArgs a) {
  const int pix = blockIdx.x * 256 + threadIdx.x;
  const int k = blockIdx.y;  // 0 = background, 1..R = regions
  const int n = blockIdx.z;
  if (pix >= a.h * a.w) return;
  const int y = pix / a.w, x = pix % a.w;
  const float gx = coord(x, a.w), gy = coord(y, a.h);
  float mx, my, heat = 0.f;
  if (k == 0) {
    mx = gx; my = gy;
    if (a.bg) {
      const float* m = a.bg + (long)n * 9;
      const float X = m[0] * gx + m[1] * gy + m[2];
      const float Y = m[3] * gx + m[4] * gy + m[5];
      const float Z = m[6] * gx + m[7] * gy + m[8];
      mx = X / (Z + 1e-10f);
      my = Y / (Z + 1e-10f);
    }
  } else {
    const long r = (long)n * a.R + (k - 1);
    const float* ds = a.dshift + r * 2;
    const float* ss = a.sshift + r * 2;
    const float cx = gx - ds[0], cy = gy - ds[1];
    float id[4], af[4];
    inv2(a.daff + r * 4, id);
    const float* sa = a.saff + r * 4;
    af[0] = sa[0] * id[0] + sa[1] * id[2];
    af[1] = sa[0] * id[1] + sa[1] * id[3];
    af[2] = sa[2] * id[0] + sa[3] * id[2];
    af[3] = sa[2] * id[1] + sa[3] * id[3];
    if (a.revert) {
      const float sg = af[0] > 0.f ? 1.f : (af[0] < 0.f ? -1.f : 0.f);
      for (int j = 0; j < 4; ++j) af[j] *= sg;
    }
    mx = af[0] * cx + af[1] * cy + ss[0];
    my = af[2] * cx + af[3] * cy + ss[1];
    heat = gauss(ds[0], ds[1], a.dcov + r * 4, gx, gy, a.use_cov, a.var) -
           gauss(ss[0], ss[1], a.scov + r * 4, gx, gy, a.use_cov, a.var);
  }
  const long hw = (long)a.h * a.w;
  float* mo = a.motion + (((long)n * (a.R + 1) + k) * hw + pix) * 2;
  mo[0] = mx;
  mo[1] = my;
  const int per = a.C * a.use_def + 1;
  const long cin = (long)(a.R + 1) * per;
  float* pin = a.pin + ((long)n * cin + (long)k * per) * hw + pix;
  pin[0] = heat;
  if (a.use_def) {
    const float* sp = a.src + (long)n * a.C * hw;
    for (int c = 0; c < a.C; ++c) pin[(long)(1 + c) * hw] = sample_zero(sp + c * hw, a.h, a.w, mx, my);
  }
}

__global__ __launch_bounds__(256) void flow_combine_kernel(const float* logits, const float* motion, int K, int h,
                                                           int w, float* flow, int N) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long hw = (long)h * w;
  if (i >= N * hw) return;
  const long n = i / hw, pix = i % hw;
  const float* lg = logits + n * K * hw + pix;
  float mx = -INFINITY;
  for (int k = 0; k < K; ++k) mx = fmaxf(mx, lg[k * hw]);
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += expf(lg[k * hw] - mx);
  float fx = 0.f, fy = 0.f;
  const float* mo = motion + (n * K * hw + pix) * 2;
  for (int k = 0; k < K; ++k) {
    const float m = expf(lg[k * hw] - mx) / s;
    fx += mo[(long)k * hw * 2 + 0] * m;
    fy += mo[(long)k * hw * 2 + 1] * m;
  }
  flow[(n * 2 + 0) * hw + pix] = fx;
  flow[(n * 2 + 1) * hw + pix] = fy;
}

}  // namespace

void aa_down(hipStream_t s, float* out, const float* in, const float* w, int N, int C, int H, int W, int k,
             int step) {
  const int ka = k / 2;
  const int Hp = H + ka + (k % 2 == 0 ? ka - 1 : ka) - k + 1, Wp = W + ka + (k % 2 == 0 ? ka - 1 : ka) - k + 1;
  const int Ho = (Hp + step - 1) / step, Wo = (Wp + step - 1) / step;
  const long total = (long)N * C * Ho * Wo;
  hipLaunchKernelGGL(aa_down_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, out, in, w, C, H, W, k,
                     ka, step, Ho, Wo, total);
}

void region_stats(hipStream_t s, const float* logits, int NR, int h, int w, float temperature, float* heat,
                  float* shift, float* covar, float* affine, float* u, float* sv) {
  hipLaunchKernelGGL(region_stats_kernel, dim3(NR), dim3(256), 0, s, logits, h, w, temperature, heat, shift,
                     covar, affine, u, sv);
}

void bg_head(hipStream_t s, const float* feat, int N, int Cin, int HW, const float* fw, const float* fb, int nout,
             int bg_type, float* out) {
  hipLaunchKernelGGL(bg_head_kernel, dim3(N), dim3(256), 0, s, feat, Cin, HW, fw, fb, nout, bg_type, out);
}

void sparse_motion(hipStream_t s, const float* src, const float* dshift, const float* dcov, const float* daff,
                   const float* sshift, const float* scov, const float* saff, const float* bg, float* motion,
                   float* pin, int N, int R, int C, int h, int w, int use_cov, int use_def, int revert, float var) {
  MotionArgs a{src, dshift, dcov, daff, sshift, scov, saff, bg, motion, pin, N, R, C, h, w, use_cov, use_def, revert,
               var};
  hipLaunchKernelGGL(sparse_motion_kernel, dim3((unsigned)((h * w + 255) / 256), R + 1, N), dim3(256), 0, s, a);
}

void flow_combine(hipStream_t s, const float* logits, const float* motion, int N, int K, int h, int w, float* flow) {
  const long total = (long)N * h * w;
  hipLaunchKernelGGL(flow_combine_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, logits, motion, K,
                     h, w, flow, N);
}

}  // namespace extdm
