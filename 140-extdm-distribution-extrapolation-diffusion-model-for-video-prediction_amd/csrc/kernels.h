// ExtDM sampling path — HIP kernels for gfx950 (MI355X / CDNA4).
//
// Layout convention: every activation is a 5-D view [B][C][T][H][W] with
// contiguous H*W planes and explicit batch/channel/frame strides (elements).
// Channel-first buffers (sc = T*H*W, st = H*W) are the reference's NCDHW; the
// MotionAdaptor's work buffers are frame-major (sc = H*W, st = C*H*W) so that
// its '(T C)' channel flattening (u12:709) is a plain stride.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace extdm {

// f16x3 operand split: hi = fp16(v), lo = fp16(v - hi) from ONE opaque fp32 value.
// Without the barrier hipcc (ROCm 7.2, gfx950) may lower the two uses of fp16(v) of a
// product v differently (v_cvt_pk_f16_f32 of the rounded product for hi, v_fma_mixlo_f16
// of the exact product inside lo), and hi + lo then misses v by an fp16 ulp.
__device__ __forceinline__ float split_src(float v) {
  asm("" : "+v"(v));
  return v;
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// f16x3 split of two fp32 values in one opaque block: hi = fp16_rn(v) packed, lo =
// fp16_rn(v - hi) packed; v - hi is exact and v_fma_mix_f32 reads hi straight from the
// packed fp16 register (4 VALU per pair instead of ~5.3 for the converted-back hi, and the
// two roundings cannot be lowered differently, cf. split_src). For operands staged through LDS only:
// hipcc's hazard recognizer does not see inside inline asm, so neither may read an MFMA
// result or feed an MFMA directly (a stw_x3 version that split the PV accumulator this way
// read it before the MFMA had written it: run-to-run differences)
__device__ __forceinline__ void split2(float a, float b, unsigned& hi, unsigned& lo) {
  float da, db;
  asm("v_cvt_pk_f16_f32 %0, %4, %5\n\t"
      "v_fma_mix_f32 %2, -%0, 1.0, %4 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %3, -%0, 1.0, %5 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_cvt_pk_f16_f32 %1, %2, %3"
      : "=&v"(hi), "=v"(lo), "=&v"(da), "=&v"(db)
      : "v"(a), "v"(b));
}
// Scaled-lo split of a conv activation operand: hi = fp16_rn(v), lo = fp16_rn((v - hi) * 2^11).
// An unscaled lo is fp16-subnormal once |v| < 2^-3 (|v - hi| < 2^-14), so a tensor of small
// activations lost bits in every lo (the f16x3 error grew as 2^-25 / |v| instead of staying
// ~2^-23 relative: tests/test_gpu_precision.py activation-scale cases). Scaled, lo stays normal
// down to |v| ~ 2^-14 (hi's own normal range). The conv MFMA pairs it with the weight hi
// scaled by 2^-11 (lo_dn below), so the three products still share one accumulator:
//   a_lo * b_hi + a_hi * (b_lo' * 2^-11) = a_lo * b_hi + (a_hi * 2^-11) * b_lo'.
// The weight side's product is exact while a_hi * 2^-11 is normal (|a_hi| >= 2^-3 in the
// row-scaled units, whose row maximum is 2^14..2^15); the few smaller weights lose bits only
// in a term 2^-17 below the row's largest. Same LDS-only rule as split2.
// 4 VALU per pair: V = 2^11 (a, b) as one v_pk_mul_f32 (exact), then lo' = fp16(-hi 2^11 + V)
// by v_fma_mix{lo,hi}_f16 reading hi from the packed register (the fma is exact, one rounding:
// the bits of fp16((v - hi) 2^11))
typedef float f32x2s_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split2s(float a, float b, unsigned& hi, unsigned& lo) {
  const f32x2s_t V = (f32x2s_t){a, b} * 2048.f;
  asm("v_cvt_pk_f16_f32 %0, %2, %3\n\t"
      "v_fma_mixlo_f16 %1, -%0, %6, %4 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %1, -%0, %6, %5 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(hi), "=&v"(lo)
      : "v"(a), "v"(b), "v"(V.x), "v"(V.y), "s"(2048.f));
}
constexpr float X3_LO_UP = 2048.f;
// the weight-side factor of the scaled-lo product (exact power of two, 4 v_pk_mul_f16 per h8)
template <typename H8>
__device__ __forceinline__ H8 lo_dn(const H8& w) {
  return w * (_Float16)(1.f / 2048.f);
}
// The same split in compiler-visible code (v_cvt_pk_f16_f32 of the pair, two v_fma_mix_f32
// reading hi from the packed register, v_cvt_pk_f16_f32 of the remainders: 4 VALU per pair),
// for values that come from or go to MFMAs: hipcc inserts the MFMA hazard waits itself.
// hi is rounded once and lo reads that rounded register, so the two cannot disagree.
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
// packed fp32 pairs: v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 (two values per VALU issue; hipcc
// folds splats, swaps and negations into op_sel / op_sel_hi / neg_lo)
typedef f32x2_t f2;
__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 pair(float a, float b) { f2 v = {a, b}; return v; }
__device__ __forceinline__ f2 splat(float a) { f2 v = {a, a}; return v; }
__device__ __forceinline__ void split2c(float a, float b, f16x2_t& hi, f16x2_t& lo) {
  hi = __builtin_convertvector((f32x2_t){a, b}, f16x2_t);
  // an opaque 1.0: with a literal, instcombine turns the fma into fsub of a converted hi
  const float one = split_src(1.0f);
  const float la = __builtin_fmaf(-(float)hi.x, one, a);
  const float lb = __builtin_fmaf(-(float)hi.y, one, b);
  lo = __builtin_convertvector((f32x2_t){la, lb}, f16x2_t);
}
// The same split with lo produced in fp16 directly: each remainder as (fp16)fma(-hi, 1, v)
// is one v_fma_mixlo_f16 / v_fma_mixhi_f16 (3 VALU per pair). v - hi is exact in fp32, so
// the single rounding to fp16 gives the bits split2c gives. Needs -fno-slp-vectorize (the
// SLP pass otherwise packs the two fmas into a v_pk_fma_f32 and converts afterwards).
__device__ __forceinline__ void split2m(float a, float b, f16x2_t& hi, f16x2_t& lo) {
  hi = __builtin_convertvector((f32x2_t){a, b}, f16x2_t);
  const float one = split_src(1.0f);
  lo.x = (_Float16)__builtin_fmaf(-(float)hi.x, one, a);
  lo.y = (_Float16)__builtin_fmaf(-(float)hi.y, one, b);
}
// m = max(m, |a|, |b|) in one v_max3_f32 (the fp16-range check of the split values;
// the same hazard rule as split2)
__device__ __forceinline__ void amax2(float& m, float a, float b) {
  asm("v_max3_f32 %0, |%1|, |%2|, %0" : "+v"(m) : "v"(a), "v"(b));
}

// The template of the last attention launch on this thread (extdm_bench_layer_kernel: bench.py
// prices a layer by the arithmetic of the kernel it actually launched). printf-style.
void note_kernel(const char* fmt, ...);
const char* noted_kernel();

struct View {
  float* p = nullptr;
  int B = 0, C = 0, T = 0, H = 0, W = 0;
  long sb = 0, sc = 0, st = 0;  // strides in elements; plane stride = W, pixel stride = 1
  int HW() const { return H * W; }
  long numel() const { return (long)B * C * T * H * W; }
  View frames(int t0, int n) const {
    View v = *this; v.p = p + (long)t0 * st; v.T = n; return v;
  }
  View chans(int c0, int n) const {
    View v = *this; v.p = p + (long)c0 * sc; v.C = n; return v;
  }
};

inline View cf_view(float* p, int B, int C, int T, int H, int W) {  // channel-first
  View v; v.p = p; v.B = B; v.C = C; v.T = T; v.H = H; v.W = W;
  v.st = (long)H * W; v.sc = (long)T * H * W; v.sb = (long)C * T * H * W; return v;
}
inline View tm_view(float* p, int B, int C, int T, int H, int W) {  // frame-major
  View v; v.p = p; v.B = B; v.C = C; v.T = T; v.H = H; v.W = W;
  v.sc = (long)H * W; v.st = (long)C * H * W; v.sb = (long)C * T * H * W; return v;
}

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_SILU = 3, ACT_SIGMOID = 4 };
enum ConvMode { MODE_CONV = 0, MODE_DECONV = 1, MODE_UP2 = 2 };

// Packed GEMM weight: A[k][m] (k = ci*KH*KW + ky*KW + kx), zero padded to
// Kpad x Mpad; for MODE_DECONV four parity planes back to back.
struct PackedW {
  float* w = nullptr;
  int K = 0, M = 0, Kpad = 0, Mpad = 0, KH = 1, KW = 1, mode = MODE_CONV;
  // direct-conv (halo tile) layout [mtile][stage][step][half][BM], see conv_halo.hip
  float* wh = nullptr;
  int hstages = 0, hbm = 0;
  // f16x3 split layout [mtile][cblock*KS + ky][(g, kx)][m32][hi|lo][lane][8] (conv_x3.hip),
  // rows pre-scaled by powers of two undone by xscale[m]
  void* wx = nullptr;
  float* xscale = nullptr;
  int xbm = 0, xbn = 0, xng = 0, xncgb = 0;
  // f16x3 implicit-GEMM layout [parity][mtile][ktile][step][m32][hi|lo][lane][8]
  // (conv_gemm_x3.hip), rows pre-scaled by powers of two undone by gscale[m]
  void* gx = nullptr;
  float* gscale = nullptr;
  int gbm = 0, gnkt = 0;
  // the same with K tap-major (k = (ky * KW + kx) * Cin + ci; Cin % 8 == 0, KH * KW not dividing
  // 32): the gather of a K tile's 8-channel groups shares one tap (conv_gemm_x3.hip TAPK)
  void* gxt = nullptr;
  int gnkt_t = 0;
  // fp32 direct VALU layout [group][ci][ky * KW + kx][vcot rounded up to 4] (conv_narrow.hip), zero past M:
  // KS x KS convs with few output channels
  float* wv = nullptr;
  int vcot = 0;
};

// Output-channel tile of the conv GEMM for M output channels (Mpad is a multiple of it).
inline int conv_bm(int M) { return M <= 32 ? 32 : ((M <= 64 || M % 128 != 0) ? 64 : 128); }

struct ConvEpi {
  const float* bias = nullptr;     // [Cout]
  const float* res = nullptr;      // residual view (same B,T,H,W as out)
  long res_sb = 0, res_sc = 0, res_st = 0;
  const float* post_scale = nullptr;  // [B][Cout] (or [Cout] if post_per_channel): v = v * s + sh (after bias/res)
  const float* post_shift = nullptr;
  int post_per_channel = 0;
  int act = ACT_NONE;
  // GroupNorm statistics of the output (the conv's epilogue computes them where the
  // kernel supports it): partials [b * stats_groups + g][slot][2] = (sum, sum of squares)
  double* stats = nullptr;
  int stats_groups = 0;
  // GroupNorm + SiLU of the residual (conv_x3 1x1 only): r -> silu(r * a.x + a.y) with
  // a = res_aff[b * Cout + c] = (rstd * gamma, beta - mean * rstd * gamma); the ResnetBlock's
  // block2 norm folded into its res_conv (u12:199-203), so h2 is never normalised in place
  const float2* res_aff = nullptr;
  // split-K workspace (conv_x3, launches of few workgroups): fp32 partials, reused by every
  // conv of the stream in turn
  float* split_ws = nullptr;
  size_t split_ws_bytes = 0;
};

// Input channels per half-stage of the halo conv for kernel size ks and tile bm.
int halo_ch(int ks, int bm);
// Direct stride-1 'same' conv through LDS halo tiles; false if the geometry is not covered.
bool conv_halo_forward(hipStream_t s, const View& out, const View& in0, const View* in1, const PackedW& w,
                       const ConvEpi& epi);

// f16x3 split-precision direct conv (conv_x3.hip): tile choice, launch (false if
// the geometry is not covered), and the activation-range flag (|v| >= 65504 seen).
struct X3Tile { int bm, bn, ng; };
X3Tile x3_tile(int ks, int cout);

// With epi.stats set, *stats_slots receives the number of partial slots per (b, group)
// the epilogue wrote (0: not computed, the caller runs the statistics pass).
bool conv_x3_forward(hipStream_t s, const View& out, const View& in0, const View* in1, const PackedW& w,
                     const ConvEpi& epi, int* stats_slots = nullptr);
// Whether conv_x3_forward covers this stride-1 'same' conv (no launch).
bool conv_x3_covers(const View& out, const View& in0, const View* in1, const PackedW& w);
// Split-K partial bytes the conv will use (0: no split) -- ConvEpi::split_ws must hold them.
size_t conv_x3_split_bytes(const View& out, const View& in0, const View* in1, const PackedW& w);
size_t conv_x3_op_split_bytes(const View& out, const PackedW& w, int C);
// Pre-split f16x3 conv input ("operand") of an activation [B][C][T][H][W]: hi / lo fp16
// halves as [hl][c8][C/16][B*T][H+2*pad][W+2*pad][8] with a zero ring of width pad:
// channel 16*cg + 8*c8 + e of a padded position is element e of its 16-B record in
// plane (hl, c8) — the MFMA k-slice a lane of half c8 reads, one ds_read_b128 each.
struct X3Op {
  _Float16* p = nullptr;
  int B = 0, C = 0, T = 0, H = 0, W = 0, pad = 0;
};
size_t x3op_halves(int B, int C, int T, int H, int W, int pad);  // allocation incl. DMA slack
// Whether conv_x3_forward_op covers this conv (3x3 'same', C % 16 == 0, whole tiles).
bool conv_x3_op_supported(const View& out, const PackedW& w, int C, int pad);
bool conv_x3_forward_op(hipStream_t s, const View& out, const X3Op& in, const PackedW& w, const ConvEpi& epi,
                        int* stats_slots = nullptr);
// init_conv's cond_fea branch over a bilinear x2 upsample of F [B][C][T][H][W], phase-composed
// (fea_x3.hip header): the 5x5 part, out [B][Co][T][2H][2W] += (epi.res), weights [4 Co][C][5][5]
// edge (non-null): F's four edge lines are written to edge [B*T][4][H][C] (fea_edge_floats)
bool conv_x3_phase_forward(hipStream_t s, const View& out, const View& in, const PackedW& w, const ConvEpi& epi,
                           float* edge = nullptr, bool dry = false);
// ... and its edge corrections from those lines, added into out (after the 5x5 launch):
// side_w / side_scale the packed f16x3 line weights [pair][side][mtile][cb][tap][m32][hl][lane][8]
// / row scales [pair][side][mt * 128], corner_w fp32 [corner][C][Co][16 px]
struct FeaSideArgs {
  const float* e;  // edge lines [P][4][L][C]
  int C, L, T, P;
  const _Float16* w; const float* wscale;
  float* out; long ob, oc, ot; int OH, OW, Co;
  int out_bytes, pair;
  int* range;
};
struct FeaCornerArgs {
  const float* e;
  int C, L, T, P;
  const float* dw;
  float* out; long ob, oc, ot; int OH, OW, Co;
};
inline size_t fea_edge_floats(int P, int C, int L) { return (size_t)P * 4 * L * C; }
bool fea_edges_supported(int C, int Co, int L);
bool fea_edges_forward(hipStream_t s, const View& out, const float* edge, int C, const void* side_w,
                       const float* side_scale, const float* corner_w, bool dry = false);
void x3_range_reset(hipStream_t s);
// 1x1 256 -> 256 f16x3 conv with register-resident weights (pw_x3.hip) on conv_x3's packed 1x1
// weights (xbm 256): single input view, HW % 64 == 0, epilogue bias + ReLU only (no residual,
// statistics or post scale). false = not covered (the caller falls back).
// EXTDM_NO_PW=1 disables it (A/B).
bool pw_x3_forward(hipStream_t s, const View& out, const View& in, const PackedW& w, const ConvEpi& e);
// Evaluation metrics (metrics.hip): per-frame PSNR and SSIM in fp64.
size_t frame_metrics_workspace(int nframes, int C, int H);
void frame_metrics(hipStream_t s, const float* a, const float* b, int N, int T, int C, int H, int W, long sN, long sT,
                   long sC, double* psnr, double* ssim, double* work);
int* x3_range_ptr();  // device address of the flag on the current device
int x3_range_read(hipStream_t s);

// out = act(conv(in0 ++ in1) + bias + res) [* s + sh]
// Returns the GroupNorm partial slots written for epi.stats (0 if none).
int conv_forward(hipStream_t s, const View& out, const View& in0, const View* in1, const PackedW& w,
                 int stride, int pad, const ConvEpi& epi);

// GroupNorm(G) over a channel-first view, optional FiLM (x*(scale+1)+shift from
// a [Mtot][NT] table at row offset, column t[b]) then SiLU, optional residual.
void groupnorm_silu(hipStream_t s, const View& x, const View& out, int groups, const float* gamma,
                    const float* beta, const float* film, int film_row, int film_nt, const int* t_batch,
                    const View* res, double* partials, int given_split = 0);
// given_split > 0: `partials` already holds that many (sum, sumsq) slots per (b, group)
// (written by the producing conv's epilogue); the statistics pass is skipped.
// The same GroupNorm + FiLM + SiLU written as the pre-split operand of the next 3x3 conv
// (its only consumer), instead of fp32.
void groupnorm_silu_x3op(hipStream_t s, const View& x, const X3Op& out, int groups, const float* gamma,
                         const float* beta, const float* film, int film_row, int film_nt, const int* t_batch,
                         double* partials, int given_split = 0);
// GroupNorm of x as a per-(b, c) affine table (rstd * gamma, beta - mean * rstd * gamma)
// [B][C] (statistics pass unless given_split > 0), for a consumer that applies the norm
// itself (ConvEpi::res_aff); stored in `partials` after the (mean, rstd) pairs
const float2* groupnorm_affine(hipStream_t s, const View& x, int groups, const float* gamma, const float* beta,
                               double* partials, int given_split = 0);

// Channel LayerNorm (biased var over C, gamma only; u12:138-147) of in0 ++ in1.
void channel_ln(hipStream_t s, const View& out, const View& in0, const View* in1, const float* gamma);
// Fused init_temporal_attn prologue: y = chanLN(x)*g; z = LayerNorm(y)*w+b;
// writes z and r = x + y (the double residual of u12:915 + 326).
void temporal_prologue(hipStream_t s, const View& x, const float* gamma, const float* lw, const float* lb,
                       const View& z, const View& r);

struct AttnGeom {
  int mode;          // 0 = shifted-window (STW), 1 = temporal (per pixel)
  int D, H, W;       // unpadded extents
  int ws0, ws1, ws2; // effective window
  int ss0, ss1, ss2; // effective shift
  int Dp, Hp, Wp;    // padded extents
  int per;           // mode 1, fused kernels (stw_x3.hip): frame slots per pixel (8, 16, 32; 0 = 16 / 32 by D)
};
// frame slots per pixel of the fused temporal attention (32 tokens per wave = 32 / per pixels)
__host__ __device__ inline int temporal_slots(const AttnGeom& g) { return g.per ? g.per : (g.D <= 16 ? 16 : 32); }
// Attention core (attn_core.hip): QK^T / softmax / PV over qkv [B][3*heads*32][T][H][W]
// into o [B][heads*32][T][H][W], token groups of <= 64 (temporal: <= 32 frames),
// dim_head 32; f16x3 (fp32-faithful) or bf16 (EXTDM_PRECISION_BF16_ATTN). False if the
// shape is not covered. bias_dense [heads][bstride][bstride].
bool attention_core(hipStream_t s, const View& qkv, const View& o, const AttnGeom& g, int heads, int dim_head,
                    const float* bias_dense, int bstride, const float* rope_cos, const float* rope_sin, float q_scale,
                    bool bf16);
// Unfused attention (dim_head 32, <= 32 tokens per group; e.g. C = 512 levels).
// qkv: channel-first [B][3*heads*32][T][H][W]; o: [B][heads*32][T][H][W].
void window_attention(hipStream_t s, const View& qkv, const View& o, const AttnGeom& g, int heads,
                      const float* bias_dense /*[heads][32][32]*/, const float* rope_cos,
                      const float* rope_sin /*[>=32][16]*/, float q_scale);
// Shapes the fused attention kernels handle: heads 8, C in {64,128,256}, a group of
// <= 32 or exactly 64 tokens, dim_head 16 or 32.
bool fused_attn_supported(int C, int ntok, int dim_head, int heads);
// Fused Residual(PreNorm(STWAttentionLayer)) in place on x (stw_fused.hip); false if
// the shape is unsupported. Weights pre-packed (see the kernel header);
// bias_dense [heads][bstride][bstride]; rope tables [64][dim_head/2].
bool stw_fused(hipStream_t s, const View& x, const AttnGeom& g, int heads, int dim_head, const float* gamma,
               const float* wqkv, const float* wp, const float* bp, const float* bias_dense, int bstride,
               const float* rcos, const float* rsin, float q_scale);
// Fused Residual(PreNorm(chanLN, AttentionLayer)) over frames (double LayerNorm, qkv,
// temporal attention with T5 bias and RoPE, to_out, double residual); out must share
// x's strides and may alias x.
bool temporal_fused(hipStream_t s, const View& x, const View& out, const AttnGeom& g, int heads, int dim_head,
                    const float* gamma, const float* ln_w, const float* ln_b, const float* wqkv, const float* wout,
                    const float* bias_dense, int bstride, const float* rcos, const float* rsin, float q_scale);
// f16x3 fused attention (stw_x3.hip): one wave per group of <= 32 tokens, C in {64, 128};
// bf16 = the QK^T / PV contractions on bf16 MFMA (BF16_ATTN, dim_head 32).
// Weights packed per unit of 32 qkv rows (attn_x3_unit_halves(C) halves each, see the
// kernel header); wsc = {2^-sq, 2^-sk, 2^-sv, 2^-sproj} undoes the power-of-two pre-scaling.
bool attn_x3_supported(int C, int ntok, int dim_head, int heads);
int attn_x3_unit_halves(int C);
// mbias: [npat][8][32][32] bias + masks per window class (stw_x3.hip kernel header).
bool stw_x3(hipStream_t s, const View& x, const AttnGeom& g, int heads, int dim_head, const float* gamma,
            const void* wpk, const float* wsc, const float* bp, const float* mbias, int npat,
            const float* rcos, const float* rsin, float q_scale, bool bf16);
// f16x3 fused STW attention over windows of <= 64 tokens (stw64_x3.hip: ada / ada_u22 4x4x4
// windows), two waves per window; the stw_x3 weight packing; mbias [npat][8][64][64] (bias +
// masks per window class, times 2^(e_q + e_k)); bf16 = the attention contractions on bf16 MFMA.
bool stw64_x3_supported(int C, int ntok, int dim_head, int heads);
bool stw64_x3(hipStream_t s, const View& x, const AttnGeom& g, int heads, int dim_head, const float* gamma,
              const void* wpk, const float* wsc, const float* bp, const float* mbias, int npat, const float* rcos,
              const float* rsin, float q_scale, bool bf16);
bool temporal_x3(hipStream_t s, const View& x, const View& out, const AttnGeom& g, int heads, int dim_head,
                 const float* gamma, const float* ln_w, const float* ln_b, const void* wpk, const float* wsc,
                 const float* mbias, const float* rcos, const float* rsin, float q_scale, bool bf16);
// TrajWarp cross-attention (u12:719-773): q [B][256][NQ], k,v [B][256][NK].
// f16x3 implicit-GEMM conv (conv_gemm_x3.hip): every mode / kernel size of conv_forward's
// fp32 GEMM; false if the weight has no f16x3 GEMM packing
// init_conv's x-branch composed with init_noise_conv into 49 border-class 13x13
// kernels (xpath_x3.hip): out[:, :Cout] = sum_c K_c * x + cbias_c (+ add) for the 3-channel x;
// add (optional, same geometry as out): the hoisted cond_fea branch (runtime fea_hoist_on)
struct XPathArgs {
  const float* x; long xb, xc, xt;  // the zero-padded pre-split copy (xpad_forward; dwords)
  int T, L, F, LP;
  float* out; long ob, oc, ot; int Cout;
  const _Float16* w; const float* rscale; const float* cbias;
  const float* add; long ab, ac, at;
  // tiles in frame-group-major order (xpath_x3.hip): groups of FG frames, every class's tiles of a
  // group consecutive; tile_start / tile_last: the class prefix of a full / the last group
  int FG, ngroups, gtiles, xcd;  // xcd: XCD-contiguous workgroup order (grid a multiple of 8)
  int tile_start[50];
  int tile_last[50];
};
bool xpath_x3_forward(hipStream_t s, const View& out, const View& x, const void* w, const float* rscale,
                      const float* cbias, const View* add = nullptr);
// the zero-padded copy of the 3-channel x both kernels above read: [B][3][T][LP][LP], x at
// (6, 6), LP = xpad_size(L), one dword per position holding its f16x3 pair (hi | lo' << 16,
// lo' = fp16((v - hi) 2^11)); the range flag (|v| >= 65504) is raised here
int xpad_size(int L);
void xpad_forward(hipStream_t s, const View& xpad, const View& x);
// maxpool(1,2,2)(init_noise_conv(x)) in one kernel (xpath_x3.hip): out [B][C][T][L/2][L/2]
struct NoisePoolArgs {
  const float* x; long xb, xc, xt;  // the zero-padded pre-split copy (xpad_forward; dwords)
  int T, L, F, LP;
  float* out; long ob, oc, ot; int Cout;
  const _Float16* w; const float* rscale; const float* bias;
  const float* add; long ab, ac, at;  // conv7c3 only: residual added in the epilogue
};
bool noise_pool_x3_forward(hipStream_t s, const View& out, const View& x, const void* w, const float* rscale,
                           const float* bias);
// A plain (1,7,7) 'same' conv of the 3-channel x (ada_u22 / wo_ref init_conv x-branch, the cond_fea
// branch hoisted into `add`): out = W * x + bias + add, from the zero-padded copy (xpad_forward), the
// weights packed like noise_pool's (Pconv7c3); L a multiple of 32, Cout a multiple of 64
bool conv7c3_x3_forward(hipStream_t s, const View& out, const View& x, const void* w, const float* rscale,
                        const float* bias, const View* add);
// Few-output-channel KS x KS convs on fp32 VALU FMAs (conv_narrow.hip): narrow_cot(KS, M) is the
// packer's output-channel group (0: not taken); false if the conv is not covered.
int narrow_cot(int KS, int M);
bool conv_narrow_forward(hipStream_t s, const View& out, const View& in0, const View* in1, const PackedW& w,
                         int stride, int pad, const ConvEpi& epi);
bool conv_gemm_x3_forward(hipStream_t s, const View& out, const View& in0, const View* in1, const PackedW& w,
                          int stride, int pad, const ConvEpi& epi);
void cross_attention(hipStream_t s, const float* q, const float* k, const float* v, float* o, int B, int C,
                     int heads, int NQ, int NK);
// f16x3 variant (cross_x3.hip); false if the shape is not covered (dim_head != 32)
bool cross_attention_x3(hipStream_t s, const float* q, const float* k, const float* v, float* o, int B, int C,
                        int heads, int NQ, int NK);
// The same with K / V pre-split once (cross_kv_split, per sampling call) into MFMA fragments
// kvp (cross_kv_halves halves): no staging in the per-step kernel.
size_t cross_kv_halves(int B, int C, int heads, int NK);
bool cross_kv_split(hipStream_t s, const float* k, const float* v, _Float16* kvp, int B, int C, int heads, int NK);
bool cross_attention_x3p(hipStream_t s, const float* q, const _Float16* kvp, float* o, int B, int C, int heads, int NQ,
                         int NK);

void copy_view(hipStream_t s, const View& dst, const View& src);
void maxpool_hw2(hipStream_t s, const View& dst, const View& src);
// bilinear (align_corners=False) resize of frames [0,t_split) from a and
// [t_split,T) from b into dst (u12:1035-1037)
void bilinear_frames(hipStream_t s, const View& dst, const View& a, const View& b, int t_split);
// per (b,c) mean and unbiased std (+eps) over T*H*W (u12:670-678)
void adaptor_stats(hipStream_t s, const View& x, float* mean, float* std_, double* partials);
void adaptor_normalize(hipStream_t s, const View& dst, const View& src, const float* mean, const float* std_);
// zero frames 0 and T - 1 of every clip of a frame-major buffer (one launch; a 2-D memset of the
// same rows ran at ~0.2 TB/s)
void zero_pad_frames(hipStream_t s, const View& x);

// Sampler step kernels.
struct StepCoef {  // per sampler step (host-computed in fp32 exactly like the reference)
  float sra, srm1;            // sqrt_recip_alphas_cumprod[t], sqrt_recipm1_alphas_cumprod[t]
  float c1, c2, sigma;        // DDPM: posterior coef1/coef2, exp(0.5*logvar)*[t!=0]; DDIM: sqrt(a_next), c, sigma
  int t;                      // model timestep
  int use_noise;              // 0 => no noise term (DDIM time_next == 0)
  int kind;                   // 0 = DDPM, 1 = DDIM
};
void sampler_step(hipStream_t s, float* x, const float* eps, int B, int n, const StepCoef* coefs,
                  const int* step_ctr, const float* noise /*[S][B][n] or null*/, uint64_t seed, int sample_base,
                  int round, int k_lo, int k_hi, float q_w, float* thresh_out);
// The same step over (4096-element chunk, sample) workgroups (sampler.hip): four radix count
// launches, the update launch and (t_next non-null) a one-workgroup launch that writes
// coefs[step + 1].t to t_next[0 .. B) (if step + 1 < nsteps) and increments *step_ctr (the captured
// step's set_t / incr). ws: the selection workspace, sampler_sel_bytes(B, n) bytes for the launched
// B and n (its layout depends on both); it needs no initialisation. thresh_out (both forms, may be
// null): the threshold of sample b at step k goes to thresh_out[k * B + b].
size_t sampler_sel_bytes(int B, int n);
void sampler_step_mw(hipStream_t s, float* x, const float* eps, int B, int n, const StepCoef* coefs, int* step_ctr,
                     const float* noise, uint64_t seed, int sample_base, int round, int k_lo, int k_hi, float q_w,
                     float* thresh_out, unsigned* ws, int* t_next, int nsteps);
void fill_normal(hipStream_t s, float* x, int B, int n, uint64_t seed, int sample_base, int round, int stream_id);
void set_t_from_step(hipStream_t s, int* t_batch, int B, const StepCoef* coefs, const int* step_ctr);
void incr_counter(hipStream_t s, int* ctr);
void t_to_int(hipStream_t s, const int64_t* t, int* t_batch, int B);

// LFAE decoder pieces (decoder.hip)
void warp_blend(hipStream_t s, float* out, const float* src, int N, int C, int S, const float* flow,
                const float* occ, int T, int fh, int fw, const float* prev);
void affine_relu(hipStream_t s, float* out, const float* in, const float* a, const float* b, int N, int C, int HW);
void avgpool2(hipStream_t s, float* out, const float* in, int planes, int Ho, int Wo);

// LFAE decoder (no occlusion): flow [B][2][T][h][w] (x,y) -> bilinear to
// image size, grid_sample(src) (align_corners=True, zeros)
void warp_frames(hipStream_t s, float* out, const float* src, const float* flow, int B, int C, int T, int S,
                 int fh, int fw, long out_sb, long out_sc, long out_st);

// LFAE encoder pieces (lfae.hip)
void aa_down(hipStream_t s, float* out, const float* in, const float* w, int N, int C, int H, int W, int k,
             int step);
void region_stats(hipStream_t s, const float* logits, int NR, int h, int w, float temperature, float* heat,
                  float* shift, float* covar, float* affine, float* u, float* sv);
void bg_head(hipStream_t s, const float* feat, int N, int Cin, int HW, const float* fw, const float* fb, int nout,
             int bg_type, float* out);
void sparse_motion(hipStream_t s, const float* src, const float* dshift, const float* dcov, const float* daff,
                   const float* sshift, const float* scov, const float* saff, const float* bg, float* motion,
                   float* pin, int N, int R, int C, int h, int w, int use_cov, int use_def, int revert, float var);
void flow_combine(hipStream_t s, const float* logits, const float* motion, int N, int K, int h, int w, float* flow);

}  // namespace extdm
