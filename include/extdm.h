/* ExtDM sampling path — C ABI of libextdm_hip.so (MI355X / gfx950).
 *
 * The drop-in boundary under the package's Python mirror of the reference API.
 * Plain pointers and sizes only; every tensor is fp32, contiguous NCDHW
 * (`b c t h w`) and caller-owned; device pointers live on the handle's device.
 * Every function returns 0 on success or a negative status; the message is in
 * extdm_last_error() (thread-local), which the Python layer raises as
 * RuntimeError. A handle is not thread-safe; different handles may run
 * concurrently (one per device / process).
 *
 * Reference interfaces replaced (file:line in the reference tree):
 *   extdm_create / extdm_load_weight / extdm_finalize
 *       Unet3D.__init__ + load_state_dict          DenoiseNet_..._u12.py:864-1003,
 *                                                   _ada.py:865-1018, _ada_u22.py:1009-1170,
 *                                                   _wo_ref_adaptor_cross_multi.py:755-904
 *       GaussianDiffusion.__init__ buffers          Diffusion.py:52-122
 *       Generator.__init__ (decoder half)           LFAE/generator.py:26-62
 *   extdm_unet_forward   Unet3D.forward / forward_with_cond_scale(cond_scale=1)
 *                                                   u12:1005-1086, ada:1020-1089,
 *                                                   ada_u22:1172-1306 (path=0), wo_ref:906-967
 *   extdm_sample         GaussianDiffusion.p_sample_loop / ddim_sample
 *                                                   Diffusion.py:180-189, 209-258
 *   extdm_sampler_step   one p_sample / DDIM update given eps
 *                                                   Diffusion.py:145-177, 231-255
 *   extdm_decode         Generator.forward_with_flow   LFAE/generator.py:152-206
 *   extdm_region_params  RegionPredictor.forward       LFAE/region_predictor.py:62-150
 *   extdm_bg_params      BGMotionPredictor.forward     LFAE/bg_motion_predictor.py:47-64
 *   extdm_flow_predict   PixelwiseFlowPredictor.forward LFAE/pixelwise_flow_predictor.py:106-153
 *   extdm_bottleneck     Generator.forward_bottle      LFAE/generator.py:95-102
 *   extdm_frame_metrics  img_psnr / calculate_ssim_function per frame (the per-frame
 *                        loops of calculate_psnr2 / calculate_ssim2, valid.py:226-233)
 *                                                   metrics/calculate_psnr.py:6-15,
 *                                                   metrics/calculate_ssim.py:6-41
 */
#ifndef EXTDM_H
#define EXTDM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ExtdmHandle ExtdmHandle;

/* Unet3D denoiser variants, one per reference module:
 *   U12      DenoiseNet_STWAtt_w_w_ref_adaptor_cross_multi_traj_u12.py (== _u22.py): BAIR
 *   ADA      ..._traj_ada.py: KTH (window 4x4x4, dim_head 16, cond_adaptor + cond_temporal_attn)
 *   ADA_U22  ..._traj_ada_u22.py: Cityscapes / UCF (b1,b2,STW,STW,adaptor,temporal per level)
 *   WO_REF   DenoiseNet_STWAtt_w_wo_ref_adaptor_cross_multi.py: SMMNIST (tc-1 cond frames,
 *            cond_fea at latent resolution, fea: [B,fea_ch,tc-1+tp,L,L]) */
enum { EXTDM_ARCH_U12 = 0, EXTDM_ARCH_ADA = 1, EXTDM_ARCH_ADA_U22 = 2, EXTDM_ARCH_WO_REF = 3 };
enum { EXTDM_SAMPLER_DDPM = 0, EXTDM_SAMPLER_DDIM = 1 };
/* Arithmetic of the direct convolutions (every tensor stays fp32):
 *   FP32   v_mfma_f32_32x32x2_f32 (exact fp32 products and sums)
 *   F16X3  fp32 operands split as hi + lo fp16 pairs, three fp16 MFMAs per product
 *          (lo*hi + hi*lo + hi*hi) into fp32 accumulators: fp32-level error, 5.3x
 *          the fp32 MFMA rate. Needs |activation| < 65504 at conv inputs; a value
 *          outside raises the range flag (extdm_range_flag; extdm_sample fails).
 *   BF16_ATTN  F16X3 convolutions; the attention QK^T / PV contractions of the STW
 *          window and temporal layers on bf16 MFMA (v_mfma_f32_32x32x16_bf16, fp32
 *          accumulate; q, k, probabilities and v rounded to bf16), the configuration
 *          BASELINE names for UCF-101 256. Not fp32-faithful: tests/test_gpu_bf16_attn.py
 *          states its tolerance against the fp32 reference. */
enum { EXTDM_PRECISION_FP32 = 0, EXTDM_PRECISION_F16X3 = 1, EXTDM_PRECISION_BF16_ATTN = 2 };

typedef struct ExtdmConfig {
  int arch;            /* EXTDM_ARCH_* */
  int dim;             /* Unet base width (64) */
  int channels;        /* init_conv input channels (256 + 256) */
  int dim_mults[4];
  int n_levels;        /* entries used in dim_mults */
  int window[3];       /* (2, 4, 4) */
  int heads;           /* attn_heads (8) */
  int dim_head;        /* attn_dim_head (32) */
  int tc, tp;          /* cond / pred frames */
  int latent;          /* flow-latent H = W (32) */
  int fea_size;        /* cond_fea H = W (16) */
  int fea_ch;          /* cond_fea channels (256) */
  int timesteps;       /* diffusion T (1000) */
  int max_batch;       /* workspace is sized for this batch (clips) */
  int device;          /* HIP device ordinal */
  /* LFAE Generator decoder (flow_params.generator_params); image = frame size */
  int image, num_channels, gen_block_expansion, gen_max_features, gen_num_down_blocks, gen_num_bottleneck_blocks;
  int precision;       /* EXTDM_PRECISION_* */
} ExtdmConfig;

int extdm_create(const ExtdmConfig* cfg, ExtdmHandle** out);
void extdm_destroy(ExtdmHandle* h);
const char* extdm_last_error(void);

/* Copy one named tensor (reference state_dict key: Unet keys without the
 * `denoise_fn.` prefix, GaussianDiffusion buffers by their own names, decoder
 * keys with a `generator.` prefix). dtype: 0 = float32, 1 = int64. Host memory. */
int extdm_load_weight(ExtdmHandle* h, const char* name, const void* host_ptr, int dtype, const int64_t* shape,
                      int ndim);
/* Pack weights into the GEMM layouts, build t-only tables (time-MLP, FiLM,
 * rotary, relative-position biases) and the workspace. */
int extdm_finalize(ExtdmHandle* h);
int64_t extdm_workspace_bytes(const ExtdmHandle* h);

/* eps = Unet3D(x, t, cond_frames, cond_fea). x, out: [B,3,tp,L,L]; t: int64 [B];
 * cond: [B,3,tc,L,L]; fea: [B,fea_ch,T,fs,fs] with T = tc+tp (tc-1+tp for WO_REF).
 * All device pointers. */
int extdm_unet_forward(ExtdmHandle* h, int B, const float* x, const int64_t* t, const float* cond,
                       const float* fea, float* out, void* stream);

/* Whole reverse loop. times[k] is the model timestep of step k and
 * times_next[k] the DDIM target (ignored for DDPM). x_T (device, may be NULL:
 * Philox stream), noise (device [S][B][n] or NULL: Philox stream), out (device
 * [B,3,tp,L,L]) receives x_0. use_graph != 0 replays one captured step. */
int extdm_sample(ExtdmHandle* h, int B, int sampler, int S, const int* times, const int* times_next, float eta,
                 const float* x_cond, const float* cond_fea, const float* x_T, const float* noise, uint64_t seed,
                 int sample_base, int round, float* out, int use_graph, void* stream);

/* Record the dynamic-threshold value s = max(1, quantile(|x0|, 0.9)) of every step and sample
 * of later extdm_sample calls into buf[k * B + b] (device fp32, cap floats >= S x B; NULL
 * stops recording). Verification hook for the captured-graph sampler (the threshold inside
 * p_mean_variance, Diffusion.py:150-163); the step itself is unchanged. */
int extdm_record_thresholds(ExtdmHandle* h, float* buf, int64_t cap);

/* One sampler update in place on x given eps (the step-k coefficients). */
int extdm_sampler_step(ExtdmHandle* h, int B, int sampler, int t, int t_next, float eta, float* x, const float* eps,
                       const float* noise, float* thresh_out, void* stream);

/* Measurement hook for bench.py: time `iters` launches of one hot-path conv
 * exactly as the forward issues it, on random operands, with HIP events on the
 * handle's stream; returns the average ms per launch and the algorithmic FLOPs
 * per launch. layer 0 = init_conv (1,7,7) channels->dim (two sources); 1, 2, 3 =
 * ResnetBlock (1,3,3) convs at levels 0, 1, 2 (downs.{0,1,2}.0.block2) from an fp32
 * input; 4 = the level-0 up ResnetBlock's 1x1 res_conv (ups.3.0.res_conv); 5 = the
 * level-0 block2 conv from block1's pre-split operand, as the F16X3 forward issues it. */
int extdm_bench_layer(ExtdmHandle* h, int B, int layer, int iters, float* ms_out, double* flops_out);
/* (6 / 7: the level-0 STW / init_temporal attention layer — one fused launch, or on the unfused
 * core route the attention core alone; 14 / 15: that STW layer's qkv / proj 1x1 conv alone and
 * 16 / 17: the temporal layer's qkv / to_out, on the core route only; 8-13: see runtime.cpp.)
 * The kernel template the last extdm_bench_layer call of `layer` launched for the attention
 * layers (e.g. "stw64_x3_kernel<64, 16, 8, false>"), written to buf (cap bytes, NUL-terminated;
 * empty when not recorded). bench.py prices a layer by that kernel's arithmetic. */
int extdm_bench_layer_kernel(ExtdmHandle* h, int layer, char* buf, int cap);

/* The F16X3 activation-range flag: nonzero if an operand split since the last reset
 * had |v| >= 65504 (results computed meanwhile are not fp32-accurate): bit 0 = a conv /
 * GEMM / cross-attention input, bit 1 = a fused-attention operand; 0 if not, <0 on
 * error; reset != 0 clears it. Synchronises `stream`. */
int extdm_range_flag(ExtdmHandle* h, int reset, void* stream);

/* One attention layer as the forward issues it (parity tests): prefix names a
 * Residual(PreNorm(STWAttentionLayer)) (e.g. "downs.0.1", shifted per the layer's
 * position, u12:961-963) or a temporal Residual(PreNorm(AttentionLayer)) (e.g.
 * "init_temporal_attn", u12:915). x, out: [B,C,T,H,W] device tensors. */
int extdm_attn_layer(ExtdmHandle* h, const char* prefix, int B, int C, int T, int H, int W, int shifted,
                     const float* x, float* out, void* stream);

/* LFAE decoder (Generator.forward_with_flow) for B clips x T frames.
 * ref: [B,C,S,S] source image; flow: [B,2,T,fh,fw] (x, y grid); occ: [B,1,T,fh,fw]
 * occlusion in [0,1] or NULL (reference quirk: without occlusion the prediction
 * equals the warped source); pred: [B,C,T,S,S]; warped: [B,C,T,S,S] or NULL
 * ('deformed'). Needs the decoder weights (keys 'generator.*') unless occ is NULL. */
int extdm_decode(ExtdmHandle* h, int B, int C, int T, int S, int fh, int fw, const float* ref, const float* flow,
                 const float* occ, float* pred, float* warped, void* stream);

/* ---- LFAE encoder ------------------------------------------
 * flow_params.model_params of the config/DM YAML files. Set before extdm_finalize on a
 * handle that holds 'region_predictor.*', 'bg_predictor.*' and/or 'generator.*'
 * (incl. 'generator.pixelwise_flow_predictor.*') weights. Images are [N][C][S][S]
 * fp32 device tensors, S = image; N <= max_batch. */
typedef struct ExtdmLfaeConfig {
  int num_regions, num_channels, image, revert_axis_swap;
  float rp_temperature, rp_scale_factor;
  int rp_pad, rp_num_blocks, rp_pca_based;
  int bg_type; /* 0 zero, 1 shift, 2 affine, 3 perspective */
  int bg_num_blocks;
  float pf_scale_factor, pf_region_var;
  int pf_num_blocks, pf_use_covar_heatmap, pf_use_deformed_source;
} ExtdmLfaeConfig;
int extdm_set_lfae(ExtdmHandle* h, const ExtdmLfaeConfig* c);

/* RegionPredictor.forward, PCA-based (LFAE/region_predictor.py:62-150):
 * shift [N][R][2], covar [N][R][2][2], affine [N][R][2][2] = U sqrt(S) with
 * torch.svd's (LAPACK sgesdd) sign convention; u [N][R][2][2], sv [N][R][2] (sqrt of
 * the singular values, the diagonal of 'd') and heatmap [N][R][h][w] optional (NULL).
 * extdm_region_hw gives the heatmap side h = w. */
int extdm_region_params(ExtdmHandle* h, int N, const float* img, float* shift, float* covar, float* affine,
                        float* u, float* sv, float* heatmap, void* stream);
int extdm_region_hw(const ExtdmHandle* h);

/* BGMotionPredictor.forward (LFAE/bg_motion_predictor.py:47-64): out [N][3][3]. */
int extdm_bg_params(ExtdmHandle* h, int N, const float* src, const float* drv, float* out, void* stream);

/* PixelwiseFlowPredictor.forward (LFAE/pixelwise_flow_predictor.py:106-153) for
 * source images src and the region params above (+ bg [N][3][3] or NULL):
 * flow [N][2][h][w] (x, y; the reference's optical_flow permuted), occ [N][1][h][w]
 * or NULL (needs the occlusion head). h = w = extdm_flow_hw(). */
int extdm_flow_predict(ExtdmHandle* h, int N, const float* src, const float* drv_shift, const float* drv_covar,
                       const float* drv_affine, const float* src_shift, const float* src_covar,
                       const float* src_affine, const float* bg, float* flow, float* occ, void* stream);
int extdm_flow_hw(const ExtdmHandle* h);

/* Generator.forward_bottle / compute_fea (LFAE/generator.py:95-102, 202-206):
 * out [N][C_bottleneck][S / 2^d][S / 2^d]. */
int extdm_bottleneck(ExtdmHandle* h, int N, const float* img, float* out, void* stream);

/* Per-frame PSNR and SSIM of two frame sets a, b (device fp32, [N][T][C][H][W] through
 * element strides sN, sT, sC; planes contiguous H*W) into device doubles psnr[N*T],
 * ssim[N*T], in fp64 like the reference's numpy evaluation. C must be 1 or 3 and
 * H, W > 10 (the 11x11 window's valid region). `work` is device scratch of
 * extdm_frame_metrics_workspace() bytes. Not tied to a handle. */
size_t extdm_frame_metrics_workspace(int N, int T, int C, int H, int W);
int extdm_frame_metrics(const float* a, const float* b, int N, int T, int C, int H, int W, long sN, long sT, long sC,
                        double* psnr, double* ssim, void* work, void* stream);

/* Bilinear resize (align_corners=False, F.interpolate(mode='bilinear')) of frames into a
 * contiguous dst [B][C][T][OH][OW]: frame t < t_split from a at frame t, frame t >= t_split from
 * b at frame t - t_split (element strides per batch / channel / frame; planes contiguous H*W;
 * a frame stride of 0 repeats one frame). Replaces the multi1248 wrapper's per-frame
 * interpolate of the cond features (multi1248.py:240-245). Not tied to a handle. */
int extdm_bilinear_frames(float* dst, int B, int C, int T, int OH, int OW, const float* a, long a_sb, long a_sc,
                          long a_st, const float* b, long b_sb, long b_sc, long b_st, int t_split, int H, int W,
                          void* stream);

#ifdef __cplusplus
}
#endif

#endif /* EXTDM_H */
