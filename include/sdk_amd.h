/*
 * sdk_amd.h — C ABI of the MI355X (gfx950) latent-diffusion hot path.
 *
 * The reference (ProgramerSalar/stable-diffusion-from-scratch) has no FFI: its
 * hot path is a chain of stock torch.nn ops plus two un-vendored flash_attn
 * entry points.  Each entry point below replaces a family of those call sites
 * (cited per function, file:line into the reference).  The library is driven
 * by the Python mirror of the reference's modules (UNetModel, AutoEncoderKL,
 * DDIMSampler) in stable-diffusion-from-scratch_amd/ through ctypes.
 *
 * Conventions (all entry points):
 *   - activations are NHWC (token-major) IEEE fp16; statistics and the sampler
 *     state are fp32; every pointer is device memory owned by the caller;
 *   - the library allocates nothing per call; work launches on `stream`
 *     (a hipStream_t, NULL = legacy default) and never synchronises, so a
 *     caller may capture the calls into a hipGraph;
 *   - return 0 on success or a negative sdk_status; sdk_last_error() returns a
 *     thread-local message for the last failure.
 */
#ifndef SDK_AMD_H
#define SDK_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* sdk_stream_t;

enum sdk_status {
  SDK_OK = 0,
  SDK_EINVAL = -1,      /* bad shape / pointer / alignment */
  SDK_EHIP = -2,        /* HIP launch error */
  SDK_EWORKSPACE = -3   /* workspace too small */
};

/* ---------------------------------------------------------------- convolution / GEMM
 * Implicit-GEMM convolution on MFMA (v_mfma_f32_32x32x16_f16, fp32 accumulate).
 * out[m, n] = sum_k A[m, k] * W[n, k]  (+ bias[n] + row_bias[b(m), n]) (+ residual[m, n])
 * where A is the im2col view of up to two K segments.  Each segment reads one
 * or two NHWC sources (a channel concat, zero-copy), optionally through a
 * GroupNorm affine (per (batch, channel) scale/shift) and SiLU, optionally
 * nearest-x2 upsampled, with zero padding applied AFTER the transform.
 * A plain Linear on tokens is the 1x1 case with h = tokens, w = 1.
 *
 * Replaces: nn.Conv2d 3x3/1x1/s2 (openai_model/utils.py:26-39 via model.py:117,181,207,218,365,531,88-90;
 *   Unet/unet.py:84-112; Encoder_Decoder/encoder.py:133,171), nn.Linear
 *   (openai_model/attention.py:40-47,133,164-168; model.py:197-200,352-357), the
 *   GroupNorm32/Normalize + SiLU in front of them (openai_model/utils.py:15-22,
 *   attention.py:10-11, Unet/unet.py:9-28), F.interpolate nearest x2 (model.py:127,
 *   Unet/unet.py:46), torch.cat skip concat (model.py:586), the emb broadcast add
 *   (model.py:241-250), the residual adds (model.py:252, attention.py:251-253,363,
 *   Unet/unet.py:135, Unet/attention.py:264) and GEGLU x*gelu(gate) (attention.py:140-141).
 */
typedef struct {
  const void* src0;        /* NHWC fp16, channels [0, c_split) */
  const void* src1;        /* NHWC fp16, channels [c_split, cin) (NULL if c_split == cin) */
  int32_t c_split;         /* multiple of 8 */
  int32_t cin;             /* multiple of 8 */
  int32_t ld0, ld1;        /* elements between consecutive pixels of src0 / src1 */
  int32_t h, w;            /* source spatial size (before upsampling) */
  int32_t ksize;           /* 1 or 3 */
  int32_t stride, pad;
  int32_t upsample;        /* 1: source is read nearest-x2 upsampled (logical 2h x 2w) */
  const float* gn_scale;   /* [batch][cin] or NULL */
  const float* gn_shift;   /* [batch][cin] or NULL */
  int32_t silu;            /* apply x*sigmoid(x) after the affine */
  int32_t pad_end;         /* extra zero rows/cols after the source (bottom/right) on top of pad:
                              the KL-VAE Downsample's F.pad(x, (0,1,0,1)) + conv s2 p0 (Unet/unet.py:64-68) */
} sdk_conv_src;

enum sdk_out_mode {
  SDK_OUT_NHWC_F16 = 0,    /* out[m*out_ld + n] fp16 */
  SDK_OUT_NCHW_F32 = 1,    /* out[(b*cout + n)*ho*wo + pix] fp32 */
  SDK_OUT_GEGLU_F16 = 2,   /* weight rows packed in 32-row (x, gate) pairs; out width cout/2 */
  SDK_OUT_ROWS_F32 = 3     /* out[m*out_ld + n] fp32 */
};

typedef struct {
  int32_t batch, ho, wo, cout;
  int32_t nseg;            /* 1 or 2 (segment 1 = fused 1x1 shortcut) */
  sdk_conv_src seg[2];
  const void* weight;      /* fp16 [cout_pad][k_total]; cout_pad = roundup(cout, 128);
                              per segment: roundup(cin, 64) / 64 channel blocks x taps x 64
                              columns (channel-block major, tap minor) */
  int32_t k_total;
  const float* bias;       /* [cout] or NULL */
  const float* row_bias;   /* [batch][row_bias_ld] or NULL (timestep-embedding broadcast) */
  int32_t row_bias_ld;
  const void* residual;    /* fp16 [M][res_ld] or NULL */
  int32_t res_ld;
  void* out;
  int32_t out_ld;
  int32_t out_mode;        /* enum sdk_out_mode */
  int32_t split_k;         /* 0 = choose; 1 = off */
  float* workspace;        /* split-K fp32 partials */
  int64_t workspace_bytes;
  int32_t variant_hint;    /* 0 = choose; 1 + variant id forces a tile configuration (autotuning) */
  int32_t act;             /* enum sdk_conv_act: applied after bias / row_bias, before the residual */
  float* gn_partial;       /* NULL, or GroupNorm statistics of the fp16 NHWC output (only when the plan's
                              gn_chunks > 0): [batch][gn_chunks][cout] float pairs (mean, M2) over
                              ho*wo/gn_chunks output pixels each — sdk_group_norm merges them instead of
                              a statistics pass over the tensor */
  int64_t weight_batch_stride;  /* 0, or per-image weights: output rows of image b (b = m / (ho*wo)) use
                                   weight + b * weight_batch_stride (elements); only the LDS-DMA tile
                                   kernels, with M-tiles inside one image (the reassociated
                                   cross-attention's per-prompt matrices) */
  int32_t split_inlaunch;  /* 1: split_k must be 2 and the plan an LDS-DMA tile kernel; the two K halves of a
                              tile are combined INSIDE the launch (each writes its fp32 accumulator blob to the
                              workspace; the second to arrive adds the first's and runs the full epilogue,
                              GroupNorm statistics included): no reduce kernel, no slab round trip through it */
  uint32_t* tile_counters; /* with split_inlaunch: >= SDK_TILE_COUNTERS zero-initialised words, one arrival
                              counter per output tile (device memory); every launch leaves them zero */
  int32_t tile_group_m;    /* unsplit LDS-DMA / phased plans: output tiles are visited in groups of this
                              many M-panels, N-tile major inside a group, so the tiles co-resident on one XCD
                              share both their A panels and their W tiles in its L2; 0: the library's choice,
                              1: M-panel major (every N-tile of a panel, then the next panel) */
} sdk_conv_args;

#define SDK_TILE_COUNTERS 16384

enum sdk_conv_act {
  SDK_ACT_NONE = 0,
  SDK_ACT_QUICK_GELU = 1   /* x * sigmoid(1.702 x): CLIP MLP fc1 (transformers QuickGELUActivation) */
};

typedef struct {
  int32_t split_k;
  int32_t grid_tiles;
  int64_t workspace_bytes;
  int32_t variant;         /* kernel variant id (sdk_kernel_name); split_k > 1 adds splitk_reduce_kernel */
  double flops;            /* algorithmic 2*M*N*K over the unpadded K */
  int32_t gn_chunks;       /* > 0: the plan can emit GroupNorm statistics (sdk_conv_args.gn_partial) */
} sdk_conv_plan_info;

int sdk_conv2d_plan(const sdk_conv_args* a, sdk_conv_plan_info* info);
int sdk_conv2d(const sdk_conv_args* a, sdk_stream_t stream);

/* ---------------------------------------------------------------- GroupNorm statistics
 * Per (batch, group) mean / variance over an NHWC tensor (optionally a 2-source
 * channel concat), folded with gamma/beta into per (batch, channel)
 * scale = gamma*rstd, shift = beta - mean*gamma*rstd consumed by sdk_conv2d.
 * Replaces the statistics half of GroupNorm32 (openai_model/utils.py:15-22, eps 1e-5),
 * Normalize (openai_model/attention.py:10-11; Unet/unet.py:9-19, eps 1e-6) and
 * FlashAttentionBlock.norm (Unet/attention.py:231, eps 1e-5).
 */
typedef struct {
  const void* src0; const void* src1;
  int32_t c_split, ld0, ld1;
  int32_t batch, hw, channels, groups;
  float eps;
  const float* gamma; const float* beta;   /* [channels] */
  float* scale; float* shift;              /* [batch][channels] */
  float* workspace; int64_t workspace_bytes;
} sdk_group_norm_args;

int64_t sdk_group_norm_workspace(int32_t batch, int32_t hw, int32_t channels);
int sdk_group_norm_affine(const sdk_group_norm_args* a, sdk_stream_t stream);

/* y = silu?(x*scale + shift) with the scale/shift of sdk_group_norm_affine; writes the
 * (possibly 2-source) input contiguous [batch*hw][ld_y].  Used in front of 3x3 convs,
 * where a per-tap prologue would repeat the transform 9x (GroupNorm32 + nn.SiLU,
 * openai_model/model.py:178-181,202-205,528-530; Unet/unet.py:116-125; encoder.py:205-206). */
int sdk_group_norm_apply(const sdk_group_norm_args* a, int32_t silu, void* y, int32_t ld_y, sdk_stream_t stream);

/* The same, written into a zero-bordered image y [batch][h+2*pad][w+2*pad][ld_y] (h*w == hw): the
 * 3x3 conv that consumes it runs with pad 0, so its implicit-GEMM gather has every tap in range
 * (no per-tap masks — the zero padding of nn.Conv2d(padding=1) is stored, not computed). */
int sdk_group_norm_apply_padded(const sdk_group_norm_args* a, int32_t silu, void* y, int32_t ld_y, int32_t h,
                                int32_t w, int32_t pad, sdk_stream_t stream);

/* GroupNorm (+ SiLU) end to end — the whole GroupNorm32 / Normalize module + nn.SiLU of the call
 * sites above: y = silu?(x*scale + shift) into y [batch][h+2*pad][w+2*pad][ld_y] (pad 0: contiguous).
 * Statistics: merged from the per-chunk channel statistics the producing sdk_conv2d emitted
 * (sdk_conv_args.gn_partial; part0 = source 0's [batch][nch0][c_split], part1 = source 1's
 * [batch][nch1][channels - c_split] for a concat; NULL = none), else computed from x (one fused
 * statistics + apply launch at hw <= 64).  a->scale / a->shift / a->workspace as for
 * sdk_group_norm_affine (the fused launch does not touch them). */
int sdk_group_norm(const sdk_group_norm_args* a, int32_t silu, void* y, int32_t ld_y, int32_t h, int32_t w,
                   int32_t pad, const float* part0, int32_t nch0, const float* part1, int32_t nch1,
                   sdk_stream_t stream);

/* The statistics half of sdk_group_norm alone: a->scale / a->shift [batch][channels] of the
 * GroupNorm affine, merged from the producers' per-chunk statistics (part0 / part1 as above) or, with
 * none, computed from x (sdk_group_norm_affine).  For a conv that applies GroupNorm + SiLU to its own
 * A operand (sdk_conv_src.gn_scale / gn_shift / silu), so the normalised tensor is never written: only
 * variant 0, the register-staged kernel, takes the GroupNorm scale / shift prologue; variant 35 (skinny)
 * is planned only without gn_scale and applies SiLU alone. */
int sdk_group_norm_finalize(const sdk_group_norm_args* a, const float* part0, int32_t nch0, const float* part1,
                            int32_t nch1, sdk_stream_t stream);

/* The post-activation GroupNorm of the DDPM (config C1) UNet (DDPM/models/layers.py:23-38 ConvBlock,
 * :311-338 ResNetBlock, :154 attention post-norm): y = [silu](x*scale + shift) + post_bias[b][c]
 * (the time embedding added after block1) + residual[pix][c] (the ResNet skip); both optional. */
int sdk_group_norm_apply_ex(const sdk_group_norm_args* a, int32_t silu, const float* post_bias, int32_t pb_ld,
                            const void* residual, int32_t res_ld, void* y, int32_t ld_y, sdk_stream_t stream);

/* ---------------------------------------------------------------- device calibration probes
 * Not on the sampling path: measure, on the box the bench runs on, the dense fp16 MFMA rate held
 * under load (back-to-back v_mfma_f32_16x16x32_f16 (m16 = 1) or 32x32x16 on random register
 * operands, `blocks` workgroups of 4 waves, `iters` iterations; seed = 32768 random fp16, sink =
 * blocks*4 floats) and the HBM copy rate, next to the spec peaks the roofline is quoted against.
 */
double sdk_probe_mfma_flops(int32_t m16, int32_t blocks, int32_t iters);
int sdk_probe_mfma(int32_t m16, int32_t blocks, int32_t iters, const void* seed, float* sink, sdk_stream_t stream);
int sdk_probe_copy(const void* src, void* dst, int64_t bytes, sdk_stream_t stream);
/* the copy with its shape chosen: mode bit 0 = 8 loads in flight per thread (else 4), bit 1 = non-temporal
   loads / stores, bits 2-7 = workgroups per CU (0: 16), bit 8 = one pass with a grid covering the buffer
   (each workgroup one contiguous chunk; bits 2-7 ignored); sdk_probe_copy is mode 0 */
int sdk_probe_copy_ex(const void* src, void* dst, int64_t bytes, int32_t mode, sdk_stream_t stream);

/* ---------------------------------------------------------------- LayerNorm
 * y = (x - mean) * rstd * gamma + beta over the last dim, fp16 in/out, fp32 math; gamma / beta fp32,
 * 16-byte aligned; cols a multiple of 8, <= 2048.
 * Replaces nn.LayerNorm norm1/2/3 (openai_model/attention.py:216-218,251-253).
 */
int sdk_layer_norm(const void* x, void* y, int32_t rows, int32_t cols, int32_t ld_x, int32_t ld_y,
                   const float* gamma, const float* beta, float eps, sdk_stream_t stream);

/* ---------------------------------------------------------------- attention
 * O = softmax(scale * Q K^T) V per (batch, head), non-causal, fp16 in/out, fp32
 * softmax; flash-style (online softmax, scores never leave the CU).
 * q/k/v/o are token-major: element (b, token, head, d) at ptr[(b*n + token)*ld + head*head_dim + d].
 * Replaces flash_attn_func (openai_model/attention.py:106-112; Unet/attention.py:257)
 * and flash_attn_qkvpacked_func (openai_model/attention.py:389-394,516-521).
 */
typedef struct {
  const void* q; const void* k; const void* v; void* o;
  int32_t q_ld, k_ld, v_ld, o_ld;
  int32_t batch, heads, nq, nk, head_dim;
  float scale;
  int32_t causal;          /* 1: key j is masked for query i when j > i (CLIP text encoder) */
} sdk_attention_args;

int sdk_attention(const sdk_attention_args* a, sdk_stream_t stream);

/* Fused cross-attention block on a cached context K|V: out = (softmax(scale * (t Wq^T)_h K_h^T) V_h)_h
 * Wo^T + bias + res, one kernel, q and o kept in LDS.  Replaces, per denoising step, the
 * to_q Linear + flash_attn_func + to_out Linear of CrossAttention.forward with a context
 * (openai_model/attention.py:63-117) and the residual add of BasicTransformerBlock
 * (attention.py:249).  t / res / out: [batch*n_img, ld] fp16; kv: [batch*nk, kv_ld] fp16
 * with K at columns [0, channels) and V at [channels, 2*channels); wq / wo: fp16 [>= channels
 * rows][w_ld = channels] (row n = output channel), or w_ld = 0: both in the fragment-packed layout of
 * sdk_xattn_pack_weight (channels * channels fp16, one contiguous KiB per MFMA fragment: whole-line weight
 * fetches); bias fp32 [channels] or NULL.
 * Shapes: sdk_cross_attention_block_supported() (channels 320 / 640, head_dim 40 / 64 / 80,
 * nk <= 80, n_img % 64 == 0); others return SDK_EINVAL (callers use the three-launch path).
 */
typedef struct {
  const void* t; const void* kv; const void* wq; const void* wo; const float* bias; const void* res;
  void* out;
  int32_t t_ld, kv_ld, w_ld, res_ld, out_ld;
  int32_t batch, n_img, nk, channels, head_dim;
  float scale;
} sdk_xattn_args;

int sdk_cross_attention_block_supported(int32_t channels, int32_t head_dim, int32_t nk, int32_t n_img);
/* One-time pack of a projection weight (fp16 [channels rows][w_ld], nn.Linear layout) into packed
 * (channels * channels fp16, 16-B aligned, device) for sdk_xattn_args.w_ld = 0; channels 320 / 640. */
int sdk_xattn_pack_weight(const void* w, int32_t w_ld, void* packed, int32_t channels, sdk_stream_t stream);
int sdk_cross_attention_block(const sdk_xattn_args* a, sdk_stream_t stream);

/* The same block with BasicTransformerBlock's two LayerNorms around it fused in
 * (openai_model/attention.py:249-250: x = attn2(norm2(x), context) + x; ... ff(norm3(x))):
 *  - in_gamma != NULL: a->t holds norm2's INPUT (the token rows, normally a->res as well) and is
 *    normalised inside the kernel (eps in_eps, fp32 gamma / beta, 16-B aligned);
 *  - out_gamma != NULL: out_ln[M, out_ln_ld] = norm3(out) is written as well.
 * Both norms produce the same bits as sdk_layer_norm on the same rows.  Either may be NULL.
 */
typedef struct {
  const float* in_gamma; const float* in_beta; float in_eps;
  const float* out_gamma; const float* out_beta; float out_eps;
  void* out_ln; int32_t out_ln_ld;
} sdk_xattn_ln_args;

int sdk_cross_attention_block_ln(const sdk_xattn_args* a, const sdk_xattn_ln_args* ln, sdk_stream_t stream);

/* ---------------------------------------------------------------- segment softmax
 * p[m, h*seglen + j] = softmax_j(scale * s[m, h*seglen + j]) for each of nseg segments of a row (fp32 in,
 * fp16 out), columns [nseg*seglen, ld_p) of p written as zeros (the K padding of the GEMM that consumes
 * p).  The middle step of the reassociated cross-attention at the 1280-channel levels, where the
 * scores of all heads against the cached context come out of ONE GEMM with per-prompt weights
 * (K_h Wq_h per head, sdk_conv_args.weight_batch_stride) and the output of another (Wo_h V_h^T).
 * Replaces: the sim.softmax(dim=-1) of CrossAttention.forward (openai_model/attention.py:106-112, in
 * flash_attn_func at the call sites :216-257).  seglen <= 128. */
int sdk_segment_softmax(const float* s, int32_t ld_s, void* p, int32_t ld_p, int32_t rows, int32_t nseg,
                        int32_t seglen, float scale, sdk_stream_t stream);

/* ---------------------------------------------------------------- fused feed-forward
 * out[m] = res[m] + W2 (a * gelu(g)) + b2,  [a | g] = t[m] W1^T + b1  — the GEGLU FeedForward of
 * BasicTransformerBlock in ONE kernel (GEGLU -> Dropout(0) -> Linear, openai_model/attention.py:129-172,
 * called as x = self.ff(self.norm3(x)) + x at :253); the 4*channels-wide intermediate stays in registers.
 * Shapes: channels == 320 (SD's 64x64-level blocks), features (the GEGLU width, 4*channels in SD) a
 * multiple of 32 (sdk_ff_supported).  t / res / out: [rows, ld] fp16, 16-B aligned, ld % 8 == 0; res may
 * be NULL or alias out.  Weights go through a one-time pack: w1 fp16 [2*features][channels] (rows
 * [0, features) = a, [features, 2*features) = gate, as nn.Linear(channels, 2*features).weight), b1 fp32
 * [2*features] or NULL, w2 fp16 [channels][features] (nn.Linear(features, channels).weight) ->
 * `packed` (sdk_ff_packed_bytes bytes, 16-B aligned, device); b2 fp32 [channels] (16-B aligned) or NULL.
 */
typedef struct {
  const void* t; const void* res; void* out; const void* packed; const float* b2;
  int32_t t_ld, res_ld, out_ld;
  int32_t rows, channels, features;
} sdk_ff_args;

int sdk_ff_supported(int32_t channels, int32_t features);
int64_t sdk_ff_packed_bytes(int32_t channels, int32_t features);
int sdk_ff_pack(const void* w1, const float* b1, const void* w2, void* packed, int32_t channels, int32_t features,
                sdk_stream_t stream);
int sdk_feed_forward(const sdk_ff_args* a, sdk_stream_t stream);

/* ---------------------------------------------------------------- 320-channel token linear
 * out[m] = [res[m] +] x[m] W^T + b for the 64x64-level transformer blocks' 320 -> 320 projections:
 * SpatialTransformer.proj_in (openai_model/attention.py:293-300, a 1x1 conv = per-token linear) and the
 * self-attention's to_out with its residual (:203-206, x = attn1(norm1(x)) + x at :251).  W stays in
 * registers, the grid walks 32-token blocks (csrc/token.hip).  x / res / out: [rows, ld] fp16, 16-B
 * aligned, ld % 8 == 0; res may be NULL or alias out; x must not overlap out.  w fp16 [320][320]
 * (nn.Linear.weight: [out][in]), 16-B aligned; bias fp32 [320] (16-B aligned) or NULL.
 */
typedef struct {
  const void* x; const void* w; const float* bias; const void* res; void* out;
  int32_t x_ld, res_ld, out_ld;
  int32_t rows, in_features, out_features;
} sdk_token_linear_args;

int sdk_token_linear_supported(int32_t in_features, int32_t out_features);
int sdk_token_linear(const sdk_token_linear_args* a, sdk_stream_t stream);

/* The same projection, also writing out_ln[m] = LayerNorm(out[m]) (fp32 gamma / beta [320], 16-B aligned;
 * the same bits as sdk_layer_norm on out): SpatialTransformer.proj_in followed by the first
 * BasicTransformerBlock's norm1 (openai_model/attention.py:330 then :251, x = attn1(norm1(x)) + x), one
 * launch instead of two.  out_ln [rows, out_ln_ld] must not overlap x, res or out. */
int sdk_token_linear_ln(const sdk_token_linear_args* a, const float* gamma, const float* beta, float eps,
                        void* out_ln, int32_t out_ln_ld, sdk_stream_t stream);

/* ---------------------------------------------------------------- sampler / glue
 * DDIM update (DDIM/ddim.py:194-204 == ldm/diffusion/ddim.py:197-205), fp32,
 * evaluated op by op without contraction so it is bit-identical to torch's CPU
 * kernels on the same inputs.  Optional fused classifier-free guidance
 * (ddim.py:171-178: e = e_u + g*(e_c - e_u)) and v-prediction (extension: e =
 * sqrt(a)*v + sqrt(1-a)*x).
 */
typedef struct {
  const float* x; const float* e; const float* e_uncond; const float* noise;
  float* x_prev; float* pred_x0;
  int64_t n;
  float sqrt_one_minus_at, sqrt_at, dir_coef, sqrt_a_prev, sigma, temperature;
  float guidance;          /* used when e_uncond != NULL */
  int32_t v_param;         /* 1: e holds v; convert with v_sqrt_a / v_sqrt_1ma */
  float v_sqrt_a, v_sqrt_1ma;
} sdk_ddim_args;

int sdk_ddim_step(const sdk_ddim_args* a, sdk_stream_t stream);

/* DDPM ancestral update (DDPM/ddpm.py:84-86):
 * x = inv_sqrt_alpha*(x - coef*eps) + sigma*noise. */
int sdk_ddpm_step(const float* x, const float* eps, const float* noise, float* out, int64_t n,
                  float inv_sqrt_alpha, float coef, float sigma, sdk_stream_t stream);

/* Sinusoidal timestep embedding cat[cos(t*f), sin(t*f)] -> fp16 (openai_model/utils.py:225-245;
 * the reference feeds time_embed with t_emb.half(), model.py:566). */
int sdk_timestep_embedding(const int64_t* t, const float* freqs, void* out, int32_t batch, int32_t dim,
                           sdk_stream_t stream);

/* NCHW fp32 -> NHWC fp16 with channel zero-padding to c_pad and a scalar pre-scale
 * (x.type(dtype), model.py:572; 1/scale_factor*z, ldm/diffusion/ddpm.py:1095). */
int sdk_nchw_to_nhwc(const float* x, void* y, int32_t batch, int32_t channels, int32_t hw, int32_t c_pad,
                     float scale, sdk_stream_t stream);

/* KL posterior sample scaled into the diffusion latent space:
 * z = scale * (mean + exp(0.5 * clamp(logvar, -30, 20)) * noise), or scale * mean when noise is NULL
 * (the posterior mode).  moments: NCHW fp32 [batch][2*channels][hw] (mean | logvar, the quant_conv
 * output), z: [batch][channels][hw].  Replaces DiagonalGaussianDistribution.sample/mode
 * (Distribution/distribution.py:31-50) + get_first_stage_encoding's scale (ldm/diffusion/ddpm.py:795-806). */
int sdk_diag_gaussian_sample(const float* moments, const float* noise, float* z, int32_t batch, int32_t channels,
                             int32_t hw, float scale, sdk_stream_t stream);

/* DDIM stochastic encode (ldm/diffusion/ddim.py:209-222 == DDIM/ddim.py:207-220) for one timestep:
 * out = sqrt_a * x0 + sqrt_1ma * noise, two correctly-rounded products and a sum (no contraction),
 * bit-identical to torch's CPU evaluation of the reference expression. */
int sdk_stochastic_encode(const float* x0, const float* noise, float* out, int64_t n, float sqrt_a,
                          float sqrt_1ma, sdk_stream_t stream);

/* Token + position embedding of the CLIP text transformer (transformers CLIPTextEmbeddings,
 * called by FrozenCLIPEmbedder.forward, clip_encoder/modules.py:241-256):
 * out[b][t][:] = fp16(tok[ids[b][t]][:] + pos[t][:]), fp32 tables [vocab][dim] / [>= seq][dim].
 * Ids outside [0, vocab) are an error (reported through sdk_last_error after the launch
 * is skipped: the ids are checked on the host by the caller). */
int sdk_token_embedding(const int64_t* ids, const float* tok, const float* pos, void* out, int32_t batch,
                        int32_t seq, int32_t dim, sdk_stream_t stream);

/* Tiled first-stage decode (ldm/diffusion/ddpm.py:1097-1139 with
 * get_fold_unfold / get_weighting / delta_border :829-997, CompVis semantics — see DESIGN.md Q14):
 * extract: latent NCHW fp32 [batch][channels][h][w] -> patches [L][batch][channels][kh][kw],
 *   L = Ly*Lx, Ly = (h-kh)/sy + 1, patch l = ly*Lx + lx (torch.nn.Unfold order);
 * fold: decoded patches [L][batch][channels][ph][pw] -> out [batch][channels][h][w] =
 *   sum_l w*patch / sum_l w with w = pix_w[i][j] * l_w[l] (l_w may be NULL), the per-pixel
 *   normalised overlap-add that Fold(o*weighting) / Fold(weighting) computes. */
int sdk_extract_patches(const float* z, float* out, int32_t batch, int32_t channels, int32_t h, int32_t w,
                        int32_t kh, int32_t kw, int32_t sy, int32_t sx, sdk_stream_t stream);
int sdk_fold_patches(const float* patches, const float* pix_w, const float* l_w, float* out, int32_t batch,
                     int32_t channels, int32_t h, int32_t w, int32_t ph, int32_t pw, int32_t sy, int32_t sx,
                     int32_t ly, int32_t lx, sdk_stream_t stream);

/* DDPM (C1) UNet glue: F.interpolate(x2, bilinear, align_corners=True) on NHWC fp16
 * (DDPM/models/layers.py:55-66 UpsampleBlock) and the exact GELU of its time MLP (unet.py:27-32). */
int sdk_upsample_bilinear2x(const void* x, void* y, int32_t batch, int32_t h, int32_t w, int32_t channels,
                            sdk_stream_t stream);
int sdk_gelu(const void* x, void* y, int64_t n, sdk_stream_t stream);

/* UNet Upsample (openai_model/model.py:120-131: F.interpolate(x, scale_factor=2, mode="nearest") then
 * conv3x3 with padding `pad`): y = [batch][2h + 2pad][2w + 2pad][channels] fp16, the nearest-x2 image with a
 * zero border of `pad`, for an unmasked (pad 0) sdk_conv2d.  x rows have stride ld_x (halfs). */
int sdk_upsample_nearest2x_padded(const void* x, int32_t ld_x, void* y, int32_t batch, int32_t h, int32_t w,
                                  int32_t channels, int32_t pad, sdk_stream_t stream);

/* ---------------------------------------------------------------- introspection */
const char* sdk_last_error(void);
int sdk_version(void);
const char* sdk_kernel_name(int32_t variant);

#ifdef __cplusplus
}
#endif
#endif /* SDK_AMD_H */
