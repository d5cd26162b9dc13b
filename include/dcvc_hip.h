/*
 * dcvc_hip.h — C ABI of the gfx950 kernels (libdcvc_hip.so).
 *
 * The reference has no kernels of its own: its hot path is stock ATen ops
 * driven by nn.Modules.  Each entry point here replaces one
 * family of those ops as the reference uses them, fused with the elementwise
 * work around it; the citation on each names the reference call sites.
 *
 * Conventions
 *   - Activations are NHWC, batch 1, in HBM.  A tensor argument is a base
 *     pointer plus (cstride, coff): element (y, x, c) lives at
 *     base[(y * W + x) * cstride + coff + c].  Writing a conv's output at a
 *     channel offset of a wider buffer is how torch.cat is expressed.
 *   - dtype codes: DCVC_F32 (float) or DCVC_BF16 (bfloat16 stored as uint16).
 *   - Every call is asynchronous on the given hipStream_t (passed as void*).
 *   - Returns DCVC_HIP_OK or a negative code; shapes are validated on the
 *     host before launch so a bad call never reaches the GPU.
 */
#ifndef DCVC_HIP_H
#define DCVC_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCVC_HIP_OK 0
#define DCVC_HIP_EINVAL (-1)
#define DCVC_HIP_ELAUNCH (-2)
#define DCVC_HIP_EUNSUPPORTED (-3)

enum dcvc_dtype { DCVC_F32 = 0, DCVC_BF16 = 1 };
/* Conv compute type (dcvc_conv_args.compute) beside DCVC_F32 / DCVC_BF16:
 * fp32 operands split into two fp16 values each (x = hi + 2^-11 lo) and
 * multiplied as xh*wh + 2^-11 (xh*wl + xl*wh) on f16 MFMA with fp32
 * accumulation (~2^-21 relative operand error); fp32 input and output views. */
#define DCVC_F16X3 2

enum dcvc_act {
  DCVC_ACT_NONE = 0,
  DCVC_ACT_LRELU = 1,   /* x >= 0 ? x : slope * x (ReLU is slope 0)      */
  DCVC_ACT_CLAMP01 = 2, /* clamp to [0, 1] (x_hat.clamp_(0, 1))          */
  DCVC_ACT_ROUND = 3    /* round half to even (torch.round of z)         */
};

/* Input transform applied while staging the conv input tile. */
enum dcvc_in_op {
  DCVC_IN_NONE = 0,
  DCVC_IN_LRELU = 1, /* lrelu(x, in_slope): ResBlock.first_layer          */
  DCVC_IN_GATE = 2   /* x[c] * lrelu(x[c + Cin], in_slope): ConvFFN2 gate */
};

typedef struct dcvc_tensor {
  void *ptr;
  int dtype;   /* dcvc_dtype */
  int H, W, C; /* logical shape of the view */
  int cstride; /* channels of the underlying buffer */
  int coff;    /* channel offset of the view */
} dcvc_tensor;

/*
 * Dense / strided 2-D convolution as an implicit GEMM on MFMA.
 * Replaces nn.Conv2d calls of the hot path (kernel 1/2/3/7, stride 1/2,
 * padding (k-1)//2, groups 1): every conv in DCVC-DC/src/models/video_net.py,
 * layers.py, video_model.py, image_model.py except the depthwise and grouped
 * ones.  Fused: input transform (in_op), bias, activation, residual add(s),
 * per-output-channel scale (the `* quant_step` multiplies), pixel shuffle r=2
 * on store (subpel_conv*), output dtype conversion.
 *   out = scale[c] * (res2 + (res + act(conv(in_op(x)) + bias)))
 * Weights are pre-packed by dcvc_conv_pack_weights.
 */
typedef struct dcvc_conv_args {
  dcvc_tensor x;
  dcvc_tensor y;          /* H, W = output size after shuffle; C = output channels after shuffle */
  const void *w;          /* packed weights (see dcvc_conv_pack_weights)   */
  const float *bias;      /* [Cout] or NULL                                */
  int cin, cout;          /* conv channels (cout before pixel shuffle)    */
  int kh, kw, stride, pad;
  int compute;            /* DCVC_BF16: bf16 MFMA, DCVC_F32: f32 MFMA,
                             DCVC_F16X3: split-fp16 MFMA (fp32 views)     */
  int in_op;              /* dcvc_in_op                                    */
  float in_slope;
  int act;                /* dcvc_act                                      */
  float slope;
  int shuffle;            /* 1: pixel_shuffle(2) on store                  */
  const float *scale;     /* per output channel (after shuffle) or NULL    */
  dcvc_tensor res;        /* ptr NULL when absent; same shape as y         */
  dcvc_tensor res2;       /* second residual, added after res              */
} dcvc_conv_args;

/* Pack reference-layout fp32 weights [Cout][Cin][kh][kw] (host pointer) into
 * the kernel layout [Cout][kh][kw][Cin_pad] (Cin_pad = Cin rounded up to 32)
 * in dtype `compute`, written to host buffer `out`.  Returns the number of
 * elements written (Cout*kh*kw*Cin_pad) or a negative code.
 * compute = DCVC_F16X3 writes uint16 fp16 halves in the split layout of
 * sconv.hip (per 32-channel chunk a hi and a lo block); out = NULL then
 * returns the element count without writing. */
int64_t dcvc_conv_pack_weights(const float *w, int cout, int cin, int kh,
                               int kw, int compute, void *out);
int dcvc_conv2d(const dcvc_conv_args *a, void *stream);
/* Runtime switches (testing / A-B): "gemm1x1" = 1 (default) routes 1x1
 * stride-1 bf16 convs to the double-buffered GEMM kernel; "conv3x3" = 1
 * (default) routes 3x3 stride-1 bf16 convs to the fixed-geometry kernels;
 * "conv3x3_resident" = 1 (default) prefers its persistent resident-weight
 * variant where the weights fit in LDS. */
int dcvc_set_option(const char *name, int value);
/* fp16 range guard of the split-fp16 kernels (compute DCVC_F16X3 and the fused
 * split blocks): a split operand carries an fp32 value v as hi + 2^-11 lo of two
 * fp16 numbers, to ~2^-21 of v while |v| < 2^15, and saturates silently above.
 * With `flag` (a device int32) set, every split kernel launched afterwards from
 * the calling host thread sets *flag = 1 when any value it splits (an input or
 * a fused intermediate) has |v| >= 2^15; the caller reads and clears it once per
 * frame and raises instead of returning an out-of-range result.  NULL (the
 * default) turns the guard off for the thread.  No reference counterpart: the
 * reference computes in fp32 (DCVC-DC/src/models/video_net.py, layers.py). */
int dcvc_split_range_flag(int *flag);
/* Kernel instantiation launched by the last dcvc_conv2d / dcvc_depthconv_block
 * call on the calling host thread, spelled as rocprofv3 reports it, with the
 * grid size in work-items (e.g. "conv3x3_kernel<48, 16, false, unsigned
 * short>@2088960"); "" before any launch.  Used to match per-launch HIP-event
 * timings with rocprof kernel and PMC summaries. */
const char *dcvc_last_kernel(void);

/*
 * Fused DepthConvBlock (DepthConv + ConvFFN) / DepthConvBlock2 (+ ConvFFN2),
 * DCVC-DC/src/models/layers.py:135-222, for bf16 feature maps with
 * Cin, Cout <= 128: one kernel, all intermediates in LDS.  Weights are the
 * packed bf16 1x1 layouts of dcvc_conv_pack_weights ([N][ld], ld = K rounded
 * up to 32); the depthwise weights are [9][Cin] fp32.  w_adaptor NULL means
 * identity (Cin == Cout).  Returns DCVC_HIP_EUNSUPPORTED for shapes without
 * an instantiated kernel (the caller then runs the unfused sequence).
 */
typedef struct dcvc_dcb_args {
  dcvc_tensor x, y;
  int cin, cout, gated;
  const void *w_conv1; int ld_conv1; const float *b_conv1;
  const float *w_dw; const float *b_dw;
  const void *w_conv2; int ld_conv2; const float *b_conv2;
  const void *w_adaptor; int ld_adaptor; const float *b_adaptor;
  const void *w_ffn1; int ld_ffn1; const float *b_ffn1;
  const void *w_ffn2; int ld_ffn2; const float *b_ffn2;
  const float *scale;
  float slope_dc, slope_ffn;
} dcvc_dcb_args;
int dcvc_depthconv_block(const dcvc_dcb_args *a, void *stream);

/*
 * Fused ConvFFN in split-fp16 arithmetic (Precision.split()),
 * DCVC-DC/src/models/layers.py:166-179 with the DepthConvBlock's optional
 * output scale:  y = scale * (x + lrelu(ffn2(lrelu(ffn1(x) + b1)) + b2)),
 * lrelu slope `slope` (0.1), fp32 views of c channels (c in {32, 48, 64, 128},
 * hidden a multiple of 64, or of 32 for c = 128; and the entropy model's
 * latent widths c in {192, 384}, hidden a multiple of 64, whose weights are
 * packed as MFMA fragments streamed from L2, DCVC-DC/src/models/
 * video_model.py:250-305); the hidden layer never leaves the CU.
 * Weights packed by dcvc_ffn_pack_weights from w1 = conv.0
 * [hidden][c] and w2 = conv.2 [c][hidden] (fp32, host); out NULL returns the
 * element count.  DCVC_HIP_EUNSUPPORTED for other shapes (the caller runs
 * the two convs).
 */
typedef struct dcvc_ffn_args {
  dcvc_tensor x, y;
  int c, hidden;
  const void *w;
  const float *b1, *b2;
  const float *scale;     /* [c] or NULL */
  float slope;
} dcvc_ffn_args;
int64_t dcvc_ffn_pack_weights(const float *w1, const float *w2, int c, int hidden, void *out);
int dcvc_conv_ffn(const dcvc_ffn_args *a, void *stream);

/*
 * The tail of a latent DepthConv in split-fp16 arithmetic,
 * DCVC-DC/src/models/layers.py:135-163 for the adaptor-free C -> C blocks
 * of the entropy model (video_model.py:250-305, c in {192, 384}):
 *   y = conv2(dw3x3(t) + bdw) + b2 + r
 * t = lrelu(conv1(x) + b1) (the previous dcvc_conv2d), r = the block input.
 * w9 = depthwise taps [9][c] fp32 (tap (dy, dx) at (dy + 1) * 3 + dx + 1),
 * w2 = conv2 [c][c] packed by dcvc_frag_pack_weights (16 x 32 MFMA
 * fragments, hi and lo planes; out NULL returns the element count).
 * Replaces the depthwise launch and the conv2 launch of the unfused block
 * with identical results.  DCVC_HIP_EUNSUPPORTED for other widths.
 */
typedef struct dcvc_dwc_args {
  dcvc_tensor t, r, y;
  int c;
  const float *w9, *bdw;
  const void *w2;
  const float *b2;
} dcvc_dwc_args;
int64_t dcvc_frag_pack_weights(const float *w, int rows, int k, void *out);
int dcvc_dw_conv2_split(const dcvc_dwc_args *a, void *stream);

/*
 * Fused DepthConv in split-fp16 arithmetic (Precision.split()),
 * DCVC-DC/src/models/layers.py:135-163:
 *   y = conv2(dw3x3(lrelu(conv1(x) + b1, slope) + ...) + bdw) + b2 + identity,
 * identity = adaptor(x) + ba (adaptor != 0) or x; the depthwise conv zero-pads
 * t1 = lrelu(conv1(x) + b1).  fp32 views; (cin, cout) in {(64, 48), (48, 32),
 * (32, 64) with adaptor; (64, 64), (48, 48), (32, 32) without}.  Weights
 * packed by dcvc_dc_pack_weights from conv1 [cin][cin], conv2 [cout][cin] and
 * the adaptor [cout][cin] (NULL without); wdw [9][cin] (tap-major) fp32.
 */
typedef struct dcvc_dc_args {
  dcvc_tensor x, y;
  int cin, cout, adaptor;
  const void *w;
  const float *b1, *wdw, *bdw, *b2, *ba;
  float slope;
} dcvc_dc_args;
int64_t dcvc_dc_pack_weights(const float *w1, const float *w2, const float *wa, int cin, int cout, void *out);
int dcvc_depth_conv_split(const dcvc_dc_args *a, void *stream);

/* Depthwise 3x3 conv, stride 1, padding 1, + bias (DepthConv.depth_conv,
 * DCVC-DC/src/models/layers.py:143-144).  w: [9][C] fp32 (tap-major). */
int dcvc_dwconv3x3(dcvc_tensor x, dcvc_tensor y, const float *w,
                   const float *bias, void *stream);

/* Bilinear backward warp, grid_sample(bilinear, border, align_corners=True)
 * with the reference's cached fp32 linspace grid (torch_warp,
 * DCVC-DC/src/models/video_net.py:11-38).  flow: 2 channels fp32 (dx, dy) in
 * pixels; gx[W], gy[H]: the linspace grid values. */
int dcvc_flow_warp(dcvc_tensor x, dcvc_tensor flow, dcvc_tensor y,
                   const float *gx, const float *gy, void *stream);

/* OffsetDiversity after its conv stack (DCVC-DC/src/models/video_model.py:
 * 45-61): bilinear x2 upsample of the 96-channel offset map, 40*tanh offsets
 * + flow, sigmoid masks, 32 grouped warps of the 48-channel feature, mask
 * multiply and the grouped (16 groups) 1x1 fusion conv. fw: [48][6] fp32. */
int dcvc_offset_diversity(dcvc_tensor feat, dcvc_tensor offs_half,
                          dcvc_tensor flow, dcvc_tensor y, const float *fw,
                          const float *fb, const float *gx, const float *gy,
                          float max_mag, void *stream);

/* The same with a caller-provided device workspace of at least
 * dcvc_offset_diversity_workspace(H, W) bytes (16-byte aligned): fp32 maps
 * run the group-planar form (the feature copied to [16][H][W][3] in the
 * workspace, one group per wave), identical results; anything else runs
 * dcvc_offset_diversity. */
int64_t dcvc_offset_diversity_workspace(int H, int W);
int dcvc_offset_diversity_ws(dcvc_tensor feat, dcvc_tensor offs_half,
                             dcvc_tensor flow, dcvc_tensor y, const float *fw,
                             const float *fb, const float *gx, const float *gy,
                             float max_mag, void *workspace, int64_t ws_bytes,
                             void *stream);

/* Bilinear resize by 2 (up) or 1/2 (down), align_corners=False
 * (bilinearupsacling / bilineardownsacling, video_net.py:41-55), followed by
 * a multiply (flow * 2.0, mv / 2). */
int dcvc_resize2x(dcvc_tensor x, dcvc_tensor y, int up, float mul,
                  void *stream);
/* 2x2 stride-2 pooling: avg (ME_Spynet, video_net.py:112) or max (UNet). */
int dcvc_pool2x2(dcvc_tensor x, dcvc_tensor y, int is_max, void *stream);

/* Generic elementwise over a view: y = a (+ b) (* per-channel scale); or
 * a dtype-converting copy.  Used for the few cats / adds that are not
 * fused into a conv. */
int dcvc_add(dcvc_tensor a, dcvc_tensor b, dcvc_tensor y, void *stream);
int dcvc_copy(dcvc_tensor x, dcvc_tensor y, void *stream);
/* Replicate pad / crop of a view into y (pad_for_y / slice_to_y and the
 * harness's F.pad(replicate), common_model.py:70-86, test_video.py:130). */
int dcvc_pad_replicate(dcvc_tensor x, dcvc_tensor y, void *stream);
/* uint8 CHW frame -> float NHWC /255 with replicate padding to y's size. */
int dcvc_frame_to_nhwc(const uint8_t *src, int h, int w, dcvc_tensor y,
                       void *stream);
/* Same with zero padding: DCVC-HEM's harness pads frames with zeros to a
 * multiple of 64 (DCVC-HEM/test_video.py:113-119, F.pad mode="constant"). */
int dcvc_frame_to_nhwc_zero_pad(const uint8_t *src, int h, int w, dcvc_tensor y,
                                void *stream);
/* YUV420 source frame (uint8 Y h x w, then U and V h/2 x w/2, the YUVReader
 * layout, DCVC-DC/src/utils/video_reader.py:121-161) -> fp32 NHWC YCbCr 4:4:4
 * in [0, 1], replicate-padded to out's size.  Chroma is upsampled as
 * ycbcr420_to_444(order=0) does it (scipy.ndimage.zoom nearest,
 * DCVC-DC/src/transforms/functional.py:61-72; test_video.py:111-112).  h, w
 * even. */
int dcvc_yuv420_to_nhwc(const uint8_t *y, const uint8_t *uv, int h, int w,
                        dcvc_tensor out, void *stream);
/* Bytes of device workspace dcvc_frame_sse needs. */
int64_t dcvc_frame_sse_workspace(void);
/* run_test's per-frame distortion (DCVC-DC/test_video.py:169-195): clamps
 * x_hat (fp32 NHWC, 3 ch, padded) to [0, 1] IN PLACE, as recon_frame.clamp_
 * does to the DPB frame, then writes to out3 (device, fp64) the squared-error
 * sums over the top-left h x w crop against the uint8 source:
 *   yuv420 = 0: per RGB channel, fp32 difference and square (PSNR(),
 *               test_video.py:65-68); src = uint8 CHW, uv unused;
 *   yuv420 = 1: Y, U, V of ycbcr444_to_420(x_hat) (functional.py:75-95)
 *               against src = Y plane and uv = U|V planes, fp64 as calc_psnr
 *               (src/utils/metrics.py:81-92).
 * Summation order is fixed (deterministic). */
int dcvc_frame_sse(dcvc_tensor x_hat, const uint8_t *src, const uint8_t *uv,
                   int h, int w, int yuv420, double *workspace, double *out3,
                   void *stream);
/* The decoded frame as run_test's --save_decoded_frame writers store it
 * (DCVC-DC/src/utils/video_writer.py:26-111, DCVC-HEM/test_video.py:68-71):
 * the top-left h x w crop of x_hat (fp32 NHWC, 3 ch) quantised as
 * clip(rint(v * 255), 0, 255) in fp32, into out (device uint8):
 *   yuv420 = 0: h x w x 3 interleaved (PNGWriter / save_torch_image);
 *   yuv420 = 1: Y plane (h x w) then U, V planes (h/2 x w/2) of
 *               ycbcr444_to_420(clip(x_hat)) (YUVWriter), h and w even. */
int dcvc_recon_to_u8(dcvc_tensor x_hat, int h, int w, int yuv420, uint8_t *out,
                     void *stream);

/*
 * Quadtree (four-part) prior step k, encoder side
 * (forward_four_part_prior write=True, DCVC-DC/src/models/common_model.py:
 * 142-252).  y: latent (C ch, fp32); params: common_params (3C ch:
 * quant_step | scales | means); sm: step scales|means (2C ch) for k > 0
 * (NULL ptr for k = 0: scales/means come from params).  For the positions of
 * step k writes: symbols/indexes (int16, NCHW order of the C/4-channel y_q_w_k
 * tensor, symbols clamped to +-30000) for the coder; y_hat_so_far values
 * (y_q + means) into yhs (C ch); y_hat * quant_step into yhat (C ch).
 * Index = build_indexes(scales) with (log_min, log_step).
 */
int dcvc_quadtree_encode_step(dcvc_tensor y, dcvc_tensor params,
                              dcvc_tensor sm, int k, dcvc_tensor yhs,
                              dcvc_tensor yhat, int16_t *symbols,
                              int16_t *indexes, float log_min, float log_step,
                              void *stream);
/* Decoder side, phase 1: indexes of step k (decompress_four_part_prior
 * scales_r, common_model.py:274-311). */
int dcvc_quadtree_indexes_step(dcvc_tensor params, dcvc_tensor sm, int k,
                               int16_t *indexes, float log_min,
                               float log_step, void *stream);
/* Decoder side, phase 2: scatter decoded symbols of step k. */
int dcvc_quadtree_decode_step(dcvc_tensor params, dcvc_tensor sm, int k,
                              const int16_t *symbols, dcvc_tensor yhs,
                              dcvc_tensor yhat, void *stream);
/* Factorized-prior symbols (BitEstimator.encode, entropy_models.py:184-187):
 * NHWC float z_hat -> NCHW int16 (clamped +-30000); and the inverse. */
int dcvc_nhwc_to_symbols(dcvc_tensor x, int16_t *symbols, void *stream);
int dcvc_symbols_to_nhwc(const int16_t *symbols, dcvc_tensor y, void *stream);

/*
 * Estimate mode (forward_one_frame), the bit counts the reference computes
 * instead of coding (DCVC-DC/src/models/common_model.py:39-61,
 * video_model.py:559-628, image_model.py:116-147).
 * dcvc_quadtree_estimate_step: step k of forward_four_part_prior
 * (common_model.py:142-252, write=False) — the y_hat outputs of
 * dcvc_quadtree_encode_step plus, per coded element (same order as its
 * symbols), bits = probs_to_bits(cdf(y_q + 0.5) - cdf(y_q - 0.5)) with
 * sigma = clamp(scale, 1e-5, 1e10), Laplace (gaussian = 0, get_y_laplace_bits)
 * or Normal (gaussian = 1, get_y_gaussian_bits).
 */
int dcvc_quadtree_estimate_step(dcvc_tensor y, dcvc_tensor params,
                                dcvc_tensor sm, int k, dcvc_tensor yhs,
                                dcvc_tensor yhat, float *bits, int gaussian,
                                void *stream);
/* get_z_bits (common_model.py:59-61): per element of the NHWC z_hat (fp32),
 * bits of BitEstimator.get_cdf(z + 0.5) - get_cdf(z - 0.5) into bits[]
 * (NHWC order).  table: [C][11] fp32 = softplus(h1), b1, tanh(a1), ...,
 * softplus(h3), b3, tanh(a3), softplus(h4), b4 (entropy_models.py:56-122). */
int dcvc_factorized_bits(dcvc_tensor z, const float *table, float *bits,
                         void *stream);
/* Deterministic (fixed-order) sum of n device floats into *out (device). */
int dcvc_sum_f32(const float *x, int64_t n, float *out, void *stream);

/*
 * DCVC-HEM dual (checkerboard) prior, DCVC-HEM/src/models/common_model.py:
 * 84-188 (forward/compress/decompress_dual_prior).  buf: the spatial prior's
 * fp32 input [y_hat_0_0 | y_hat_1_1 (C) | means | scales | quant_step], 4C
 * channels, written by the caller's prior fusion (params) and by step 0
 * (y_hat part); sm: the spatial prior's output [scales_0 | means_0 |
 * scales_1 | means_1] for k = 1 (NULL ptr for k = 0).  Step k writes, per
 * site of its checkerboard half, int32 symbols / int16 CDF indexes in the
 * NCHW order of y_q_w_k (C/2 channels), and y_hat * quant_step into yhat.
 */
int dcvc_dual_prior_encode_step(dcvc_tensor y, dcvc_tensor buf, dcvc_tensor sm,
                                int k, dcvc_tensor yhat,
                                const float *post_scale, int32_t *symbols,
                                int16_t *indexes, float log_min,
                                float log_step, void *stream);
int dcvc_dual_prior_indexes_step(dcvc_tensor buf, dcvc_tensor sm, int k,
                                 int16_t *indexes, float log_min,
                                 float log_step, void *stream);
int dcvc_dual_prior_decode_step(dcvc_tensor buf, dcvc_tensor sm, int k,
                                const int32_t *symbols, dcvc_tensor yhat,
                                const float *post_scale, void *stream);
/* Estimate form (write=False): per-site bits, Laplace (gaussian = 0) or
 * Normal (gaussian = 1) with sigma clamped to [scale_min, 1e10]
 * (get_y_laplace_bits 1e-5 / get_y_gaussian_bits 0.11, common_model.py:58-70). */
int dcvc_dual_prior_estimate_step(dcvc_tensor y, dcvc_tensor buf,
                                  dcvc_tensor sm, int k, dcvc_tensor yhat,
                                  const float *post_scale, float *bits,
                                  int gaussian, float scale_min, void *stream);
/* post_scale (nullable, [C] fp32): yhat = (y_hat * quant_step) * post_scale,
 * the caller's y_hat * curr_q (video_model.py:278-279, 302-303) fused in. */
/* y[..] = value (a channel window of a concat buffer: the reference's
 * torch.zeros_like stand-ins for an absent ref_y / ref_mv_y). */
int dcvc_fill(dcvc_tensor y, float value, void *stream);
/* y = x / q[c], fp32 (y / curr_q, video_model.py:270, 289). */
int dcvc_channel_div(dcvc_tensor x, const float *q, dcvc_tensor y, void *stream);
/* HEM factorized symbols: int32, no clamp (BitEstimator.encode /
 * decode_stream, DCVC-HEM/src/entropy_models/entropy_models.py:182-195). */
int dcvc_nhwc_to_symbols_i32(dcvc_tensor x, int32_t *symbols, void *stream);
int dcvc_symbols_i32_to_nhwc(const int32_t *symbols, dcvc_tensor y,
                             void *stream);
/* SELayer (DCVC-HEM/src/models/video_net.py:157-170): scale_out[c] =
 * sigmoid(W2 relu(W1 mean_hw(x)))[c]; w1 [reduced][C], w2 [C][reduced]
 * fp32 (nn.Linear, no bias); work: >= 256 * C floats of device scratch. */
int dcvc_se_scale(dcvc_tensor x, const float *w1, const float *w2, int reduced,
                  float *work, float *scale_out, void *stream);
/* y = a + x * scale[c] (ConvBlockResidual: up_dim(x) + SE(x1),
 * video_net.py:185-188). */
int dcvc_se_apply(dcvc_tensor a, dcvc_tensor x, const float *scale,
                  dcvc_tensor y, void *stream);

/* MS-SSIM of the YUV420 path (calc_msssim, DCVC-DC/src/utils/metrics.py:15-62,
 * called per plane at test_video.py:182-184), fp64 as the reference computes
 * it.  dcvc_yuv_planes_f64 writes calc_msssim's inputs: the uint8/255 source
 * planes and the clamped recon's ycbcr444_to_420 planes of the h x w crop,
 * each as [Y h*w | U | V (h/2)*(w/2)] doubles.  dcvc_ssim_level writes to
 * out2 the means of calc_ssim's ssim and cs maps for two h x w planes
 * (11x11 'valid' Gaussian window `window121`, C1/C2 for data_range 1);
 * workspace: dcvc_ssim_workspace() bytes.  dcvc_down2_f64 is the
 * ndimage.convolve(ones(2,2)/4, mode='reflect')[::2, ::2] step between levels
 * (out: ceil(h/2) x ceil(w/2)).  The level loop and the final weighted
 * product run on the host. */
int dcvc_yuv_planes_f64(dcvc_tensor x_hat, const uint8_t *y, const uint8_t *uv,
                        int h, int w, double *src_planes, double *rec_planes,
                        void *stream);
int64_t dcvc_ssim_workspace(void);
int dcvc_ssim_level(const double *a, const double *b, int h, int w,
                    const double *window121, double C1, double C2,
                    double *workspace, double *out2, void *stream);
int dcvc_down2_f64(const double *in, int h, int w, double *out, void *stream);
/* RGB MS-SSIM (pytorch_msssim.ms_ssim, DCVC-DC/test_video.py:188,
 * DCVC-HEM/test_video.py:153; the package is absent here, so its published
 * algorithm is followed and the result is parity unpinned).
 * dcvc_rgb_planes_f64: the three fp64 source (uint8/255) and clamped recon
 * planes of the h x w crop; levels use dcvc_ssim_level and
 * dcvc_avgpool2_f64 = F.avg_pool2d(kernel 2, padding h%2 / w%2,
 * count_include_pad=True) (out: (h + 2(h%2) - 2)/2 + 1 rows). */
int dcvc_rgb_planes_f64(dcvc_tensor x_hat, const uint8_t *src, int h, int w,
                        double *src_planes, double *rec_planes, void *stream);
int dcvc_avgpool2_f64(const double *in, int h, int w, double *out, void *stream);

/* Debug aid: fill the LDS of `blocks` workgroups with all-ones bytes (NaN in
 * bf16 / fp32), to expose kernels that read LDS they never wrote
 * (scripts/lds_poison_check.py).  Not used by the codec. */
int dcvc_debug_poison_lds(int bytes, int blocks, void *stream);
/* Debug aid: fill the VGPRs of `blocks` 256-thread workgroups (120 VGPRs per
 * wave) with all-ones bits, to expose kernels that read registers they never
 * wrote.  Not used by the codec. */
int dcvc_debug_poison_vgpr(int blocks, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* DCVC_HIP_H */
