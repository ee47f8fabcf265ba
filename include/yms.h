/* yms.h -- C-ABI of the MI355X-native YOLO-MS / YOLOv8 detector hot path.
 *
 * Plain C, no torch types: raw device pointers, sizes and a hipStream_t passed as void*.
 * Every call is stream-ordered and asynchronous, allocates nothing (caller-owned outputs
 * and workspaces), is thread-compatible, and returns a status instead of throwing.
 *
 * Activation layout: NHWC.  A "view" of an activation is (ptr, ld, off): element
 * (n, y, x, c) lives at ptr[((n*H + y)*W + x)*ld + off + c].  ld and off are multiples of 8
 * elements; channels in [C, round_up(C,8)) of a buffer are kept zero by the producers.
 * dtype: YMS_F32 / YMS_BF16 / YMS_F16 for activations and packed weights; every
 * accumulation, BN statistic and parameter gradient is fp32.
 *
 * Reference interfaces each entry point replaces (paths relative to the reference repo
 * rafaelghiorzi/YOLO-MS):
 *   yms_conv_fwd            components.py:69-77 Conv.forward (Conv2d->BN->SiLU), the
 *                           Bottleneck residual add (:87-93), the C2f/SPPF/neck/head torch.cat
 *                           (:119, :146, yolov8_neck.py:79-91, yolov8_head.py:122) via y_off,
 *                           and the head's biased 1x1 nn.Conv2d (yolov8_head.py:86-109)
 *   yms_conv_dgrad/_wgrad   autograd of the above (train.py:371 loss.backward())
 *   yms_bn_*                components.py:73 nn.BatchNorm2d(eps=1e-3, momentum=0.03), train+eval
 *   yms_sppf_pool_*         components.py:136-146 three chained MaxPool2d(5,1,2)
 *   yms_upsample2x_*        components.py:153-160 Upsample (nearest x2)
 *   yms_head_decode         yolov8_head.py:127-158 make_anchors + DFL (components.py:162-191)
 *   yms_nms_*               train.py:63-113 / tools/test.py:166-218 post-process and the
 *                           torchvision.ops.nms(boxes, scores, iou) call at train.py:93
 */
#ifndef YMS_H
#define YMS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int yms_status;
#define YMS_OK 0
#define YMS_ERR_INVALID 1
#define YMS_ERR_UNSUPPORTED 2
#define YMS_ERR_LAUNCH 3

#define YMS_F32 0
#define YMS_BF16 1
#define YMS_F16 2

#define YMS_ACT_NONE 0
#define YMS_ACT_SILU 1

/* One convolution: input [n, h, w, cin] -> output [n, ho, wo, cout], square kernel k,
 * stride, pad (ho = (h + 2*pad - k)/stride + 1). */
typedef struct {
  int n, h, w, cin, cout, k, stride, pad, ho, wo, dtype;
} yms_conv_shape;

const char* yms_version(void);
/* A new stream restricted to ncus CUs (mode 0: lowest CU indices, 1: spread), for the backward's
 * weight-gradient side stream (hipExtStreamCreateWithCUMask).  *stream_out: hipStream_t. */
yms_status yms_stream_create_cu_subset(int ncus, int mode, void** stream_out);
const char* yms_status_string(yms_status s);

/* ---- weights ------------------------------------------------------------------------ */
/* Elements of the packed weight for the forward / dgrad GEMM (16-bit or fp32 per dtype). */
size_t yms_conv_packed_elems(const yms_conv_shape* s, int for_dgrad);
/* w: fp32 [cout][cin][k][k] (nn.Conv2d layout) -> packed dtype layout.
 * for_dgrad = 0: [cout_pad][K] with K = (kh, kw, cin_pad8) chunk order;
 * for_dgrad = 1: [cin_pad][K'] with K' = (kh, kw, cout_pad8). */
yms_status yms_conv_pack_weight(const yms_conv_shape* s, const float* w, void* packed,
                                int for_dgrad, void* stream);

/* Batched packing (one launch for all of a plan's packs; training repacks every step).
 * yms_pack_job_init fills a job on the host (YMS_ERR_UNSUPPORTED for stride-2 dgrad packs,
 * which keep yms_conv_pack_weight); the job array must be in device memory for the launch.
 * Each job's `packed` is taken as a byte offset from dst_base (dst_base NULL: absolute), so one
 * device job table serves every arena (and HIP-graph capture needs no host->device copy). */
typedef struct {
  const float* w;
  void* packed;
  int cout, cin, ks, rows, kp_elems, c8_in, for_dgrad, dtype;
  /* optional second source (sibling convs packed as one, yms_pack_job_init sets NULL / 0): output
   * channels co >= split read w2[co - split] instead of w[co] */
  const float* w2;
  int split;
} yms_pack_job;
yms_status yms_pack_job_init(const yms_conv_shape* s, const float* w, void* packed, int for_dgrad,
                             yms_pack_job* job);
yms_status yms_conv_pack_weights_batched(int njobs, const yms_pack_job* jobs_dev, void* dst_base, void* stream);

/* ---- convolution (implicit GEMM on MFMA) --------------------------------------------- */
/* Rows of BN partial statistics written by yms_conv_fwd(stats != NULL): fp32 -- one per 128
 * output pixels; bf16/f16 -- one per persistent block (and 128-row half of its tiles).  The stats
 * workspace is [rows][2][stats_ld] floats followed by [rows] float pixel counts (so
 * rows * (2*stats_ld + 1) floats), stats_ld = yms_conv_stats_ld(). */
int yms_conv_stats_rows(const yms_conv_shape* s);
int yms_conv_stats_ld(const yms_conv_shape* s);
/* Process-wide route switch of the direct small-channel 3x3 kernel (conv_direct.hip; default on,
 * YMS_DIRECT=0 in the environment at the first call turns it off).  on = 0 / 1 sets it, on < 0 only
 * queries; returns the previous setting.  It changes yms_conv_stats_rows, so callers flip it only
 * while no plan sized under the other setting is in use (tests and A/B runs). */
int yms_conv_direct_set(int on);
/* Forward.  stats == NULL: y = act(conv(x)*scale[c] + shift[c]) (+ res) (scale/shift may
 * be NULL = identity).  stats != NULL (training): y = conv(x) (pre-BN z) and statistics rows
 * (sum z, sum (z - row mean)^2, pixel count) into stats. */
yms_status yms_conv_fwd(const yms_conv_shape* s, const void* x, int x_ld, int x_off,
                        const void* wpacked, void* y, int y_ld, int y_off,
                        const float* scale, const float* shift, int act,
                        const void* res, int res_ld, int res_off, float* stats, void* stream);
/* Stem convolution (yolov8_backbone.py:30-40, the backbone's first Conv(cin, c1, 3, 2, 1), replacing
 * the NHWC input pack + yms_conv_fwd pair): x is the model's NCHW fp32 input [n][cin][h][w], w the
 * fp32 nn.Conv2d weight [cout][cin][3][3] (rounded to s->dtype in the kernel, as the packing
 * does).  Supported: yms_conv_stem_supported(s) (cin 1..3, k 3, stride 2, pad 1, cout % 8 == 0,
 * cout <= 96, bf16 / f16).  Same epilogues as yms_conv_fwd without the residual; statistics:
 * yms_conv_stem_stats_rows(s) rows (one per 8 x 32 output tile), counts after the rows. */
int yms_conv_stem_supported(const yms_conv_shape* s);
int yms_conv_stem_stats_rows(const yms_conv_shape* s);
yms_status yms_conv_stem_fwd(const yms_conv_shape* s, const float* x, const float* w, void* y, int y_ld,
                             int y_off, const float* scale, const float* shift, int act, float* stats,
                             int stats_ld, void* stream);
/* Stem weight gradient with the BN + SiLU backward apply fused in (the stem's dz has no other
 * consumer: the input needs no gradient): dz = scale*(da - coef[c] - (z - mean)*invstd*coef[C+c]),
 * da = gy * SiLU'(z*scale + shift) (act), rounded to s->dtype as the apply pass stores it; then
 * dw[cout][cin][3][3] (+)= sum_pixels dz (x) im2col(x), x the NCHW fp32 input as in
 * yms_conv_stem_fwd.  mean_invstd / coef as yms_bn_act_bwd_apply; ws >= yms_conv_stem_wgrad_ws_bytes. */
size_t yms_conv_stem_wgrad_ws_bytes(const yms_conv_shape* s);
yms_status yms_conv_stem_wgrad(const yms_conv_shape* s, const float* x, const void* gy, int gy_ld, int gy_off,
                               const void* z, int z_ld, int z_off, const float* scale, const float* shift,
                               const float* mean_invstd, const float* coef, int act, float* ws, size_t ws_bytes,
                               float* dw, int accumulate, void* stream);
/* dx (+)= conv_transpose(dz, W) with wpacked_t = yms_conv_pack_weight(.., for_dgrad=1). */
yms_status yms_conv_dgrad(const yms_conv_shape* s, const void* dz, int dz_ld, int dz_off,
                          const void* wpacked_t, void* dx, int dx_ld, int dx_off,
                          int accumulate, void* stream);
/* Input gradient with the PRODUCER's BN + act backward reduce fused into its epilogue: the producer
 * (components.py:69-77 Conv before this one) wrote this conv's input x as act(BN(z)), and this dgrad
 * is the last writer of dx = that producer's output gradient.  dx is stored / accumulated as by
 * yms_conv_dgrad; from the FINAL dx values (as stored) each persistent block writes one partial row
 * ws[r][2][cin] = (sum da, sum da * xhat), da = dx * act'(z*scale + shift), xhat = (z - mean)*invstd
 * (z: view of the dx pixels; scale / shift / mean_invstd as yms_bn_act_bwd_reduce), which replaces
 * the yms_bn_act_bwd_reduce pass: yms_bn_act_bwd_finalize(cin, ws, rows = yms_conv_dgrad_bnred_rows(s), ..).
 * Supported where yms_conv_dgrad_bnred_rows(s) > 0 (the direct 3x3 input-gradient kernel's shapes:
 * 16-bit, 3x3, pad 1, stride 1 or 2, 32 / 64 reduction channels, cin <= 32 and a multiple of 8). */
int yms_conv_dgrad_bnred_rows(const yms_conv_shape* s);
yms_status yms_conv_dgrad_bnred(const yms_conv_shape* s, const void* dz, int dz_ld, int dz_off,
                                const void* wpacked_t, void* dx, int dx_ld, int dx_off, int accumulate,
                                const void* z, int z_ld, int z_off, const float* scale, const float* shift,
                                const float* mean_invstd, int act, float* ws, void* stream);
/* dw[cout][cin][k][k] (+)= sum_pixels x (*) dz, fp32; ws = split-K partial slabs. */
size_t yms_conv_wgrad_ws_bytes(const yms_conv_shape* s);
yms_status yms_conv_wgrad(const yms_conv_shape* s, const void* x, int x_ld, int x_off,
                          const void* dz, int dz_ld, int dz_off, float* ws, size_t ws_bytes,
                          float* dw, int accumulate, void* stream);

/* ---- batch norm + activation ---------------------------------------------------------- */
/* Eval: scale = g/sqrt(rv+eps), shift = b - rm*scale (bias-only conv: g=NULL -> scale 1, shift b). */
yms_status yms_bn_fold(int c, const float* gamma, const float* beta, const float* rmean,
                       const float* rvar, float eps, float* scale, float* shift, void* stream);
/* Train: merge the statistics rows of `count` pixels -> mean/invstd, scale/shift, and update the
 * running buffers (unbiased var, momentum) exactly like nn.BatchNorm2d.  mean_invstd: [2][c].
 * Row r = (sum z, sum (z - mean_r)^2) over n_r pixels, n_r = ((float*)stats)[rows*2*stats_ld + r]
 * (the producers' count table; empty rows allowed); rows are merged with Chan's update in fp64.
 * The stats table is consumed: long tables are pre-reduced in place. */
yms_status yms_bn_finalize(int c, float* stats, int rows, int stats_ld, long count,
                           const float* gamma, const float* beta, float* rmean, float* rvar,
                           float momentum, float eps, float* mean_invstd, float* scale,
                           float* shift, void* stream);
/* The same with the invstd row of mean_invstd mi_ld floats after the mean row (>= c): the channel
 * slice of a wider [2][mi_ld] table, for sibling convs whose outputs are slots of one buffer and
 * share one BN backward pass over all their channels (yolov8_head.py:84-85, 99-100). */
yms_status yms_bn_finalize_ld(int c, float* stats, int rows, int stats_ld, long count,
                              const float* gamma, const float* beta, float* rmean, float* rvar,
                              float momentum, float eps, float* mean_invstd, int mi_ld, float* scale,
                              float* shift, void* stream);
/* y = act(z*scale + shift) (+ res), over npix pixels x c channels. */
yms_status yms_affine_act(int dtype, long npix, int c, const void* z, int z_ld, int z_off,
                          const float* scale, const float* shift, int act,
                          const void* res, int res_ld, int res_off,
                          void* y, int y_ld, int y_off, void* stream);
/* Backward of y = silu(bn(z)) (+res):
 *   reduce: partial sums of da and da*xhat (da = gy * silu'(a), a = z*scale+shift) -> ws
 *   finalize: dgamma, dbeta (+=) and the two per-channel coefficients
 *   apply: dz = scale*(da - mean(da) - xhat*mean(da*xhat)), written over dz (may alias z);
 *          gres = gy (gres_acc=0) or gres += gy (gres_acc=1) when gres != NULL (residual). */
int yms_bn_bwd_rows(long npix, int c);   /* partial rows = reduce blocks; ws holds rows*2*c floats */
yms_status yms_bn_act_bwd_reduce(int dtype, long npix, int c, const void* z, int z_ld, int z_off,
                                 const void* gy, int gy_ld, int gy_off, const float* scale,
                                 const float* shift, const float* mean_invstd, int act,
                                 float* ws, void* stream);
yms_status yms_bn_act_bwd_finalize(int c, const float* ws, int rows, long count,
                                   float* dgamma, float* dbeta, float* coef, void* stream);
yms_status yms_bn_act_bwd_apply(int dtype, long npix, int c, const void* z, int z_ld, int z_off,
                                const void* gy, int gy_ld, int gy_off, const float* scale,
                                const float* shift, const float* mean_invstd, const float* coef,
                                int act, void* dz, int dz_ld, int dz_off,
                                void* gres, int gres_ld, int gres_off, int gres_acc, void* stream);
/* reduce + finalize in ONE launch: the last reduce block to finish (agent-scope release/acquire
 * ticket on *counter) sums the partial rows.  *counter must be 0 on entry (it is 0 again on exit);
 * dgamma/dbeta/coef as yms_bn_act_bwd_finalize (any may be NULL). */
yms_status yms_bn_act_bwd_reduce_finalize(int dtype, long npix, int c, const void* z, int z_ld, int z_off,
                                          const void* gy, int gy_ld, int gy_off, const float* scale,
                                          const float* shift, const float* mean_invstd, int act, float* ws,
                                          unsigned* counter, float* dgamma, float* dbeta, float* coef,
                                          void* stream);
/* Bias-only backward of the head's 1x1 nn.Conv2d: dbias = sum over pixels of gy (one launch;
 * counter as above). */
yms_status yms_bias_bwd(int dtype, long npix, int c, const void* gy, int gy_ld, int gy_off,
                        float* ws, unsigned* counter, float* dbias, void* stream);

/* ---- SPPF pools / upsample / layout ---------------------------------------------------- */
/* buf holds 4 consecutive channel slots of width c at channel offset off: slot0 = input x,
 * slots 1..3 <- maxpool5 applied 1,2,3 times (= clipped 5x5 / 9x9 / 13x13 window max). */
yms_status yms_sppf_pool_fwd(int dtype, int n, int h, int w, int c, void* buf, int ld, int off,
                             void* stream);
/* gbuf: grads of the 4 slots; accumulates slot3->slot2->slot1->slot0 through the cascaded
 * pools with PyTorch's first-max argmax (slots 1..2 grads are modified in place). */
size_t yms_sppf_ws_bytes(int n, int h, int w, int c);
yms_status yms_sppf_pool_bwd(int dtype, int n, int h, int w, int c, const void* buf, int ld,
                             int off, void* gbuf, int gld, int goff, void* ws, void* stream);
yms_status yms_upsample2x_fwd(int dtype, int n, int h, int w, int c, const void* x, int x_ld,
                              int x_off, void* y, int y_ld, int y_off, void* stream);
yms_status yms_upsample2x_bwd(int dtype, int n, int h, int w, int c, const void* gy, int gy_ld,
                              int gy_off, void* gx, int gx_ld, int gx_off, int accumulate,
                              void* stream);
/* NCHW fp32 images -> NHWC dtype, channels padded with zeros up to ld. */
yms_status yms_pack_input(int dtype, int n, int c, int h, int w, const float* x, void* y, int ld,
                          void* stream);
/* NHWC view (dtype) <-> NCHW contiguous (dtype_nchw: YMS_F32/BF16/F16). */
yms_status yms_nhwc_to_nchw(int dtype, int dtype_nchw, int n, int h, int w, int c, const void* x,
                            int ld, int off, void* y, void* stream);
yms_status yms_nchw_to_nhwc(int dtype_nchw, int dtype, int n, int h, int w, int c, const void* x,
                            void* y, int ld, int off, int accumulate, void* stream);
/* hipMemsetAsync(p, 0, bytes) / device-to-device hipMemcpyAsync on the stream. */
yms_status yms_zero(void* p, size_t bytes, void* stream);
yms_status yms_copy(void* dst, const void* src, size_t bytes, void* stream);
/* y = cast(x) elementwise (fp32 <-> dtype), count elements. */
yms_status yms_cast(int dtype_in, int dtype_out, long count, const void* x, void* y, void* stream);

/* ---- depthwise k x k conv (YOLO-MS MS-Block inverted bottleneck) --------------- */
/* groups = c, stride 1, pad k/2, k in {3,5,7,9}, c % 8 == 0; w: fp32 [c][k][k] (nn.Conv2d(groups=c)
 * weight, used unpacked).  Not in the reference's code (annotations.md:66-133 diagram only). */
typedef struct {
  int n, h, w, c, k, dtype;
} yms_dw_shape;
/* rows of BN partial statistics written by yms_dwconv_fwd(stats != NULL): one per spatial tile */
int yms_dwconv_stats_rows(const yms_dw_shape* s);
/* stats == NULL: y = act(conv*scale + shift) (scale/shift NULL = identity); else y = conv (pre-BN
 * z) and per-tile (sum z, sum (z - tile mean)^2) rows [rows][2][stats_ld] followed by [rows] pixel
 * counts. */
yms_status yms_dwconv_fwd(const yms_dw_shape* s, const void* x, int x_ld, int x_off, const float* w, void* y,
                          int y_ld, int y_off, const float* scale, const float* shift, int act, float* stats,
                          int stats_ld, void* stream);
/* dx (+)= depthwise conv of dz with the 180-degree rotated kernel */
yms_status yms_dwconv_dgrad(const yms_dw_shape* s, const void* dz, int dz_ld, int dz_off, const float* w, void* dx,
                            int dx_ld, int dx_off, int accumulate, void* stream);
/* dw[c][t] (+)= sum_pixels x(p + d_t) dz(p), fp32, via per-block partials in ws (deterministic) */
size_t yms_dwconv_wgrad_ws_bytes(const yms_dw_shape* s);
yms_status yms_dwconv_wgrad(const yms_dw_shape* s, const void* x, int x_ld, int x_off, const void* dz, int dz_ld,
                            int dz_off, float* ws, size_t ws_bytes, float* dw, int accumulate, void* stream);
/* y (+)= a + b over npix x c channels (b may be NULL); c % 8 == 0 */
yms_status yms_add_views(int dtype, long npix, int c, const void* a, int a_ld, int a_off, const void* b, int b_ld,
                         int b_off, void* y, int y_ld, int y_off, int accumulate, void* stream);
/* Backward of y = a + b in one pass: ga (+)= g, gb (+)= g (acc1 / acc2: accumulate). */
yms_status yms_add_grad2(int dtype, long npix, int c, const void* g, int g_ld, int g_off, void* ga, int ga_ld,
                         int ga_off, int acc1, void* gb, int gb_ld, int gb_off, int acc2, void* stream);

/* ---- mAP@0.5 evaluation (validate_epoch's torchmetrics call, train.py:41-47,146,152-153) ---- */
/* GPU: per image (det_off / gt_off prefix offsets, n_images + 1 entries), rank every detection in
 * its class (stable, score descending), keep the first 100, and greedily match them to the
 * image's ground truths at IoU >= 0.5 (COCOeval semantics) -> tp[d], kept[d] flags.
 * rank_ws: n_det ints of scratch.  max_gt_per_image <= 2048. */
yms_status yms_map_match(int n_images, const float* det_boxes, const float* det_scores, const int* det_labels,
                         const int* det_off, const float* gt_boxes, const int* gt_labels, const int* gt_off,
                         uint8_t* tp, uint8_t* kept, int* rank_ws, int max_gt_per_image, void* stream);
/* HOST (not stream-ordered; host arrays): COCOeval.accumulate at one IoU threshold -> per-class
 * AP (-1 for classes without ground truth) and their mean. */
yms_status yms_map_accumulate(int n_det, const float* scores, const int* labels, const int* image,
                              const uint8_t* tp, const uint8_t* kept, int n_classes, const int* n_gt,
                              double* ap, double* map);

/* ---- input pipeline ------------------------------------------------------ */
/* dataset.py:132-134 per-sample A.Resize(INTER_LINEAR) + A.Normalize(mean, std) + ToTensorV2 and
 * collate_fn's torch.stack (:260), batched: images = device array of n
 * { const uint8_t* src; int h, w, pitch, flags; } (HWC RGB uint8 rows of `pitch` bytes; flags bit 0
 * horizontal flip, bit 1 vertical flip, applied before the resize); out = [n][3][out_h][out_w] of
 * dtype (YMS_F32 / YMS_BF16 / YMS_F16), (v / 255 - mean[c]) / std[c] (mean, std: host float[3]).
 * cv2 half-pixel bilinear coordinates with edge clamping; fp32 weights (cv2's 8-bit fixed-point
 * rounding is not reproduced). */
yms_status yms_resize_normalize(int dtype, int n, const void* images, int out_h, int out_w, const float* mean,
                                const float* std, void* out, void* stream);
/* The training transform (dataset.py:84-131: HueSaturationValue, Rotate, ShiftScaleRotate, RandomScale,
 * Affine shear, Perspective, flips, then Resize + Normalize + ToTensorV2 + stack), batched: images =
 * device array of n AugImage records (yms_augment_image_bytes() bytes each; layout in
 * csrc/preprocess.hip / yms.data.AugImage): the decoded HWC uint8 source, an optional HSV shift
 * (cv2 8-bit HSV, albumentations LUT semantics) and up to 8 geometric stages, each a 3x3 matrix
 * from its output pixel-index coordinates to its input frame plus that frame's size and border rule
 * (reflect-101 / clamp / constant 0).  The per-image parameters are sampled on the host
 * (yms.data.sample_augmentation); one bilinear sample of the source per output pixel. */
size_t yms_augment_image_bytes(void);
yms_status yms_augment_normalize(int dtype, int n, const void* images, int out_h, int out_w, const float* mean,
                                 const float* std, void* out, void* stream);

/* ---- detection loss ------------------------------------------------------- */
/* The reference's ComputeLoss (yolov8/tools/loss.py:94-677; python binding
 * yolov8.tools.loss.ComputeLoss mirrors its constructor and call) on the raw training head maps:
 * maps[l] / grads[l] are NHWC [batch, hs[l], ws_[l], ld] (64 DFL logits, then nc class logits;
 * grads NULL = value only, grads[l] written in full for channels < 64 + nc).  targets: device fp32
 * [n_targets][6] = (image, class, cx, cy, w, h) normalised; boxes scale by (img_w, img_h).
 * iou_type 0 iou, 1 giou, 2 diou, 3 ciou.  pos_weight: NULL or device fp32 [nc].  lambdas (host):
 * box, cls, dfl gains (7.5, 0.5, 1.5 in the reference).  out (device fp32 [4]) = total, box, cls,
 * dfl; grads = d(total)/d(maps).  ws: yms_det_loss_ws_bytes() bytes of device scratch. */
size_t yms_det_loss_ws_bytes(int batch, int anchors, int nc, int n_targets);
yms_status yms_det_loss(int dtype, int batch, int nc, int nlevels, const void* const* maps, void* const* grads,
                        const int* hs, const int* ws_, const float* strides, int ld, const float* targets,
                        int n_targets, float img_w, float img_h, int iou_type, const float* pos_weight,
                        const float* lambdas, void* ws, size_t ws_bytes, float* out, void* stream);
/* bufs[i] (device, dtype, counts[i] elements; 1 <= nbuf <= 4) *= g (device fp32 scalar), in place:
 * the loss's map gradients times the incoming d(out)/d(total) at backward time (replaces
 * `grad * g.to(grad.dtype)` in yolov8/tools/loss.py's autograd backward; a no-op when g == 1). */
yms_status yms_scale_by_device_scalar(int dtype, int nbuf, void* const* bufs, const long* counts, const float* g,
                                      void* stream);

/* ---- head decode + NMS ------------------------------------------------------------------- */
/* Raw head maps lvl[i]: NHWC [n, h_i, w_i, no_ld] with channels (64 DFL box logits, nc cls
 * logits).  out: [n, A, 4+nc] fp32 = (cx, cy, w, h)*stride_i, sigmoid(cls).  When nms_score
 * is not NULL the NMS prep is fused: boxes_xyxy [n,A,4], score [n,A], label [n,A] (-1 when
 * score <= conf). */
yms_status yms_head_decode(int dtype, int n, int nc, int nlev, const void* const* lvl,
                           const int* hs, const int* ws, int no_ld, const float* strides,
                           float* out, float conf, float* boxes_xyxy, float* nms_score,
                           int* label, void* stream);
/* Standalone DFL integral: x [n][4*ch][A] (dtype) -> out [n][4][A] = sum_j j*softmax_j. */
yms_status yms_dfl(int dtype, int n, int A, int ch, const void* x, void* out, void* stream);
/* Same prep from an already-decoded [n, A, 4+nc] fp32 tensor. */
yms_status yms_nms_prep(int n, int A, int nc, const float* pred, float conf, float* boxes_xyxy,
                        float* score, int* label, void* stream);
/* Class-wise NMS over the prep output.  keep_idx[n][A] (anchor ids), keep_lbl[n][A],
 * counts[n]; per image the kept rows are ordered by class ascending, then by descending
 * score (ties by anchor id), exactly like the reference's per-class torchvision loop.
 * ws: at least yms_nms_ws_bytes_min() bytes; with yms_nms_ws_bytes() bytes (+ ~530 B per anchor
 * of suppressee lists) big sparse-overlap segments may also take the graph kernels.  Every routing
 * gives the same keep lists. */
size_t yms_nms_ws_bytes(int n, int A, int nc);
size_t yms_nms_ws_bytes_min(int n, int A, int nc);
yms_status yms_nms_classwise(int n, int A, int nc, const float* boxes_xyxy, const float* score,
                             const int* label, double iou, int64_t* keep_idx, int* keep_lbl,
                             int* counts, void* ws, size_t ws_bytes, void* stream);
/* Plain torchvision.ops.nms(boxes[m,4], scores[m], iou) on one set -> keep[m], *count. */
yms_status yms_nms_single(int m, const float* boxes, const float* scores, double iou,
                          int64_t* keep, int* count, void* ws, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* YMS_H */
