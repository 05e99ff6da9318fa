/*
 * tpgan.h — C-ABI of libtpgan_hip.so, the MI355X (gfx950) kernels of the TP-GAN
 * generator/discriminator hot path.
 *
 * The reference (PandaKenWei/TP-GAN) has no FFI: its hot path is torch.nn layers called
 * from Python.  Each entry point below replaces one aten call the
 * reference's layer factories make; the Python host side (tp-gan_amd/tpgan_lib.py) binds
 * them with ctypes and keeps the reference's module/class/state_dict API on top.
 *
 *   tpg_conv2d_fwd          nn.Conv2d / nn.ConvTranspose2d forward + bias + activation
 *                           (+ residual add) — ModificationLayer.py:54-123 conv(),
 *                           :158-202 deconv(), :298-302 ResidualBlock.forward,
 *                           and the ReflectionPad2d of :83-96 (pad_mode = reflect);
 *                           also Linear (fc1, D_and_G_model.py:212) as a full-kernel conv.
 *   tpg_conv2d_bwd_data     the input gradient of the same op (aten convolution_backward)
 *   tpg_conv2d_bwd_filter   the weight gradient (accumulated into fp32)
 *   tpg_act_bwd             activation' mask (LeakyReLU 0.01 / ReLU, from the saved output)
 *                           + bias gradient
 *   tpg_fold_taps           im2col-lite for the 3-channel convs (taps folded into channels)
 *   tpg_copy4d              dtype/layout conversion and torch.cat into a channel slice
 *                           (D_and_G_model.py:100,102,104,293,298,307,311,312,317,318,323,324)
 *   tpg_local_fuse_fwd/bwd  LocalFuser (D_and_G_model.py:132-159): zero-pad + max over 4 parts
 *   tpg_maxout2_fwd/bwd     fc2 maxout, MaxPool1d(2,2) (D_and_G_model.py:214,290)
 *   tpg_adam                the optimizer update (UtilityMethods.py:14-41 getOptimizer 'Adam')
 *   tpg_dwconv2d_*          depthwise 3x3 conv of MobileNetV2's inverted residuals (MobileNetV2.py:105)
 *   tpg_maxpool2d_*         ResNet stem MaxPool2d(3, 2, 1) (ResNet.py:33)
 *   tpg_avgpool_*           AdaptiveAvgPool2d(1) (MobileNetV2.py:173, ResNet.py:45)
 *   tpg_bn_fold             eval-mode BatchNorm2d folded into conv weights (MobileNetV2.py:100-112)
 *   tpg_bn_train_fwd/bwd    training-mode BatchNorm2d (+ fused activation) with running statistics
 *   tpg_landmark_boxes      get_5_landmarks_pixal_position (UtilityMethods.py:148-164) + the crop
 *                           boxes of DataAndDataset.process (DataAndDataset.py:42-54)
 *   tpg_crop_normalize      PIL crop + ToTensor + x*2-1 (DataAndDataset.py:51-54,216-220,252-255)
 *
 * Conventions
 *   - Every tensor is described by tpg_tensor: a device pointer, a dtype and the element
 *     strides of its LOGICAL NCHW view (n, c, h, w).  Kernels are fastest on
 *     channels-last (NHWC) tensors whose pixel stride is a multiple of 8 elements, which
 *     is what the host side allocates; any other strides are accepted on slower paths.
 *   - Weights are the fp32 master parameters, logical [a][b][kh][kw]
 *     (Conv2d: a = out, b = in; ConvTranspose2d: a = in, b = out), any strides.
 *   - Ownership: every pointer is caller-owned device memory; the library never
 *     allocates or frees and keeps no state besides a thread-local error string.
 *   - Work space: query tpg_conv2d_workspace(); pass at least that many bytes.
 *   - Streams: every call enqueues on the given stream only, never synchronises, and is
 *     therefore legal inside hipStreamBeginCapture (hipGraph) regions.
 *   - Errors: 0 on success, negative for a bad descriptor / unsupported shape, positive
 *     hipError_t for a launch failure; tpg_last_error() returns the message.
 */
#ifndef TPGAN_H
#define TPGAN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* tpg_stream_t; /* hipStream_t */

enum { TPG_F32 = 0, TPG_BF16 = 1, TPG_F16 = 2 };
enum { TPG_ACT_NONE = 0, TPG_ACT_RELU = 1, TPG_ACT_LEAKY = 2, TPG_ACT_RELU6 = 3 };
enum { TPG_PAD_ZERO = 0, TPG_PAD_REFLECT = 1 };
enum { TPG_OP_FWD = 0, TPG_OP_BWD_DATA = 1, TPG_OP_BWD_FILTER = 2 };

typedef struct tpg_tensor {
  void* data;
  int32_t dtype;      /* TPG_F32 / TPG_BF16 / TPG_F16 */
  int32_t reserved;
  int64_t stride[4];  /* element strides of the logical (n, c, h, w) view */
} tpg_tensor;

typedef struct tpg_conv_desc {
  int32_t n;                      /* batch */
  int32_t in_c, in_h, in_w;       /* input  (logical NCHW) */
  int32_t out_c, out_h, out_w;    /* output (logical NCHW) */
  int32_t kh, kw;                 /* kernel */
  int32_t stride_h, stride_w;
  int32_t pad_t, pad_b, pad_l, pad_r;
  int32_t pad_mode;               /* TPG_PAD_*; reflect only for transposed == 0 */
  int32_t transposed;             /* 0: Conv2d, 1: ConvTranspose2d (output_padding = out - natural) */
  int32_t dtype;                  /* activation / arithmetic dtype: TPG_F32 (exact fp32 MFMA), TPG_BF16 or
                                     TPG_F16 (16-bit MFMA operands, fp32 accumulate) */
  int32_t act;                    /* TPG_ACT_* applied after bias (+ residual) */
  float slope;                    /* LeakyReLU negative slope */
  float res_scale;                /* ResidualBlock scaling_factor (ModificationLayer.py:300) */
  int32_t ksplit;                 /* 0 = automatic; >= 1 forces the K split (bwd_filter: pixel splits) */
  int32_t algo;                   /* 0 = automatic; bwd_filter: 1..5 = tile 256x128, 128x128, 128x64,
                                     64x128, 64x64 (used with ksplit >= 1; autotuners set both);
                                     6..9 = kernel-row halo kernel, tile 128x64, 128x32, 64x64,
                                     64x32 (stride-1 bf16 Conv2d, 3/5/7-wide kernels, output
                                     width a multiple of 64); 10, 11 = image-halo kernel, tile
                                     128x32, 64x32 (2x2 / 3x3 kernels, output width 8/16/32/64·m,
                                     64 / width dividing the height); 12 = kernel-row halo kernel,
                                     tile 256x32 (one a-tile up to 256 output channels: dY read
                                     once per b-tile); -30 when not covered */
  int32_t flags;                  /* TPG_FLAG_*: WPACKED = w.data is the image tpg_conv2d_pack_jobs /
                                     tpg_pack_run produced for this descriptor and op */
  int32_t data_ksplit;            /* 0 = automatic; >= 1 forces the k-step split of the forward and
                                     input-gradient launches (1: no split, so no split-K finish
                                     launch); set by autotuners; ignored in deterministic mode */
  int32_t data_algo;              /* forward / input-gradient kernel of small-map convs with several
                                     taps: 0 = planner's rule, 1 = the halo-tiled kernel, 2 = the
                                     tap-DMA pointwise kernel where eligible (16-bit, channels a
                                     multiple of 32); set by autotuners */
  int32_t in_act;                 /* tpg_conv2d_bwd only: TPG_ACT_* of the layer that PRODUCED x (x = that
                                     layer's activated output, saved by this op's forward): the input
                                     gradient leaves the launch as dx * in_act'(x) -- the producer's
                                     activation backward, applied in this launch's epilogue (after a
                                     DX_ACCUM add), so the producer's own backward takes it as its
                                     already-masked g.  0 (TPG_ACT_NONE) everywhere else */
  float in_slope;                 /* LeakyReLU negative slope of in_act */
} tpg_conv_desc;

enum { TPG_FLAG_WPACKED = 1, TPG_FLAG_CONCURRENT = 2, TPG_FLAG_DX_ACCUM = 4 };
/* CONCURRENT: the op runs beside other streams' work (plan grids for a quarter of the chip:
   fewer splits).  DX_ACCUM (tpg_conv2d_bwd_data / tpg_conv2d_bwd): dx holds another gradient
   contribution of the same input on entry and the input-gradient launch adds it in its
   epilogue (dx = dgrad + dx; e.g. a residual block's shortcut gradient), instead of a
   separate add; zero-padded, non-GEMM-form geometries only (-32 otherwise). */

/* Workspace bytes needed by op (TPG_OP_*) for this descriptor. */
size_t tpg_conv2d_workspace(const tpg_conv_desc* d, int32_t op);

/* Pre-packed weights (fwd and bwd_data convert the fp32 master weight into the kernels'
 * tile order on every call unless desc.flags has TPG_FLAG_WPACKED):
 *   tpg_conv2d_packed_bytes  bytes of the packed image of (d, op), op = FWD or BWD_DATA
 *   tpg_conv2d_pack_jobs     describe packing w into wp as <= max_jobs opaque jobs of
 *                            tpg_pack_job_bytes() each, written to host memory `jobs`;
 *                            returns the job count (negative on error)
 *   tpg_pack_prepare         lay a host job array out for one launch; returns its block count
 *   tpg_pack_run             run n prepared jobs (copied to device memory) in ONE launch
 * The image assumes 16-byte aligned channels-last activations (and dense NHWC for the
 * full-kernel GEMM forms); a call whose tensors need another plan returns -21. */
size_t tpg_conv2d_packed_bytes(const tpg_conv_desc* d, int32_t op);
size_t tpg_pack_job_bytes(void);
int32_t tpg_conv2d_pack_jobs(const tpg_conv_desc* d, int32_t op, tpg_tensor w, void* wp, void* jobs,
                             int32_t max_jobs);
int64_t tpg_pack_prepare(void* jobs, int32_t n);
int32_t tpg_pack_run(const void* jobs_dev, int32_t n, int64_t nblocks, tpg_stream_t stream);

/* y = act(conv(x, w) + bias [+ res_scale * residual]).  residual.data may be NULL; bias may be NULL. */
int32_t tpg_conv2d_fwd(const tpg_conv_desc* d, tpg_tensor x, tpg_tensor w, const float* bias,
                       tpg_tensor residual, tpg_tensor y, void* ws, size_t ws_bytes, tpg_stream_t stream);

/* dx = dconv/dx applied to g (g is the already-masked output gradient, see tpg_act_bwd). */
int32_t tpg_conv2d_bwd_data(const tpg_conv_desc* d, tpg_tensor g, tpg_tensor w, tpg_tensor dx,
                            void* ws, size_t ws_bytes, tpg_stream_t stream);

/* dw += dconv/dw (fp32, dw strides given by the tensor; dw.dtype must be TPG_F32). */
int32_t tpg_conv2d_bwd_filter(const tpg_conv_desc* d, tpg_tensor x, tpg_tensor g, tpg_tensor dw,
                              void* ws, size_t ws_bytes, tpg_stream_t stream);

/* Fused per-layer backward of tpg_conv2d_fwd's op (replaces aten convolution_backward of the
 * nn.Conv2d / nn.ConvTranspose2d built at ModificationLayer.py:101 / :186, plus the activation
 * backward of the layer's LeakyReLU / ReLU):
 *   g  = gy * act'(y)          (y = the forward's saved output; written to g — with
 *                               TPG_ACT_NONE g is gy itself and g may be empty)
 *   dx = input gradient of g   (dx.data NULL: skipped)
 *   dw += weight gradient      (dw.data NULL: skipped; desc.algo / ksplit as tpg_conv2d_bwd_filter)
 *   dbias += sum of g          (NULL: skipped)
 * For a stride-1 "same" zero-padded Conv2d the activation' is applied while the input
 * gradient's halo is staged (the input-gradient launch writes g as it goes) and the bias sum
 * rides on the weight-gradient launch (one MFMA against ones per fragment); other layers run
 * tpg_act_bwd first.  w may be a pre-packed image (desc.flags WPACKED, bwd_data layout).
 * g must have y's strides for the fused form.  desc.in_act != NONE: dx = (input gradient
 * [+ dx's DX_ACCUM entry values]) * in_act'(x), fused into the input-gradient epilogue where x
 * has dx's strides (an in-place pass over dx otherwise); needs x and dx. */
int32_t tpg_conv2d_bwd(const tpg_conv_desc* d, tpg_tensor x, tpg_tensor w, tpg_tensor y, tpg_tensor gy,
                       tpg_tensor g, tpg_tensor dx, tpg_tensor dw, float* dbias, void* ws, size_t ws_bytes,
                       tpg_stream_t stream);

/* Launch groups (the four LocalPathways of D_and_G_model.py:18-110 run layer by layer in
 * lockstep, replacing four per-patch launches per op with one).  Between begin and end, the
 * calling thread's conv / activation-backward calls record their kernels instead of launching
 * them; tpg_group_member() opens the next member (one independent problem, e.g. one patch's
 * tpg_conv2d_fwd or tpg_conv2d_bwd).  tpg_group_end() launches the record: where every member
 * issued the same kernel sequence, one grid per position covers all members, otherwise the
 * launches run one by one in call order.  A call that needs another kernel flushes the record
 * first, so the semantics are always those of the calls run in order.  Tensors and workspaces
 * of the recorded calls must stay allocated until tpg_group_end returns. */
void tpg_group_begin(void);
void tpg_group_member(void);
int32_t tpg_group_end(void);

/* g = gy * act'(y) over logical [n, c, h, w]; dbias[c] += sum g (dbias may be NULL). */
int32_t tpg_act_bwd(int32_t n, int32_t c, int32_t h, int32_t w, int32_t act, float slope,
                    tpg_tensor gy, tpg_tensor y, tpg_tensor g, float* dbias, tpg_stream_t stream);

/* out = in over logical [n, c, h, w] with dtype conversion; in and out may have any strides
 * (an out view offset into a wider channels-last buffer implements torch.cat). */
int32_t tpg_copy4d(int32_t n, int32_t c, int32_t h, int32_t w, tpg_tensor in, tpg_tensor out,
                   tpg_stream_t stream);

/* Tap folding for thin-input convs (3-channel images): y[n][(fy*fw + fx)*c + ci][y'][x'] =
 * x[n][ci][y'*sh + fy - pt][x'*sw + fx - pl] (zero outside), y logical [n, fh*fw*c, oh, ow];
 * the conv on y with the weight viewed as [out][fh*fw*c][kh/fh][kw/fw] equals the original
 * (ModificationLayer.py:54-123 conv() on the RGB inputs of D_and_G_model.py:33,193,415).
 * backward != 0: x (as dx) = the sum over every folded copy of y (as the incoming gradient). */
int32_t tpg_fold_taps(int32_t n, int32_t c, int32_t h, int32_t w, int32_t fh, int32_t fw, int32_t sh, int32_t sw,
                      int32_t pt, int32_t pl, int32_t oh, int32_t ow, tpg_tensor x, tpg_tensor y, int32_t backward,
                      tpg_stream_t stream);

/* LocalFuser: part k (logical [n, c, ph[k], pw[k]]) is placed at (top[k], left[k]) of an
 * out_h x out_w zero canvas; y = max over k, argmax = first k attaining it (uint8, NHWC order). */
int32_t tpg_local_fuse_fwd(int32_t n, int32_t c, int32_t out_h, int32_t out_w, const tpg_tensor* parts,
                           const int32_t* ph, const int32_t* pw, const int32_t* top, const int32_t* left,
                           tpg_tensor y, uint8_t* argmax, tpg_stream_t stream);
int32_t tpg_local_fuse_bwd(int32_t n, int32_t c, int32_t out_h, int32_t out_w, tpg_tensor gy,
                           const uint8_t* argmax, const tpg_tensor* dparts, const int32_t* ph,
                           const int32_t* pw, const int32_t* top, const int32_t* left, tpg_stream_t stream);

/* fc2 maxout: y[b, j] = max(x[b, 2j], x[b, 2j+1]) (first index wins ties), x logical [b, 2m]. */
int32_t tpg_maxout2_fwd(int32_t b, int32_t m, tpg_tensor x, tpg_tensor y, uint8_t* argmax, tpg_stream_t stream);
int32_t tpg_maxout2_bwd(int32_t b, int32_t m, tpg_tensor gy, const uint8_t* argmax, tpg_tensor dx,
                        tpg_stream_t stream);

/* In-place Adam (torch.optim.Adam semantics, L2 weight_decay added to the gradient) on a
 * flat fp32 buffer (the four pointers 4-byte aligned, all at the same offset inside 16 bytes).  state is a caller-owned device
 * float[4] {step, 1 - beta1^step, sqrt(1 - beta2^step), unused}, zero-initialised before the
 * first call: step > 0 sets the step count explicitly, step == 0 advances the device counter
 * by one (what a captured hipGraph replays), step < 0 leaves the counter as it is -- a slice of
 * the buffer updated under the step the last call set (the per-bucket updates of an optimizer
 * overlapped with the backward: one numel = 0, step = 0 call per step, then one step = -1 call
 * per bucket).  grad_scale multiplies the gradient. */
int32_t tpg_adam(int64_t numel, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                 float lr, float beta1, float beta2, float eps, float weight_decay, int32_t step,
                 float grad_scale, float* state, tpg_stream_t stream);

/* Overflow guard of the loss-scaled fp16 step (torch.cuda.amp.GradScaler's skip): state[3] :=
 * 1 if any of grad[0..numel) is inf / NaN, else 0 (device-side, graph-capturable).  A tpg_adam
 * call on the same state then leaves parameters, moments and the step counter untouched. */
int32_t tpg_grad_check(int64_t numel, const float* grad, float* state, tpg_stream_t stream);

/* ---- identity-feature extractors (MobileNetV2.py, ResNet.py, FeatureExtract.py) ---- */

/* G-step image losses (tpgan_train._g_losses, build-defined; weights config.py:59-82) fused
 * into single launches (SURVEY.md §3C loss suite).  x (the fake), r (the target), a_i, b_i:
 * logical (n, c, h, w) views of any strides, TPG_F32 / TPG_BF16 / TPG_F16; gradients are
 * written in the dtype and strides of the given tensor.  The forward writes one fp32 scalar
 * to *out (device), summing fixed per-block partials in a fixed order (deterministic); ws:
 * at least tpg_loss_workspace() bytes of device scratch.  Backward: gout = device pointer to
 * the scalar's gradient.
 *   image:  w_pix * mean|x - r| + w_sym * mean|x - flip_w(x)|
 *           + w_tv * (mean|x[y+1] - x[y]| + mean|x[:, x+1] - x[:, x]|)
 *   L1 set: sum_i weight_i * mean|a_i - b_i|   (da_i may have data NULL: no gradient) */
#define TPG_L1_MAX_SEGS 8
typedef struct tpg_l1_seg {
  int32_t n, c, h, w;
  tpg_tensor a, b, da;
  float weight;
} tpg_l1_seg;
size_t tpg_loss_workspace(void);
int32_t tpg_image_losses_fwd(int32_t n, int32_t c, int32_t h, int32_t w, tpg_tensor x, tpg_tensor r, float w_pix,
                             float w_sym, float w_tv, float* ws, size_t ws_bytes, float* out, tpg_stream_t stream);
int32_t tpg_image_losses_bwd(int32_t n, int32_t c, int32_t h, int32_t w, tpg_tensor x, tpg_tensor r, float w_pix,
                             float w_sym, float w_tv, const float* gout, tpg_tensor dx, tpg_stream_t stream);
int32_t tpg_l1_set_fwd(int32_t nseg, const tpg_l1_seg* segs, float* ws, size_t ws_bytes, float* out,
                       tpg_stream_t stream);
int32_t tpg_l1_set_bwd(int32_t nseg, const tpg_l1_seg* segs, const float* gout, tpg_stream_t stream);

/* SSD landmark head of the MobileNetV2 pretraining (MobileNetV2.py:342-649, batch 1 and per-point
 * .item() loops in the reference; here one block per image).  All pointers are fp32 / int32 / u8
 * device memory, dense:  pred (B, n, 2) pixel locations, cls (B, n, C) logits (C >= 5, class 4
 * = background), truth (B, 8) four landmarks, keys (B, n) uniform [0, 1) draws.
 *   tpg_ssd_loss_fwd  MultiTaskLoss.forward (:445-534): labels (B, n) = the landmark each anchor
 *                     is assigned to (within the k (= int(ratio * n)) nearest of a landmark, the
 *                     nearest such landmark, first on ties) or -1; sel (B, n) = 1 for the
 *                     background anchors in the class loss (all of them, or the ones with the
 *                     int(#positives * ratio_nb) smallest keys when there are more); terms
 *                     (B, TPG_SSD_TERMS): [0] alpha * loc + beta * cls, [1..4] location MSE per
 *                     landmark, [5..8] class CE per landmark, [9] background CE, [10] background
 *                     count, [11..14] positives per landmark.  n <= TPG_SSD_MAXN, 1 <= k <= n.
 *   tpg_ssd_loss_bwd  gradients of mean_b terms[b][0] times *gout (device scalar) w.r.t. pred
 *                     (dloc) and cls (dcls), from the forward's labels / sel / terms.
 *   tpg_ssd_decode    MultiTaskDecoder.forward (:551-597): per image and class, the anchors whose
 *                     softmax confidence exceeds conf, greedy NMS (suppress within nms_thr,
 *                     inclusive), the first top_k kept: keep (B, C, top_k) anchor indices (-1 =
 *                     none), score (B, C, top_k). */
#define TPG_SSD_TERMS 16
#define TPG_SSD_MAXN 4096
int32_t tpg_ssd_loss_fwd(int32_t B, int32_t n, int32_t C, const float* pred, const float* cls, const float* truth,
                         float width, float height, int32_t k, double ratio_nb, float alpha, float beta,
                         const float* keys, int32_t* labels, uint8_t* sel, float* terms, tpg_stream_t stream);
int32_t tpg_ssd_loss_bwd(int32_t B, int32_t n, int32_t C, const float* pred, const float* cls, const float* truth,
                         float width, float height, float alpha, float beta, const int32_t* labels,
                         const uint8_t* sel, const float* terms, const float* gout, float* dloc, float* dcls,
                         tpg_stream_t stream);
int32_t tpg_ssd_decode(int32_t B, int32_t n, int32_t C, const float* loc, const float* cls, float conf, float nms_thr,
                       int32_t top_k, int32_t* keep, float* score, tpg_stream_t stream);

/* Depthwise Conv2d (groups == in_c == out_c, MobileNetV2.py:105), kernels up to 3x3, zero
 * padding: y = act(dwconv(x, w) + bias [+ res_scale * residual]).  w logical [C][1][kh][kw]
 * fp32 (any strides); x / y / residual channels-last, 16-byte aligned rows of desc.dtype. */
int32_t tpg_dwconv2d_fwd(const tpg_conv_desc* d, tpg_tensor x, tpg_tensor w, const float* bias,
                         tpg_tensor residual, tpg_tensor y, tpg_stream_t stream);
/* dx = input gradient of the depthwise conv for the masked output gradient g (overwrites dx). */
int32_t tpg_dwconv2d_bwd_data(const tpg_conv_desc* d, tpg_tensor g, tpg_tensor w, tpg_tensor dx,
                              tpg_stream_t stream);
/* dw += weight gradient (fp32 dw, logical [C][1][kh][kw]). */
int32_t tpg_dwconv2d_bwd_filter(const tpg_conv_desc* d, tpg_tensor x, tpg_tensor g, tpg_tensor dw,
                                tpg_stream_t stream);

/* MaxPool2d(k, s, p) (ResNet.py:33): padding never wins; argmax (uint8, NHWC order of y) is the
 * first window tap r*k+s attaining the maximum.  bwd overwrites dx (gather form, no atomics). */
int32_t tpg_maxpool2d_fwd(int32_t n, int32_t c, int32_t h, int32_t w, int32_t k, int32_t s, int32_t p,
                          int32_t oh, int32_t ow, tpg_tensor x, tpg_tensor y, uint8_t* argmax,
                          tpg_stream_t stream);
int32_t tpg_maxpool2d_bwd(int32_t n, int32_t c, int32_t h, int32_t w, int32_t k, int32_t s, int32_t p,
                          int32_t oh, int32_t ow, tpg_tensor gy, const uint8_t* argmax, tpg_tensor dx,
                          tpg_stream_t stream);

/* AdaptiveAvgPool2d(1) (MobileNetV2.py:173, ResNet.py:45): y[n][c] = mean over h x w
 * (y logical [n][c][1][1]); bwd: dx = gy / (h*w) broadcast (overwrites dx). */
int32_t tpg_avgpool_fwd(int32_t n, int32_t c, int32_t h, int32_t w, tpg_tensor x, tpg_tensor y,
                        tpg_stream_t stream);
int32_t tpg_avgpool_bwd(int32_t n, int32_t c, int32_t h, int32_t w, tpg_tensor gy, tpg_tensor dx,
                        tpg_stream_t stream);

/* Eval-mode BatchNorm2d folded into the preceding conv (MobileNetV2.py:100-112):
 * w_out = w * gamma / sqrt(var + eps) per output channel, b_out = (bias - mean) * that + beta
 * (bias may be NULL).  w / w_out logical [cout][cin][kh][kw] fp32, any strides. */
int32_t tpg_bn_fold(int32_t cout, int32_t cin, int32_t kh, int32_t kw, tpg_tensor w, const float* bias,
                    const float* gamma, const float* beta, const float* mean, const float* var, float eps,
                    tpg_tensor w_out, float* b_out, tpg_stream_t stream);

/* Training-mode BatchNorm2d over N*H*W per channel (+ fused activation), pixel-dense channels-last
 * x / y of one dtype: y = act((x - mean) / sqrt(var + eps) * gamma + beta) with batch mean and
 * biased variance; save_mean / save_invstd (float[c]) are kept for the backward; running stats
 * (may both be NULL) move by momentum using the unbiased variance, as nn.BatchNorm2d.
 * ws: float[2c] scratch. */
int32_t tpg_bn_train_fwd(int32_t n, int32_t c, int32_t h, int32_t w, tpg_tensor x, const float* gamma,
                         const float* beta, float* running_mean, float* running_var, float momentum,
                         float eps, int32_t act, float slope, tpg_tensor y, float* save_mean,
                         float* save_invstd, float* ws, tpg_stream_t stream);
/* Backward of the above from dy (gradient of the activation output) and the saved y, x:
 * dx (may have data NULL) overwritten; dgamma / dbeta (may be NULL) accumulated (+=). */
int32_t tpg_bn_train_bwd(int32_t n, int32_t c, int32_t h, int32_t w, int32_t act, float slope,
                         tpg_tensor dy, tpg_tensor y, tpg_tensor x, const float* gamma,
                         const float* save_mean, const float* save_invstd, tpg_tensor dx, float* dgamma,
                         float* dbeta, float* ws, tpg_stream_t stream);

/* Data path, replaces UtilityMethods.get_5_landmarks_pixal_position
 * (UtilityMethods.py:148-164), TestDataset's landmark rescale (DataAndDataset.py:243-246) and the
 * box arithmetic of process() (DataAndDataset.py:42-54), for n faces at once.
 *   lm       device float[n][npts][2] landmark (x, y)
 *   scale    device float[n][2] (sx, sy) multiplied into the 5 points after the means, or NULL
 *   pts_idx  HOST int32[5][2] inclusive index ranges (five_pts_idx; an empty range gives NaN,
 *            as numpy's mean of an empty slice)
 *   patch_wh HOST int32[4][2] (width, height) of left_eye, right_eye, nose, mouth (40x40, 40x40, 40x32, 48x32)
 *   lm5      device float[n][5][2] the five points (before the mouth midpoint)
 *   boxes    device int32[n][4][4] (left, upper, right, lower) per patch, exactly PIL's crop box
 *   status   device int32[n]: 0, or 1 where a point was NaN/inf (the reference raises ValueError
 *            from math.floor there; the box row is then meaningless) */
int32_t tpg_landmark_boxes(int32_t n, int32_t npts, const float* lm, const float* scale, const int32_t* pts_idx,
                           const int32_t* patch_wh, float* lm5, int32_t* boxes, int32_t* status,
                           tpg_stream_t stream);
/* Crop + normalise u8 images into up to 8 outputs in one launch: out_k[b, c, y, x] =
 * u/255*2-1 with u = img[b, c, upper+y, left+x], or 0 outside the image (PIL crop fill), where
 * (left, upper) = boxes[b*box_stride + 4*slots[k] + {0, 1}], or (0, 0) when slots[k] < 0.
 *   img_stride  HOST int64[4] element strides of the u8 image's logical (n, c, h, w) view (HWC: h*w*c, 1, w*c, c)
 *   outs        HOST tpg_tensor[njobs] (f32 or bf16, logical NCHW), out_hw HOST int32[njobs][2] */
int32_t tpg_crop_normalize(int32_t n, int32_t c, int32_t in_h, int32_t in_w, const uint8_t* img,
                           const int64_t* img_stride, int32_t njobs, const tpg_tensor* outs, const int32_t* out_hw,
                           const int32_t* slots, const int32_t* boxes, int32_t box_stride, tpg_stream_t stream);

/* Deterministic mode (process-wide, off by default; SURVEY.md §5 race detection): every
 * reduction runs in a fixed order — no split-K fp32 atomics in the conv forward / input
 * gradient, weight gradients with one pixel split (each dW element added once), bias
 * gradients summed by one block — so two runs on the same inputs are bit-identical.  Slower;
 * meant for parity and run-to-run tests. */
void tpg_set_deterministic(int32_t on);
int32_t tpg_get_deterministic(void);

/* Library version string and the thread-local message of the last failed call. */
const char* tpg_version(void);
const char* tpg_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* TPGAN_H */
