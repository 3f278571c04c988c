/*
 * rgbd_hip.h — C ABI of librgbd_hip.so, the MI355X (gfx950) kernels of the RGB-D
 * DGGM + E-DSAM hot path (reference: TheoBald200814/RGB-D-Instance-Segmentation,
 * mask2former/utils/custom_model.py v0.4.0 and data_process.py).
 *
 * Conventions (SURVEY.md §8(b) "What the C-ABI replacement must export"):
 *   - every pointer is a DEVICE pointer unless the name ends in _host;
 *   - no entry point allocates: callers pass a workspace sized by the matching
 *     *_workspace_size() query (bytes, 256-aligned internally);
 *   - all work is enqueued on `stream` (a hipStream_t passed as void*), nothing
 *     synchronises, so every entry point is hipGraph-capturable;
 *   - return 0 on success, a positive hipError_t on a launch/runtime error, or a
 *     negative RGBD_E* code on a bad argument (checked on the host before any launch).
 *   - dtype: RGBD_F32 (exact-f32 MFMA, the parity mode) or RGBD_BF16 (bf16 MFMA with
 *     f32 accumulation).  Depth planes, DGGM planes, ratios and every discrete
 *     decision are always float32 (SURVEY §7 hard part (i)).
 * Layouts: NCHW = [B][C][H][W]; NHWC = [B][H][W][C]; both dense.
 */
#ifndef RGBD_HIP_H
#define RGBD_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RGBD_OK 0
#define RGBD_E_ARG (-1)      /* null pointer / non-positive size */
#define RGBD_E_SHAPE (-2)    /* shape combination the kernel does not support */
#define RGBD_E_DTYPE (-3)

#define RGBD_F32 0
#define RGBD_BF16 1

#define RGBD_NBINS 512
#define RGBD_MAX_MODES 3

/* Per-image result of the E-DSAM depth decomposition (device memory, one per image).
 * status: 0 ok; 1 histogram range not finite (all-NaN / inf depth: numpy raises
 * "supplied range ... is not finite"); 2 "Too many bins for data range" (numpy
 * ValueError).  Reference: custom_model.py:701-798. */
typedef struct rgbd_decomp_info {
  int32_t status;
  int32_t n_modes;            /* 0..3 selected depth modes (custom_model.py:720-752)   */
  int32_t n_masks;            /* len(region_masks): n_modes+1, or 4 when no mode      */
  int32_t peak_bin[RGBD_MAX_MODES];
  float first_edge, last_edge;/* histogram range after numpy's +-0.5 expansion        */
  float center[RGBD_MAX_MODES];
  float lo[RGBD_MAX_MODES], hi[RGBD_MAX_MODES];  /* interval windows (:754-772)      */
  int32_t hist[RGBD_NBINS];   /* np.histogram counts (:714-718)                      */
} rgbd_decomp_info;

const char* rgbd_version(void);

/* ---------------------------------------------------------------- K1 DGGM-pre
 * Replaces calculate_gradient_features (data_process.py:1247-1305) as called by
 * map_10channel_case2 (dataloader.py:414-421), fused with the 10-channel assembly:
 *   pv[b,0:3]  = (rgb/255 - mean)/std          (image-processor rescale+normalise)
 *   pv[b,3:6]  = (depth/255 - mean)/std        (depth as RGB, :389-410)
 *   pv[b,6:9]  = normalised Sobel magnitude x3 (:415-417)
 *   pv[b,9]    = valid-gradient mask           (:420)
 * rgb_u8: [B][H][W][3] (may be NULL: channels 0:3 untouched); depth_u8: [B][H][W];
 * pv: float32 [B][10][H][W].  Bit-exact to the oracle (IEEE sqrt/div, no FMA). */
size_t rgbd_assemble_workspace_size(int B);
int rgbd_assemble_pixel_values(const uint8_t* rgb_u8, const uint8_t* depth_u8, int B, int H, int W,
                               float* pv, void* ws, void* stream);

/* ---------------------------------------------------------------- a11 labels
 * Replaces the label half of map_10channel_case2 (dataloader.py:391-423): the processor's
 * convert_segmentation_map_to_binary_masks (transformers image_processing_pil_mask2former.py:81-115)
 * on the annotation's instance channel.
 * rgbd_instance_presence: instance_map uint8 [B][H][W] (16-byte aligned; H*W % 16 == 0 when
 *   B > 1) -> presence uint32 [B][8] (zeroed here), bit id of image b = id occurs in the map.
 * rgbd_instance_masks: for j < n, masks[j] (float32 [H][W], 16-byte aligned, H*W % 16 == 0) =
 *   (instance_map[image_of[j]] == ids[j]) as 1.0 / 0.0; ids / image_of int32 [n] on the device.
 * The host orders ids ascending per image and drops ignore_index, like np.unique. */
int rgbd_instance_presence(const uint8_t* instance_map, int B, int H, int W, uint32_t* presence, void* stream);
int rgbd_instance_masks(const uint8_t* instance_map, int H, int W, const int* ids, const int* image_of, int n,
                        float* masks, void* stream);

/* ---------------------------------------------------------------- a11 resizes
 * For frames not at model resolution, the resizes of map_10channel_case2 (dataloader.py:405-414):
 * rgbd_resize_pil_bilinear: the image processor's PIL.Image.resize(BILINEAR) of uint8 images
 *   src [B][H][W][C] (C = 3: colour / depth-as-RGB, C = 1) -> dst [B][out_h][out_w][C], bit-exact
 *   to Pillow's Resample.c (horizontal pass first, 22-bit fixed-point coefficients);
 * rgbd_resize_pil_nearest: PIL NEAREST (the instance map), any C;
 * rgbd_resize_cv2_linear: cv2.resize(depth, INTER_LINEAR) of the 'L' depth [B][H][W] ->
 *   [B][out_h][out_w] (OpenCV's 11-bit fixed-point linear resize; cv2 is absent here: unpinned).
 * ws: rgbd_resize_workspace_size(B, H, W, C, out_h, out_w) bytes (tables + the horizontal pass). */
size_t rgbd_resize_workspace_size(int B, int H, int W, int C, int out_h, int out_w);
int rgbd_resize_pil_bilinear(const uint8_t* src, int B, int H, int W, int C, int out_h, int out_w, uint8_t* dst,
                             void* ws, void* stream);
int rgbd_resize_pil_nearest(const uint8_t* src, int B, int H, int W, int C, int out_h, int out_w, uint8_t* dst,
                            void* ws, void* stream);
int rgbd_resize_cv2_linear(const uint8_t* src, int B, int H, int W, int out_h, int out_w, uint8_t* dst, void* ws,
                           void* stream);

/* ---------------------------------------------------------------- K3 E-DSAM decomposition
 * Replaces, per image and ONCE for all three DSAMs, DSAModule.forward lines 661-687:
 * to_grayscale (custom_model.py:466-480) -> nanmin/nanmax -> np.histogram(512) ->
 * find_peaks(prominence=0.01*max) -> top-3 modes -> windows(ratio) -> region masks ->
 * adaptive_max_pool2d to each DSAM input resolution.
 * depth3: float32 NCHW planes, image b channel c at depth3 + b*batch_stride + c*H*W;
 * depth_channels 3 = ImageNet-normalised depth-as-RGB (grey computed, the v0.4.0 call
 * site :339-350), 1 = an already-grey map (DSAModule.forward called directly).
 * ratio: float32 [B] (device; the predicted window-size ratio, never synced to host).
 * codes[s]: uint8 [B][out_h[s]][out_w[s]], bit i = pooled region mask i (conv_layers[i]).
 * info: rgbd_decomp_info [B]. */
size_t rgbd_edsam_decompose_workspace_size(int B);
int rgbd_edsam_decompose(const float* depth3, long long batch_stride, int depth_channels, int B, int H, int W,
                         const float* ratio, int n_scales, const int* out_h_host,
                         const int* out_w_host, uint8_t* const* codes_host, rgbd_decomp_info* info,
                         void* ws, void* stream);
/* The same decomposition, also writing code_masks[s] (device uint32 [n_scales], OVERWRITTEN):
 * bit k set when region code k occurs in codes[s] — the codes the bf16 DSAM filters are packed
 * for (rgbd_dsam_pack_weights' code_mask), without a pass of its own over the code planes. */
int rgbd_edsam_decompose_masks(const float* depth3, long long batch_stride, int depth_channels, int B, int H,
                               int W, const float* ratio, int n_scales, const int* out_h_host,
                               const int* out_w_host, uint8_t* const* codes_host, rgbd_decomp_info* info,
                               uint32_t* code_masks, void* ws, void* stream);
/* The same decomposition in two phases, for callers that overlap the ratio-free part with the
 * ratio predictor (the hot path: phase A on a side stream beside K4, phase B after it).
 * Phase A, rgbd_edsam_modes: grey plane (kept in ws, 4 B/px), nanmin/nanmax, histogram, modes
 * and centres into info (status, hist, n_modes, n_masks, peak_bin, center, edges; lo/hi zero);
 * code_masks (may be NULL; device uint32 [n_masks]) is zeroed for phase B.
 * Phase B, rgbd_edsam_codes: the windows at ratio (info lo/hi) and the region codes at each
 * resolution from phase A's grey plane; code_masks as in rgbd_edsam_decompose_masks (may be
 * NULL; when given, the array phase A zeroed, n_masks >= n_scales).  ws: rgbd_edsam_modes_workspace_size(B, H, W) bytes, phase B on the workspace phase A
 * filled, stream-ordered after it.  Results identical to rgbd_edsam_decompose(_masks). */
size_t rgbd_edsam_modes_workspace_size(int B, int H, int W);
int rgbd_edsam_modes(const float* depth3, long long batch_stride, int depth_channels, int B, int H, int W,
                     rgbd_decomp_info* info, uint32_t* code_masks, int n_masks, void* ws, void* stream);
int rgbd_edsam_codes(const void* ws, int B, int H, int W, const float* ratio, int n_scales, const int* out_h_host,
                     const int* out_w_host, uint8_t* const* codes_host, rgbd_decomp_info* info,
                     uint32_t* code_masks, void* stream);

/* ---------------------------------------------------------------- K2 DGGM gated fusion
 * Replaces DepthGradientInjectionResidual.forward (custom_model.py:1204-1269) for one
 * scale, fused with the final sum (custom_model.py:355):
 *   out = cp1 + (color + ReLU(W . (bilinear(grad) * nearest(mask)) + b))
 * cp1/color/out: dtype NCHW [B][C][h][w] (cp1 may equal color; cp1 NULL gives the bare
 * module output color + ReLU(...)); grad: float32 planes
 * (3 channels) and mask (1 channel) at grad/mask + b*pv_batch_stride + c*H*W;
 * weight float32 [C][3]; bias float32 [C]. */
int rgbd_dggm_fuse_fwd(int dtype, const void* cp1, const void* color, const float* grad,
                       const float* mask, long long pv_batch_stride, int B, int H, int W, int C,
                       int h, int w, const float* weight, const float* bias, void* out,
                       void* stream);
/* Backward of the gated branch: dW[C][3] and db[C] (float32, OVERWRITTEN) from the
 * upstream gradient dout (dtype NCHW).  The residual paths are identity. */
size_t rgbd_dggm_fuse_bwd_workspace_size(int B, int C, int h, int w);
int rgbd_dggm_fuse_bwd(int dtype, const void* dout, const float* grad, const float* mask,
                       long long pv_batch_stride, int B, int H, int W, int C, int h, int w,
                       const float* weight, const float* bias, float* dweight, float* dbias,
                       void* ws, void* stream);

/* All backbone scales in one launch (the fused hot path calls these): n <= 4 scales given as
 * host arrays of device pointers and sizes; same arithmetic per element as the single-scale
 * forms (bitwise identical results).  cp1_host may be NULL (no residual); workspace for the
 * backward from rgbd_dggm_fuse_bwd_multi_workspace_size. */
int rgbd_dggm_fuse_fwd_multi(int dtype, int n, const void* const* cp1_host, const void* const* color_host,
                             void* const* out_host, const float* const* weight_host, const float* const* bias_host,
                             const int* C_host, const int* h_host, const int* w_host, const float* grad,
                             const float* mask, long long pv_batch_stride, int B, int H, int W, void* stream);
/* rgbd_dggm_fuse_fwd_multi with per-scale cp1 layout: bit k of cp1_nhwc_mask set = scale k's cp1
 * is NHWC dtype [B][h][w][C] (C % 8 == 0; the DSAM cascade's layout), else NCHW. */
int rgbd_dggm_fuse_fwd_multi_mixed(int dtype, int n, const void* const* cp1_host, int cp1_nhwc_mask,
                                   const void* const* color_host, void* const* out_host,
                                   const float* const* weight_host, const float* const* bias_host, const int* C_host,
                                   const int* h_host, const int* w_host, const float* grad, const float* mask,
                                   long long pv_batch_stride, int B, int H, int W, void* stream);
size_t rgbd_dggm_fuse_bwd_multi_workspace_size(int n, const int* C_host, const int* h_host, const int* w_host,
                                               int B);
int rgbd_dggm_fuse_bwd_multi(int dtype, int n, const void* const* dout_host, const float* const* weight_host,
                             const float* const* bias_host, float* const* dweight_host, float* const* dbias_host,
                             const int* C_host, const int* h_host, const int* w_host, const float* grad,
                             const float* mask, long long pv_batch_stride, int B, int H, int W, void* ws,
                             void* stream);

/* ---------------------------------------------------------------- layout helpers */
int rgbd_nchw_to_nhwc(int dtype, const void* src, void* dst, int B, int C, int H, int W,
                      void* stream);
/* Up to four bf16 conversions as rgbd_nchw_to_nhwc in one launch (the hot path's colour maps in
 * the forward, its upstream gradients G[1..3] in the backward); C % 8 == 0.  Bitwise the
 * per-tensor results. */
typedef struct rgbd_nhwc_job {
  const void* src;  /* [B][C][H][W] bf16 (device) */
  void* dst;        /* [B][H][W][C] bf16 (device) */
  int B, C, H, W;
} rgbd_nhwc_job;
int rgbd_nchw_to_nhwc_multi(int n, const rgbd_nhwc_job* jobs, void* stream);  /* jobs: host array */
/* Packs DSAModule weights (conv_layers[0..3].weight, rgb_projection.weight; float32
 * [4][Cout][Cin][3][3] and [Cout][Cin][3][3]) into the implicit-GEMM B operands.
 * RGBD_F32 (segment form):
 *   wfwd [Cout][5][9][Cin]  (forward: k = (seg, tap, ci))
 *   wbwd [Cin][5][9][Cout]  (dX: k = (seg, tap, co), taps NOT flipped; see csrc)
 * RGBD_BF16 (code-merged form, Cin and Cout multiples of 32): for each 4-bit region code k
 * the merged filter W_k = proj + sum_{i in k} conv_i, as contiguous per-(code, tap, 32-channel
 * chunk) tiles with the 16-byte chunks of each 64-byte row XOR-swizzled by 2*((row >> 3) & 1),
 *   wfwd [16 k][9 tap][Cin/32][Cout][32],  wbwd [16 k][9 tap][Cout/32][Cin][32],
 * each followed by a 192x32-element tail pad;
 * only the codes whose bit is set in *code_mask (a device uint32, e.g. from
 * rgbd_dsam_code_masks; NULL = all 16) are written, and wbwd may be NULL (inference).
 * rgbd_dsam_packed_elems gives the element count of each of wfwd / wbwd. */
long long rgbd_dsam_packed_elems(int dtype, int Cin, int Cout);
int rgbd_dsam_pack_weights(int dtype, const float* conv_w, const float* proj_w, int Cin,
                           int Cout, const uint32_t* code_mask, void* wfwd, void* wbwd, void* stream);
/* masks[i] (device uint32, OVERWRITTEN) = OR over the bytes of code map i of (1 << code):
 * the region codes present at one DSAM input resolution (n <= 8 maps). */
int rgbd_dsam_code_masks(int n, const uint8_t* const* codes_host, const long long* nbytes_host,
                         uint32_t* masks, void* stream);

/* ---------------------------------------------------------------- K5 DSAM masked conv
 * Forward of one DSAModule for the whole batch (replaces the per-sample Python loop of
 * custom_model.py:339-352 and DSAModule.forward :682-699):
 *   out = residual + sum_{i<4} Conv3x3s2_i(x * m_i) + sum_{i<n_masks[b]} b_i + Proj3x3s2(x)
 * x_nhwc: dtype [B][h][w][Cin]; code: uint8 [B][h][w] (pooled region codes at x's
 * resolution); bias float32 [4][Cout]; residual/out_nchw: dtype [B][Cout][ho][wo];
 * out_nhwc (optional, may be NULL): dtype [B][ho][wo][Cout].  ws: workspace of
 * rgbd_dsam_conv_workspace_size bytes (split-K slabs of the bf16 path). */
size_t rgbd_dsam_conv_workspace_size(int dtype, int B, int Cin, int h, int w, int Cout);
int rgbd_dsam_fwd(int dtype, const void* x_nhwc, const uint8_t* code, const rgbd_decomp_info* info,
                  int B, int Cin, int h, int w, int Cout, const void* wfwd, const float* bias,
                  const void* residual, void* out_nchw, void* out_nhwc, void* ws, void* stream);
/* The same forward with everything in NHWC (RGBD_BF16 only; the hot path's cascade): residual_nhwc
 * (may be NULL) and out_nhwc dtype [B][ho][wo][Cout]; no NCHW output.  Same arithmetic and
 * rounding as rgbd_dsam_fwd (res + (acc + bias), one rounding). */
int rgbd_dsam_fwd_nhwc(int dtype, const void* x_nhwc, const uint8_t* code, const rgbd_decomp_info* info,
                       int B, int Cin, int h, int w, int Cout, const void* wfwd, const float* bias,
                       const void* residual_nhwc, void* out_nhwc, void* ws, void* stream);
/* dX of one DSAModule, plus the upstream gradient of its input's other consumer:
 *   dx = gin + sum_i m_i * ConvT_i(gout) + ConvT_proj(gout)
 * gout_nhwc: dtype [B][ho][wo][Cout].  At least one of dx_nchw (dtype [B][Cin][h][w]) and
 * dx_nhwc (dtype [B][h][w][Cin]) is written.  The optional gin comes in the layout of the pass
 * that adds it: gin_nchw (dtype [B][Cin][h][w]) when dx_nchw is written, gin_nhwc (RGBD_BF16
 * only, [B][h][w][Cin]) when only dx_nhwc is (the hot path's cascade: NHWC in, NHWC out). */
int rgbd_dsam_bwd_data(int dtype, const void* gout_nhwc, const uint8_t* code, int B, int Cin, int h,
                       int w, int Cout, const void* wbwd, const void* gin_nchw, const void* gin_nhwc,
                       void* dx_nchw, void* dx_nhwc, void* ws, void* stream);
/* dW / db of one DSAModule: dconv_w float32 [4][Cout][Cin][3][3], dproj_w float32
 * [Cout][Cin][3][3], dbias float32 [4][Cout] (all OVERWRITTEN).  gout_nchw: dtype
 * [B][Cout][ho][wo] (required for RGBD_F32; optional for RGBD_BF16, whose bias sums then read
 * gout_nhwc); gout_nhwc: the same gradient as [B][ho][wo][Cout] (required for RGBD_BF16,
 * ignored for RGBD_F32); x_nhwc as in the forward. */
size_t rgbd_dsam_bwd_weight_workspace_size(int dtype, int B, int Cin, int h, int w, int Cout);
int rgbd_dsam_bwd_weight(int dtype, const void* gout_nchw, const void* gout_nhwc, const void* x_nhwc,
                         const uint8_t* code, const rgbd_decomp_info* info, int B, int Cin, int h,
                         int w, int Cout, float* dconv_w, float* dproj_w, float* dbias, void* ws,
                         void* stream);

/* Planning ahead (RGBD_BF16).  What a bf16 leg sets up before its GEMM (per-tile code sets and
 * the work list of a forward / dX leg; per-code live units, items and tap masks of a dW leg)
 * depends only on the region codes, so a caller may plan every leg of a step at once, right
 * after rgbd_edsam_decompose (two launches for all forward / dX legs), and run the legs later
 * with the _planned entry points: same arguments as the plain ones plus the leg's plan buffer,
 * and ws then needs only rgbd_dsam_run_workspace_size bytes (split-K / dW partials, which legs
 * run one after another on one stream may share).  Results are bitwise those of the plain
 * entry points.  A plan buffer serves one run of one leg (the run uses up its work counters):
 * plan again before running the leg again, and leave the buffer untouched until the leg ran. */
enum { RGBD_LEG_FWD = 0, RGBD_LEG_DX = 1, RGBD_LEG_DW = 2 };
typedef struct rgbd_dsam_leg {
  int kind;                /* RGBD_LEG_* */
  const uint8_t* code;     /* the DSAM's region codes [B][h][w] (device) */
  int B, Cin, h, w, Cout;  /* the DSAModule's shape; h x w = its input resolution */
  void* plan;              /* rgbd_dsam_plan_size bytes (device), OVERWRITTEN */
} rgbd_dsam_leg;
size_t rgbd_dsam_plan_size(int kind, int B, int Cin, int h, int w, int Cout);
size_t rgbd_dsam_run_workspace_size(int kind, int B, int Cin, int h, int w, int Cout);
int rgbd_dsam_plan(int n, const rgbd_dsam_leg* legs, void* stream);  /* legs: host array */
int rgbd_dsam_fwd_nhwc_planned(int dtype, const void* x_nhwc, const uint8_t* code,
                               const rgbd_decomp_info* info, int B, int Cin, int h, int w, int Cout,
                               const void* wfwd, const float* bias, const void* residual_nhwc,
                               void* out_nhwc, const void* plan, void* ws, void* stream);
int rgbd_dsam_bwd_data_planned(int dtype, const void* gout_nhwc, const uint8_t* code, int B, int Cin,
                               int h, int w, int Cout, const void* wbwd, const void* gin_nchw,
                               const void* gin_nhwc, void* dx_nchw, void* dx_nhwc, const void* plan,
                               void* ws, void* stream);
int rgbd_dsam_bwd_weight_planned(int dtype, const void* gout_nchw, const void* gout_nhwc,
                                 const void* x_nhwc, const uint8_t* code, const rgbd_decomp_info* info,
                                 int B, int Cin, int h, int w, int Cout, float* dconv_w, float* dproj_w,
                                 float* dbias, const void* plan, void* ws, void* stream);
/* dW of several bf16 DSAM legs that are ready together (the hot path's dsam1 and dsam0 once the dX
 * cascade has finished; hot_path.py): one persistent GEMM launch over the legs' joint work list —
 * two back-to-back whole-chip launches would each drain on a partly idle chip; its workgroups
 * then drain the legs' bias channel sums — and one launch for both legs' combines.  Per leg the results are bitwise those of rgbd_dsam_bwd_weight_planned
 * with gout_nchw = NULL (the autograd of DSAModule.forward, custom_model.py:682-699).  n: 1 or 2;
 * every run has its own plan and ws (rgbd_dsam_run_workspace_size(RGBD_LEG_DW, ...)).  Legs of
 * different output tile shapes run one launch each. */
typedef struct rgbd_dsam_dw_run {
  const void* gout_nhwc;   /* upstream gradient [B][ho][wo][Cout] bf16 (device) */
  const void* x_nhwc;      /* the DSAM's input [B][h][w][Cin] bf16 (device) */
  const uint8_t* code;     /* region codes [B][h][w] (device) */
  int B, Cin, h, w, Cout;
  float* dconv_w;          /* [4][Cout][Cin][3][3] */
  float* dproj_w;          /* [Cout][Cin][3][3] */
  float* dbias;            /* [4][Cout] */
  const void* plan;        /* this leg's RGBD_LEG_DW plan (rgbd_dsam_plan) */
  void* ws;
} rgbd_dsam_dw_run;
int rgbd_dsam_bwd_weight_planned_multi(int n, const rgbd_dsam_dw_run* runs, const rgbd_decomp_info* info,
                                       void* stream);  /* runs: host array */

/* ---------------------------------------------------------------- optimizer step
 * AdamW (the HF Trainer's optimizer, finetuning.py:98, lr 1e-5 constant per config.json:12-13) over
 * n <= 48 fp32 tensors in one launch, the element update of torch.optim.AdamW (decoupled weight
 * decay, no amsgrad): params, grads, exp_avg, exp_avg_sq, numel are host arrays of device
 * pointers / sizes; step points at the (already incremented) step count on the device. */
int rgbd_adamw_multi(int n, float* const* params, const float* const* grads, float* const* exp_avg,
                     float* const* exp_avg_sq, const long long* numel, const float* step, double lr, double beta1,
                     double beta2, double eps, double weight_decay, void* stream);
/* The same update, also writing each updated parameter's bfloat16 copy (round to nearest even, the
 * bits torch's .to(torch.bfloat16) gives) into shadows[i] (a host array of device pointers; an
 * entry may be NULL): the next forward's bf16 GEMM operands without a cast launch per weight. */
int rgbd_adamw_multi_shadow(int n, float* const* params, const float* const* grads, float* const* exp_avg,
                            float* const* exp_avg_sq, void* const* shadows, const long long* numel,
                            const float* step, double lr, double beta1, double beta2, double eps,
                            double weight_decay, void* stream);

/* ---------------------------------------------------------------- K4 ratio predictor
 * EnhancedDepthImageRatioPredictor.forward (custom_model.py:1444-1487) for the batch:
 * depth3 (float32 planes as for the decomposition) -> ratio float32 [B] in [0.01, 0.5],
 * left on device (the reference's k.item() host sync of :339-351 is gone).
 * Weights (they receive no gradient in v0.4.0, Q2) are packed once:
 *   weights_host: RGBD_RATIO_NW device pointers to the float32 state_dict tensors, order
 *     scale1_conv.0.{weight,bias}, scale2_conv.0.*, scale3_conv.0.*, feature_fusion.0.*,
 *     attention.0.*, attention.2.*, feature_extractor.0.*, feature_extractor.4.*,
 *     fc_layers.0.*, fc_layers.3.*, fc_layers.6.*, fc_layers.8.*
 *   bn_host: RGBD_RATIO_NBN x {weight, bias, running_mean, running_var} device pointers for
 *     scale1_conv.1, scale2_conv.1, scale3_conv.1, feature_fusion.1, feature_extractor.1,
 *     feature_extractor.5.  training=1 uses batch statistics and updates the running stats
 *     in place (torch semantics, `momentum`), and applies dropout with a counter hash of
 *     `seed` + *seed_counter; the forward then increments *seed_counter on the device (a
 *     u64 the caller owns; NULL = `seed` alone), so a captured graph's replays draw fresh
 *     masks.  training=0 uses the running stats.  B <= 32. */
#define RGBD_RATIO_NW 24
#define RGBD_RATIO_NBN 6
size_t rgbd_ratio_packed_size(int dtype);
int rgbd_ratio_pack(int dtype, const float* const* weights_host, void* packed, void* stream);
size_t rgbd_ratio_workspace_size(int dtype, int B, int H, int W);
/* Byte offset in the workspace of the gated attention features x * sigmoid(attention(x))
 * (the input of feature_extractor, custom_model.py:1468-1471) as rgbd_ratio_forward leaves
 * them: float32 NHWC [B][H][W][128]; bf16 channel-quarter-major [B][4][H][W][32] (channel
 * 32q + k at [b][q][y][x][k]); valid until the workspace is reused (diagnostics / tests). */
size_t rgbd_ratio_features_offset(int dtype, int B, int H, int W);
/* Byte offset in the workspace of the AdaptiveAvgPool(4) output of feature_extractor[0:4]
 * (conv5 -> BN -> ReLU -> pool, custom_model.py:1412-1416) as rgbd_ratio_forward leaves it:
 * float32 [B][256][4][4] (diagnostics / tests). */
size_t rgbd_ratio_pooled_offset(int dtype, int B, int H, int W);
int rgbd_ratio_forward(int dtype, int training, float momentum, const float* depth3, long long batch_stride,
                       int B, int H, int W, const void* packed, float* const* bn_host, unsigned long long seed,
                       unsigned long long* seed_counter, float* ratio, void* ws, void* stream);
/* The same with option bits: RGBD_RATIO_F_PHASE2 runs the bf16 train mode's gated features
 * through the phase-2 recompute (stem + fusion) instead of the gate kernel over phase 1's stored
 * fusion output — the same values by another route, for tests that compare the two. */
#define RGBD_RATIO_F_PHASE2 1
int rgbd_ratio_forward_ex(int dtype, int training, float momentum, const float* depth3, long long batch_stride,
                          int B, int H, int W, const void* packed, float* const* bn_host, unsigned long long seed,
                          unsigned long long* seed_counter, float* ratio, void* ws, int flags, void* stream);

/* ---------------------------------------------------------------- f3 point-sampled mask terms
 * The mask terms of the Mask2Former matcher and loss (transformers 5.15 modeling_mask2former.py,
 * the library the reference trains through): sample_point (:245-275), the matcher's pair-wise
 * sigmoid-CE and dice costs (:328-375, :445-470) and loss_masks' sigmoid-CE / dice over the
 * matched pairs (:278-325, :580-630).  All float32.
 * rgbd_point_sample: out[m][p] = grid_sample(maps[m] ([h][w]), 2*coords - 1, bilinear,
 *   align_corners=False, zeros) at coords[m / maps_per_coord][p] = (x, y) in [0, 1]^2 (one point
 *   set per group of maps_per_coord consecutive maps);
 *   rgbd_point_sample_bwd ADDS the transposed scatter of gout into gmaps (f32 atomics).
 * rgbd_match_cost: image b's cost [Q][T_b] at cost + coff[b] = w_mask * CE + w_class *
 *   class_cost + w_dice * DICE over pred [B][Q][P] and the targets' sampled labels at tgt +
 *   toff[b]*P (toff int [B+1], coff int64 [B], device), clamped to +-1e10, NaN -> 0.
 * rgbd_point_losses: per row n of logits / labels [N][P]: ce[n] = mean BCEWithLogits, dice[n] =
 *   1 - (2 sum sig*y + 1) / (sum sig + sum y + 1), sums[n] = (sum sig*y, sum sig, sum y);
 *   rgbd_point_losses_bwd: glogits [N][P] from the per-row upstream gradients g_ce, g_dice [N]. */
int rgbd_point_sample(const float* maps, int nmaps, int h, int w, const float* coords, int maps_per_coord, int P,
                      float* out, void* stream);
/* the same sample from maps of dtype RGBD_F32 or RGBD_BF16 (widened exactly: the bf16 logits
 * the model produces under autocast are sampled without a float32 copy); f32 output */
int rgbd_point_sample_t(int dtype, const void* maps, int nmaps, int h, int w, const float* coords, int maps_per_coord,
                        int P, float* out, void* stream);
/* the same with the point set of map m given per map: coords [S][P][2], set_of_map int [nmaps]
 * (device) — every image's target masks against that image's points in one launch (the matcher
 * draws one point set per image, modeling_mask2former.py:459-463) */
int rgbd_point_sample_sets(int dtype, const void* maps, int nmaps, int h, int w, const float* coords,
                           const int* set_of_map, int P, float* out, void* stream);
int rgbd_point_sample_bwd(const float* gout, int nmaps, int h, int w, const float* coords, int maps_per_coord,
                          int P, float* gmaps, void* stream);
int rgbd_match_cost(const float* pred, int B, int Q, int P, const float* tgt, const int* toff,
                    const float* class_cost, const long long* coff, float w_mask, float w_class, float w_dice,
                    float* cost, void* stream);
/* rgbd_match_cost with the class cost read from the matcher's softmax instead of a gathered
 * table: class_cost[b][q][t] = -probs[b][q][labels[toff[b] + t]], probs float32 [B][Q][C],
 * labels int64 [sum T_b] (every image's class labels, concatenated) (:448-450). */
int rgbd_match_cost_probs(const float* pred, int B, int Q, int P, const float* tgt, const int* toff,
                          const float* probs, int C, const long long* labels, const long long* coff, float w_mask,
                          float w_class, float w_dice, float* cost, void* stream);
/* rgbd_topk_rows: idx [rows][k] int64 = the indices of the k largest of each row of x [rows][n]
 *   float32 — loss_masks' uncertainty selection torch.topk(unc, k, dim=1, sorted=False)
 *   (modeling_mask2former.py:711): every element above the k-th largest, then the lowest-index
 *   elements equal to it; NaN ranks largest (torch's key order).  The set only: indices are
 *   written in increasing order.  n <= rgbd_topk_rows_max_n() (the row is held in LDS). */
size_t rgbd_topk_rows_max_n(void);
int rgbd_topk_rows(const float* x, int rows, int n, int k, long long* idx, void* stream);
int rgbd_point_losses(const float* logits, const float* labels, int N, int P, float* ce, float* dice,
                      float* sums, void* stream);
int rgbd_point_losses_bwd(const float* logits, const float* labels, int N, int P, const float* sums,
                          const float* g_ce, const float* g_dice, float* glogits, void* stream);

/* The decoder memory of one feature level (Mask2FormerTransformerModule.forward :2095-2109):
 *   out[p][b][c] = proj[b][c][p] + embed[c]   (proj dtype [B][C][HW]: the input projection's
 *   output; embed float32 [C]: level_embed.weight[level]; out float32 [HW][B][C]: the permuted
 *   memory, contiguous).  _bwd from g float32 [HW][B][C]: dproj[b][c][p] = g[p][b][c] in proj's
 *   dtype, dembed[c] = sum over pixels and images (fixed order; ws:
 *   rgbd_level_memory_workspace_size bytes). */
size_t rgbd_level_memory_workspace_size(int B, int C, int HW);
int rgbd_level_memory_fwd(int dtype, const void* proj, const float* embed, int B, int C, int HW, float* out,
                          void* stream);
int rgbd_level_memory_bwd(int dtype, const float* g, int B, int C, int HW, void* dproj, float* dembed, void* ws,
                          void* stream);

/* ---------------------------------------------------------------- f2 deformable attention
 * Replaces multi_scale_deformable_attention (transformers 5.15 modeling_mask2former.py:798-837),
 * the core of each pixel-decoder encoder layer (:1011).  value: dtype [B][S][NH][D] with
 * S = sum of the L level sizes; shapes_host: host int [L][2] = (H, W) per level (L <= 4);
 * loc: float32 [B][Q][NH][L][P][2] sampling locations in [0, 1] (x, y); attw: float32
 * [B][Q][NH][L][P] softmaxed weights; out: dtype [B][Q][NH*D].  D in {16, 32, 64}.
 * Bilinear, zero padding, align_corners=False (grid_sample's rule). */
int rgbd_msda_fwd(int dtype, const void* value, int B, int L, const int* shapes_host, int NH, int D, int Q,
                  int P, const float* loc, const float* attw, void* out, void* stream);
/* Backward: gvalue float32 [B][S][NH][D] (zeroed here, then accumulated with atomics), gloc
 * float32 like loc, gattw float32 like attw (both OVERWRITTEN); gout dtype like out. */
int rgbd_msda_bwd(int dtype, const void* value, int B, int L, const int* shapes_host, int NH, int D, int Q,
                  int P, const float* loc, const float* attw, const void* gout, float* gvalue, float* gloc,
                  float* gattw, void* stream);

/* The sampling locations of two-coordinate reference points (:990-994) in one pass:
 *   loc[b][q][h][l][p][c] = ref[b][q][l][c] + off[b][q][h][l][p][c] / norm[l][c]
 * ref float32 [B][Q][L][2]; off dtype [B][Q][NH][L][P][2] (the sampling-offset projection);
 * norm float32 [L][2] = (W_l, H_l); the division in off's dtype (torch's bf16 / int64), the sum
 * in float32.  _bwd: goff = (gloc rounded to off's dtype) / norm, rounded to off's dtype. */
int rgbd_msda_locations(int dtype, const float* ref, const void* off, const float* norm, int B, int Q, int NH,
                        int L, int P, float* loc, void* stream);
int rgbd_msda_locations_bwd(int dtype, const float* gloc, const float* norm, int B, int Q, int NH, int L, int P,
                            void* goff, void* stream);

/* ---------------------------------------------------------------- f3 matcher assignment
 * Replaces scipy.optimize.linear_sum_assignment(cost_matrix.cpu()) in
 * Mask2FormerHungarianMatcher.forward (transformers 5.15 modeling_mask2former.py:474): a batch of
 * n cost matrices (float32, row-major, at cost + meta[4k+0], meta[4k+1] rows x meta[4k+2] cols;
 * meta is a DEVICE int64 [n][4]) solved with scipy 1.15's shortest-augmenting-path algorithm in
 * float64, one wavefront per matrix, same optimum as scipy including ties.  Outputs (int64,
 * min(rows, cols) each, at rows_out / cols_out + meta[4k+3]) are scipy's (row_ind, col_ind);
 * status[k] = 0 ok, 1 infeasible, 2 NaN / -inf entries (scipy's ValueErrors).
 * max(max_rows, max_cols) <= 2048. */
size_t rgbd_lsa_lds_bytes(int max_rows, int max_cols);
int rgbd_lsa_batch(int n, const float* cost, const long long* meta, int max_rows, int max_cols,
                   int64_t* rows_out, int64_t* cols_out, int* status, void* stream);

/* ---------------------------------------------------------------- f1 mask predictor
 * Replaces the dense work of Mask2FormerMaskPredictor.forward (transformers 5.15
 * modeling_mask2former.py:2040-2056; called 10x per forward from :1896 and :1929).
 * rgbd_mask_logits: einsum("bqc,bchw->bqhw") (:2046) as an MFMA GEMM.
 *   emb: dtype [B][Q][C] (the mask embeddings, mask_embedder output), pix: dtype NCHW
 *   [B][C][H][W] (pixel decoder mask features), logits: dtype [B][Q][H][W] (OVERWRITTEN).
 *   C % 32 == 0; emb / pix / logits 16-byte aligned.  f32: exact-f32 MFMA products, f32 sums. */
int rgbd_mask_logits(int dtype, const void* emb, const void* pix, int B, int Q, int C, int H, int W,
                     void* logits, void* stream);
/* rgbd_mask_attention: the attention mask of :2048-2054 from those logits —
 *   bilinear resample to th x tw (align_corners=False, torch's source-index rule), rounded to
 *   dtype, sigmoid rounded to dtype, < 0.5 — written as bytes 0/1 (torch.bool) to
 *   attn [B*heads][Q][th*tw] (head-major repeat, :2052-2053). */
int rgbd_mask_attention(int dtype, const void* logits, int B, int Q, int H, int W, int th, int tw,
                        int heads, uint8_t* attn, void* stream);

/* ---------------------------------------------------------------- f1 masked cross-attention
 * The attention core of nn.MultiheadAttention's math path as the masked-attention decoder layers
 * call it (transformers 5.15 modeling_mask2former.py:1640-1647 with the mask of :2048-2055),
 * float32 arithmetic: per bh (= batch * heads + head), S = (q * scale) k^T, masked entries -inf,
 * P = softmax(S), out = P v.  Sequence-major, as the module's projections lay them out:
 * q [Q][BH][head_dim], k / v [L][BH][head_dim], out [Q][BH][head_dim], lse [Q][BH] (log-sum-exp
 * of the masked scaled scores, saved for the backward); mask bool bytes [BH][Q][L] (1 = not
 * allowed; NULL = no mask: the decoder layers' self-attention, Mask2FormerAttention :1525-1570).
 * head_dim == 32.  A fully masked row gives NaN, as torch's softmax does.
 * ws: rgbd_masked_attn_fwd_workspace_size(BH, Q, L) bytes (per-key-split partials).
 * rgbd_masked_attn_bwd: dq, dk, dv (OVERWRITTEN) from dout; deterministic (no atomics);
 *   ws: rgbd_masked_attn_bwd_workspace_size(BH, Q, L) bytes.
 * q, k, v, out, dout, dk, dv 16-byte aligned;
 * dtype (RGBD_F32 / RGBD_BF16) is the type of q, k, v, out, dout, dq, dk, dv (bf16: the
 * module under torch.autocast, whose projections produce bf16); the arithmetic is float32 on
 * the widened operands either way, lse / delta float32. */
size_t rgbd_masked_attn_fwd_workspace_size(int BH, int Q, int L);
int rgbd_masked_attn_fwd(int dtype, const void* q, const void* k, const void* v, const uint8_t* mask, int BH, int Q,
                         int L, int head_dim, float scale, void* out, float* lse, void* ws, void* stream);
size_t rgbd_masked_attn_bwd_workspace_size(int BH, int Q, int L);
int rgbd_masked_attn_bwd(int dtype, const void* q, const void* k, const void* v, const uint8_t* mask, const void* out,
                         const float* lse, const void* dout, int BH, int Q, int L, int head_dim, float scale,
                         void* dq, void* dk, void* dv, void* ws, void* stream);

/* ---------------------------------------------------------------- f4 instance post-processing
 * Replaces Mask2FormerImageProcessor.post_process_instance_segmentation (transformers 5.15
 * image_processing_mask2former.py:627-744; called by the reference's process_prediction,
 * mask2former/predictor.py:697-700) with return_coco_annotation / return_binary_maps False.
 *   class_logits float32 [B][Q][C1] (C1 = classes + no-object), mask_logits float32 [B][Q][h][w];
 *   target_h_host / target_w_host: per-image output sizes (the reference's target_sizes; pass
 *   384 x 384 for "no resize"); seg_host: B device pointers to float32 [Ht][Wt] maps (written:
 *   segment id per pixel, -1 = none); topk_idx int32 [B][Q]: flat (query * C + class) indices in
 *   the order CPU torch.topk(sorted=False) returns them (libstdc++ nth_element, restated);
 *   pred_scores float32 [B][Q] (class prob x mask score); seg_id int32 [B][Q]: the segment id of
 *   each top-k entry, -1 when dropped (empty mask at the target size or score < threshold).
 *   Q * (C1 - 1) <= 20480 (the selection runs in LDS).  ws: rgbd_pp_instance_workspace_size. */
size_t rgbd_pp_instance_workspace_size(int B, int Q);
int rgbd_pp_instance(const float* class_logits, const float* mask_logits, int B, int Q, int C1, int h, int w,
                     const int* target_h_host, const int* target_w_host, double threshold, float* const* seg_host,
                     int* topk_idx, float* pred_scores, int* seg_id, void* ws, void* stream);
/* return_binary_maps=True of the same call (image_processing_mask2former.py:731-733, used by the
 * reference's Evaluator, model_essential_part.py:87-92): after rgbd_pp_instance on the same ws and
 * stream, writes image b's kept masks at its target size, stacked in segment-id order, as float32
 * 0/1 into out [n_kept][Ht][Wt] (n_kept = the number of seg_id[b][:] >= 0). */
int rgbd_pp_binary_maps(const void* ws, int B, int Q, int b, int Ht, int Wt, const int* seg_id, float* out,
                        void* stream);

/* ---------------------------------------------------------------- f4 segm mAP: mask IoU
 * The mask IoU of torchmetrics MeanAveragePrecision(iou_type="segm") as the reference's
 * Evaluator uses it (model_essential_part.py:56-157; pycocotools maskApi rleIou underneath).
 * rgbd_pack_mask_bits: masks uint8 [n][npx] ({0, nonzero}) -> bits u64 [n][ceil(npx / 64)]
 *   (bit j of word w = pixel 64 w + j) and area int32 [n] (OVERWRITTEN).
 * rgbd_mask_intersections: inter int32 [na][nb] = popcount(a_i AND b_j) over packed masks of the
 *   same npx.  IoU = inter / (area_a + area_b - inter), 0 when inter == 0 (rleIou). */
int rgbd_pack_mask_bits(const uint8_t* masks, int n, long long npx, unsigned long long* bits, int* area,
                        void* stream);
int rgbd_mask_intersections(const unsigned long long* a, int na, const unsigned long long* b, int nb, long long npx,
                            int* inter, void* stream);

/* ---------------------------------------------------------------- f1 / f2 dense layers
 * The nn.Linear layers of the Mask2Former decoder (transformers 5.15 modeling_mask2former.py:
 * self_attn q/k/v/out_proj :1480-1483, fc1/fc2 :1711-1714), of the pixel decoder's encoder
 * layers (value_proj / sampling_offsets / attention_weights / output_proj :862-868, fc1/fc2
 * :1030-1036) and of Swin-T (modeling_swin.py qkv :420-424, output :540, MLP :560/574, patch
 * merging :344), forward and backward, as one MFMA GEMM family (csrc/gemm.hip):
 *   C[b][m][n] = act(sum_k op(A)[m][k] op(B)[k][n] + bias[n]) (+ R[b][m][n])
 *   a_t = 0: A stored [M][lda] (K contiguous); a_t = 1: A stored [K][lda] (M contiguous)
 *   b_t = 0: B stored [N][ldb] (K contiguous, an nn.Linear weight); b_t = 1: [K][ldb]
 *   forward Y = X W^T + b: (0, 0); dX = dY W: (0, 1); dW = dY^T X: (1, 1)
 *   act RGBD_ACT_RELU_GRAD: C = acc where R > 0 else 0 (ReLU backward; bias must be NULL).
 *   A and B share dtype (RGBD_F32 / RGBD_BF16); C is that dtype, or float32 with c_f32 = 1
 *   (weight gradients of bf16 GEMMs, autocast's float32 residual streams); R has C's dtype.
 *   c_f32 = 2 (bf16): C float32 holding the bf16-rounded results, R in bf16 — a bf16 GEMM's
 *   output widened for a float32 consumer (autocast's dX of a float32 input) in the store.  bias: float32 [N] or NULL.  batch strides sa / sb / sr / sc
 *   in elements.  splits > 1: split-K with float32 partials in ws (rgbd_gemm_workspace_size),
 *   summed in split order (deterministic).  bf16: float32 accumulation; f32: exact f32 MFMA. */
#define RGBD_ACT_NONE 0
#define RGBD_ACT_RELU 1
#define RGBD_ACT_GELU 2
#define RGBD_ACT_RELU_GRAD 3
/* OR'ed into act: bias is indexed by the row m instead of the column n (float32 [M]) — the
 * output channel of a convolution computed as C[b][o][p] = W[o][k] col[b][k][p] (NCHW). */
#define RGBD_BIAS_M 16
size_t rgbd_gemm_workspace_size(int M, int N, int batch, int splits);
int rgbd_gemm(int dtype, int a_t, int b_t, int M, int N, int K, const void* A, long long lda, long long sa,
              const void* B, long long ldb, long long sb, const float* bias, int act, const void* R, long long ldr,
              long long sr, void* C, long long ldc, long long sc, int c_f32, int batch, int splits, void* ws,
              void* stream);
/* rgbd_colsum: out[n] = sum over rows m of y[m * ld + n] (the bias gradient), float32, fixed
 * order (row chunks, then the chunks in order), one launch; ws: rgbd_colsum_workspace_size(rows,
 * N) bytes, ZERO before its first use (it starts with per-column-block tickets that every call
 * leaves at zero again).  Calls sharing a workspace must be stream-ordered. */
size_t rgbd_colsum_workspace_size(int rows, int N);
int rgbd_colsum(int dtype, const void* y, int rows, int N, long long ld, float* out, void* ws, void* stream);
/* LayerNorm over the last dimension (nn.LayerNorm(C, eps) of the decoder layers :1700-1719, the
 * pixel decoder's encoder layers :1022-1040, Swin's layernorm_before / _after :602-640):
 *   y = (x - mean) * rstd * gamma + beta, mean / rstd float32 [rows] saved for the backward.
 *   x_dtype / y_dtype: RGBD_F32 or RGBD_BF16 each (under torch.autocast a bf16 input gives a
 *   float32 output); gamma / beta float32 [C].  Statistics in float32, two passes over the
 *   register-resident row (C <= 1536).
 * rgbd_layernorm_bwd: dx = rstd * (g - mean_c(g) - xhat * mean_c(g * xhat)), g = gamma * dy,
 *   dx in x_dtype; dgamma = sum_rows dy * xhat, dbeta = sum_rows dy, float32 [C] (OVERWRITTEN;
 *   per-block partials in ws summed in block order: deterministic). */
int rgbd_layernorm_fwd(int x_dtype, const void* x, const float* gamma, const float* beta, int rows, int C,
                       float eps, int y_dtype, void* y, float* mean, float* rstd, void* stream);
/* rgbd_add_layernorm_fwd: the post-norm residual LN(x + r) of the decoder / pixel-decoder encoder
 *   layers (modeling_mask2former.py:1094-1101 / :1661-1683 `layer_norm(residual + hidden)`) in one
 *   pass: s = x + r in float32 arithmetic, rounded to the promoted dtype (float32 when either is
 *   float32, else bf16), written to s_out (the input the backward's rgbd_layernorm_bwd takes),
 *   and y = LN(s) as rgbd_layernorm_fwd; y2 (optional, bf16) receives y rounded to bf16 as well —
 *   the operand the consuming bf16 GEMMs would otherwise cast from y.  clamp > 0: y =
 *   clamp(LN(s), -clamp, clamp) (the encoder layer's clamp in training, :1094-1097; NaN kept).
 *   C % 4 == 0, C <= 1536, 16-byte aligned x / r / s_out / y / y2 (RGBD_E_SHAPE otherwise: the
 *   caller adds and normalises separately).
 * rgbd_add_layernorm_bwd: rgbd_layernorm_bwd on s with the forward's clamp undone in the
 *   gradient (zero where clamp(y) != y, y recomputed in the forward's order) and ds_bf16
 *   (optional) = ds rounded to bf16 — the gradient the bf16 branch r receives. */
int rgbd_add_layernorm_fwd(int x_dtype, const void* x, int r_dtype, const void* r, const float* gamma,
                           const float* beta, int rows, int C, float eps, float clamp, int y_dtype, void* s_out,
                           void* y, void* y2, float* mean, float* rstd, void* stream);
int rgbd_add_layernorm_bwd(int s_dtype, const void* s_in, int dy_dtype, const void* dy, const float* gamma,
                           const float* beta, const float* mean, const float* rstd, int rows, int C, float clamp,
                           void* ds, void* ds_bf16, float* dgamma, float* dbeta, void* ws, void* stream);
size_t rgbd_layernorm_bwd_workspace_size(int rows, int C);
int rgbd_layernorm_bwd(int x_dtype, const void* x, int dy_dtype, const void* dy, const float* gamma,
                       const float* mean, const float* rstd, int rows, int C, void* dx, float* dgamma,
                       float* dbeta, void* ws, void* stream);

/* f2 convolutions as GEMMs (csrc/conv.hip): the im2col operand of
 *   Y[b][o][p] = sum_k W[o][k] col[b][k][p] (+ bias[o])  (rgbd_gemm, RGBD_BIAS_M),
 * k = (c*KH + ky)*KW + kx (torch unfold's row order = the flattened OIHW weight's columns), for
 *   kernel 3: 3x3, stride 1, padding 1 (Mask2FormerPixelDecoder's FPN output convolution; its dX
 *             is the same convolution of dY with the flipped, transposed weight);
 *   kernel 4: 4x4, stride 4, padding 0, H and W multiples of 4 (SwinPatchEmbeddings.projection,
 *             modeling_swin.py; custom_model.py:330).
 * x NCHW [B][C][H][W]; col [B][C*k*k][Ho*Wo] in x's dtype (RGBD_F32 / RGBD_BF16). */
int rgbd_im2col(int dtype, const void* x, int B, int C, int H, int W, int kernel, void* col, void* stream);

/* f2 GroupNorm (nn.GroupNorm of the pixel decoder: the input projections, the FPN adapter and the
 * FPN output layer — transformers 5.15 modeling_mask2former.py Mask2FormerPixelDecoder.__init__,
 * called from Mask2FormerPixelDecoder.forward; custom_model.py:383), NCHW [B][C][HW], G groups
 * of C / G consecutive channels, biased variance (torch).  relu = 1 fuses the ReLU that follows
 * the FPN output layer's norm.  mean_rstd: [B][G][2] float32, written by the forward and read
 * by the backward.  ws: rgbd_groupnorm_workspace_size(B, C) bytes (per-channel partials).
 * Backward: dx in x's dtype; dgamma / dbeta may be NULL (no affine). */
size_t rgbd_groupnorm_workspace_size(int B, int C);
int rgbd_groupnorm_fwd(int x_dtype, const void* x, const float* gamma, const float* beta, int B, int C, int G, int HW,
                       float eps, int relu, int y_dtype, void* y, float* mean_rstd, void* ws, void* stream);
int rgbd_groupnorm_bwd(int x_dtype, const void* x, int dy_dtype, const void* dy, const float* gamma, const float* beta,
                       const float* mean_rstd, int B, int C, int G, int HW, int relu, void* dx, float* dgamma,
                       float* dbeta, void* ws, void* stream);

/* ---------------------------------------------------------------- f2 Swin-T window attention
 * The (shifted-)window self-attention core of every SwinLayer of the backbone
 * (transformers 5.15 modeling_swin.py SwinLayer.forward :529-582 with SwinAttention :418-468):
 * pad to multiples of the window, roll by -shift, 7x7 windows, softmax(q k^T * scale +
 * relative-position bias + shift mask (-100)) v, un-window, roll back, crop — by index
 * arithmetic on the original token layout.  q / k / v: dtype rows [B*H*W][ldq] (head h at
 * columns 32 h .. 32 h + 31; ldq = 3C when one GEMM produced all three), the projections of
 * the LayerNorm'ed map; bq / bk / bv float32 [C] (the projections of the zero padding rows; may
 * be NULL); table float32 [169][heads] (relative_position_bias_table); out dtype [B*H*W][ldo].
 * window == 7, 0 <= shift < 7, head_dim 32; rows 16-byte aligned. */
int rgbd_swin_window_attn(int dtype, const void* q, const void* k, const void* v, long long ldq, const float* bq,
                          const float* bk, const float* bv, const float* table, int B, int H, int W, int heads,
                          int window, int shift, float scale, void* out, long long ldo, void* stream);

/* ---------------------------------------------------------------- kernel timing (bench only)
 * When enabled, launch functions bracket their main kernel with hipEvents recorded on the
 * launch stream; rgbd_timing_read synchronises those events and returns the summed
 * milliseconds and launch count for one kernel name ("rp_conv3x3", "rp_chain", "dsam_fwd",
 * "dsam_dx", "dsam_wgrad", "decompose", "dggm_fwd", "dggm_bwd", "assemble"), then resets.
 * Do not enable while a stream is being captured into a graph. */
int rgbd_timing_enable(int on);
double rgbd_timing_read(const char* name, int* count);

#ifdef __cplusplus
}
#endif
#endif /* RGBD_HIP_H */
