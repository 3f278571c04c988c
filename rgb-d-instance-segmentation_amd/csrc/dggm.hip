// K1 (DGGM-pre + 10-channel assembly) and K2 (DGGM gated fusion fwd/bwd) for gfx950.
//
// K1 follows calculate_gradient_features (reference mask2former/utils/data_process.py:1247-1305)
// as called by map_10channel_case2 (mask2former/utils/dataloader.py:386-425).  The Sobel sums
// of u8 depth are exact integers; sqrt and the normalising division use IEEE-rounded
// intrinsics, so the planes are bit-exact to the numpy/OpenCV float32 result.
//
// K2 follows DepthGradientInjectionResidual.forward (custom_model.py:1204-1269) fused with the
// final sum backbone_k = cp1_k + cp2_k (custom_model.py:355).  One thread owns one output
// pixel and walks a channel chunk, so the resampled gate (3 bilinear taps x 4 + 1 nearest) is
// computed once per pixel and the NCHW planes are streamed with coalesced accesses.
#include "common.hpp"
#include "timing.hpp"

using namespace rgbd;

namespace {

__constant__ float kMean[3] = {0.485f, 0.456f, 0.406f};
__constant__ float kStd[3] = {0.229f, 0.224f, 0.225f};

struct PrepWs {
  uint32_t min_bits;  // min over mag > 0 (non-negative floats order as their bits)
  uint32_t max_bits;  // max over all mag
};

__global__ void k_prep_init(PrepWs* ws, int B) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) {
    ws[b].min_bits = 0x7f800000u;
    ws[b].max_bits = 0u;
  }
}

__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  if (i < 0) return -i;
  if (i >= n) return 2 * n - 2 - i;
  return i;
}

__device__ __forceinline__ float norm_u8(uint8_t v, int c) {
  // numpy: (x.astype(f32) * f32(1/255) - mean_c) / std_c, one rounding per op
  float x = __fmul_rn((float)v, 0.003921568859368563f);
  return div_rn(__fsub_rn(x, kMean[c]), kStd[c]);
}

__global__ __launch_bounds__(256) void k_prep_pass1(const uint8_t* __restrict__ rgb,
                                                    const uint8_t* __restrict__ depth, int H, int W,
                                                    float* __restrict__ pv, PrepWs* ws) {
  const int b = blockIdx.y;
  const long long HW = (long long)H * W;
  const uint8_t* d = depth + b * HW;
  float* out = pv + b * 10 * HW;
  float vmax = 0.f, vmin = __uint_as_float(0x7f800000u);
  for (int p = blockIdx.x * 256 + threadIdx.x; p < (int)HW; p += 256 * gridDim.x) {
    const int y = p / W, x = p % W;
    const uint8_t dv = d[p];
    if (rgb) {
      const uint8_t* px = rgb + (b * HW + p) * 3;
      for (int c = 0; c < 3; ++c) out[c * HW + p] = norm_u8(px[c], c);
    }
    for (int c = 0; c < 3; ++c) out[(3 + c) * HW + p] = norm_u8(dv, c);
    const int ym = reflect101(y - 1, H), yp = reflect101(y + 1, H);
    const int xm = reflect101(x - 1, W), xp = reflect101(x + 1, W);
    auto at = [&](int yy, int xx) { return (int)d[(long long)yy * W + xx]; };
    const int gx = (at(ym, xp) - at(ym, xm)) + 2 * (at(y, xp) - at(y, xm)) + (at(yp, xp) - at(yp, xm));
    const int gy = (at(yp, xm) - at(ym, xm)) + 2 * (at(yp, x) - at(ym, x)) + (at(yp, xp) - at(ym, xp));
    float mag = sqrt_rn((float)(gx * gx + gy * gy));  // exact integer argument (< 2^24)
    if (dv == 0) mag = 0.f;                               // invalid depth (:1265, :1278)
    out[6 * HW + p] = mag;                                // scratch until pass 2
    out[9 * HW + p] = mag > 0.f ? 1.f : 0.f;              // valid-gradient mask (:1282)
    vmax = fmaxf(vmax, mag);
    if (mag > 0.f) vmin = fminf(vmin, mag);
  }
  vmax = -wave_min(-vmax);
  vmin = wave_min(vmin);
  __shared__ float rmax[4], rmin[4];
  if ((threadIdx.x & 63) == 0) {
    rmax[threadIdx.x >> 6] = vmax;
    rmin[threadIdx.x >> 6] = vmin;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // one atomic pair per block (same-address atomics serialise)
    atomicMax(&ws[b].max_bits, __float_as_uint(fmaxf(fmaxf(rmax[0], rmax[1]), fmaxf(rmax[2], rmax[3]))));
    atomicMin(&ws[b].min_bits, __float_as_uint(fminf(fminf(rmin[0], rmin[1]), fminf(rmin[2], rmin[3]))));
  }
}

__global__ __launch_bounds__(256) void k_prep_pass2(int H, int W, float* __restrict__ pv,
                                                    const PrepWs* ws) {
  const int b = blockIdx.y;
  const long long HW = (long long)H * W;
  float* out = pv + b * 10 * HW;
  const uint32_t mnb = ws[b].min_bits;
  const float mn = __uint_as_float(mnb), mx = __uint_as_float(ws[b].max_bits);
  const bool scale = (mnb != 0x7f800000u) && (mx > mn);  // :1285-1293
  const float den = __fsub_rn(mx, mn);
  for (long long p = blockIdx.x * 256ll + threadIdx.x; p < HW; p += 256ll * gridDim.x) {
    const float mag = out[6 * HW + p];
    const float v = scale ? div_rn(__fsub_rn(mag, mn), den) : 0.f;
    out[6 * HW + p] = v;
    out[7 * HW + p] = v;
    out[8 * HW + p] = v;
  }
}

// ------------------------------------------------------------------ K2 fusion
struct Gate {
  float g[3];
};

// torch upsample_bilinear2d (align_corners=False) source index + nearest (legacy floor).
__device__ __forceinline__ void src_lin(int dst, int in, int out, int& i0, int& i1, float& l1) {
  const float scale = (float)in / (float)out;
  float s = scale * (dst + 0.5f) - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = s - (float)i0;
}
__device__ __forceinline__ int src_nearest(int dst, int in, int out) {
  const float scale = (float)in / (float)out;
  int s = (int)floorf((float)dst * scale);
  return s < in - 1 ? s : in - 1;
}

__device__ __forceinline__ Gate gate_at(const float* __restrict__ grad, const float* __restrict__ mask,
                                        int H, int W, int h, int w, int y, int x) {
  int y0, y1, x0, x1;
  float ly1, lx1;
  src_lin(y, H, h, y0, y1, ly1);
  src_lin(x, W, w, x0, x1, lx1);
  const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
  const long long HW = (long long)H * W;
  const float m = mask[(long long)src_nearest(y, H, h) * W + src_nearest(x, W, w)];
  Gate gt;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float* gp = grad + c * HW;
    const float v = ly0 * (lx0 * gp[(long long)y0 * W + x0] + lx1 * gp[(long long)y0 * W + x1]) +
                    ly1 * (lx0 * gp[(long long)y1 * W + x0] + lx1 * gp[(long long)y1 * W + x1]);
    gt.g[c] = v * m;  // gated_depth_grad = bilinear * nearest(mask) (:1246)
  }
  return gt;
}

constexpr int kFuseCh = 16;  // channels per thread

template <typename T>
__global__ __launch_bounds__(256) void k_dggm_fuse_fwd(const T* __restrict__ cp1, const T* __restrict__ color,
                                                       const float* __restrict__ grad,
                                                       const float* __restrict__ mask, long long pvs,
                                                       int H, int W, int C, int h, int w,
                                                       const float* __restrict__ wt,
                                                       const float* __restrict__ bias, T* __restrict__ out) {
  const int b = blockIdx.z;
  const int hw = h * w;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= hw) return;
  const int y = p / w, x = p % w;
  const Gate gt = gate_at(grad + b * pvs, mask + b * pvs, H, W, h, w, y, x);
  const int c0 = blockIdx.y * kFuseCh;
  const int c1 = min(C, c0 + kFuseCh);
  for (int c = c0; c < c1; ++c) {
    const long long o = ((long long)b * C + c) * hw + p;
    float pre = bias[c] + wt[c * 3 + 0] * gt.g[0] + wt[c * 3 + 1] * gt.g[1] + wt[c * 3 + 2] * gt.g[2];
    const float enh = pre > 0.f ? pre : 0.f;
    const float cp2 = Num<T>::to_f(color[o]) + enh;  // color_feat + depth_enhancement (:1255)
    out[o] = Num<T>::from_f(cp1 ? Num<T>::to_f(cp1[o]) + cp2 : cp2);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_dggm_fuse_bwd_partial(const T* __restrict__ dout,
                                                               const float* __restrict__ grad,
                                                               const float* __restrict__ mask,
                                                               long long pvs, int B, int H, int W,
                                                               int C, int h, int w,
                                                               const float* __restrict__ wt,
                                                               const float* __restrict__ bias,
                                                               float* __restrict__ partial) {
  // partial[tile][c][4] = sum over the tile's pixels of dout*relu'(pre) * (1, g0, g1, g2).
  // A "tile" is the pixel range [tile*ppt, (tile+1)*ppt): each thread accumulates its pixels in
  // registers first, then one block reduction per channel (fixed order: deterministic).
  __shared__ float red[4][kFuseCh][4];
  const int hw = h * w;
  const long long P = (long long)B * hw;
  const long long ppt = ((P + gridDim.x - 1) / gridDim.x + 255) / 256 * 256;
  const long long q0 = (long long)blockIdx.x * ppt;
  const int c0 = blockIdx.y * kFuseCh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float acc[kFuseCh][4];
#pragma unroll
  for (int cc = 0; cc < kFuseCh; ++cc)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[cc][j] = 0.f;
  for (long long q = q0 + threadIdx.x; q < q0 + ppt && q < P; q += 256) {
    const int b = (int)(q / hw), p = (int)(q % hw);
    const Gate gt = gate_at(grad + b * pvs, mask + b * pvs, H, W, h, w, p / w, p % w);
#pragma unroll
    for (int cc = 0; cc < kFuseCh; ++cc) {
      const int c = c0 + cc;
      if (c >= C) break;
      const float pre = bias[c] + wt[c * 3 + 0] * gt.g[0] + wt[c * 3 + 1] * gt.g[1] + wt[c * 3 + 2] * gt.g[2];
      const float d = pre > 0.f ? Num<T>::to_f(dout[((long long)b * C + c) * hw + p]) : 0.f;
      acc[cc][0] += d;
      acc[cc][1] += d * gt.g[0];
      acc[cc][2] += d * gt.g[1];
      acc[cc][3] += d * gt.g[2];
    }
  }
#pragma unroll
  for (int cc = 0; cc < kFuseCh; ++cc)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float s = wave_sum(acc[cc][j]);
      if (lane == 0) red[wave][cc][j] = s;
    }
  __syncthreads();
  if (threadIdx.x < kFuseCh * 4) {
    const int cc = threadIdx.x >> 2, j = threadIdx.x & 3;
    if (c0 + cc >= C) return;
    const float s = ((red[0][cc][j] + red[1][cc][j]) + red[2][cc][j]) + red[3][cc][j];
    partial[((long long)blockIdx.x * C + c0 + cc) * 4 + j] = s;
  }
}

__global__ __launch_bounds__(256) void k_dggm_fuse_bwd_final(const float* __restrict__ partial, int ntiles, int C,
                                                              float* __restrict__ dw, float* __restrict__ db) {
  // one block per (c, j); fixed-shape tree over the tiles: deterministic
  __shared__ float red[256];
  const int t = blockIdx.x;
  float s = 0.f;
  for (int i = threadIdx.x; i < ntiles; i += 256) s += partial[(long long)i * C * 4 + t];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x) return;
  const int c = t >> 2, j = t & 3;
  if (j == 0)
    db[c] = red[0];
  else
    dw[c * 3 + (j - 1)] = red[0];
}

}  // namespace

extern "C" {

size_t rgbd_assemble_workspace_size(int B) { return align256(sizeof(PrepWs) * (size_t)(B > 0 ? B : 1)); }

int rgbd_assemble_pixel_values(const uint8_t* rgb_u8, const uint8_t* depth_u8, int B, int H, int W,
                               float* pv, void* ws, void* stream) {
  RGBD_REQUIRE(depth_u8 && pv && ws, RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && H > 0 && W > 0, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  PrepWs* w = (PrepWs*)ws;
  TimerScope ts("assemble", s);
  k_prep_init<<<ceil_div(B, 64), 64, 0, s>>>(w, B);
  const long long HW = (long long)H * W;
  RGBD_REQUIRE(HW < (1ll << 31), RGBD_E_SHAPE);
  dim3 grid((unsigned)std::min<long long>(ceil_div(HW, 256), 128), B);
  k_prep_pass1<<<grid, 256, 0, s>>>(rgb_u8, depth_u8, H, W, pv, w);
  k_prep_pass2<<<grid, 256, 0, s>>>(H, W, pv, w);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_dggm_fuse_fwd(int dtype, const void* cp1, const void* color, const float* grad,
                       const float* mask, long long pv_batch_stride, int B, int H, int W, int C,
                       int h, int w, const float* weight, const float* bias, void* out,
                       void* stream) {
  RGBD_REQUIRE(color && grad && mask && weight && bias && out, RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && H > 0 && W > 0 && C > 0 && h > 0 && w > 0, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(ceil_div((long long)h * w, 256), ceil_div(C, kFuseCh), B);
  TimerScope ts("dggm_fwd", s);
  if (dtype == RGBD_F32)
    k_dggm_fuse_fwd<float><<<grid, 256, 0, s>>>((const float*)cp1, (const float*)color, grad, mask,
                                                pv_batch_stride, H, W, C, h, w, weight, bias, (float*)out);
  else if (dtype == RGBD_BF16)
    k_dggm_fuse_fwd<bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)cp1, (const bf16_t*)color, grad, mask,
                                                 pv_batch_stride, H, W, C, h, w, weight, bias,
                                                 (bf16_t*)out);
  else
    return RGBD_E_DTYPE;
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

static int dggm_bwd_tiles(int B, int h, int w) { return std::min(ceil_div((long long)B * h * w, 256), 64); }

size_t rgbd_dggm_fuse_bwd_workspace_size(int B, int C, int h, int w) {
  return align256(sizeof(float) * 4 * (size_t)C * dggm_bwd_tiles(B, h, w));
}

int rgbd_dggm_fuse_bwd(int dtype, const void* dout, const float* grad, const float* mask,
                       long long pv_batch_stride, int B, int H, int W, int C, int h, int w,
                       const float* weight, const float* bias, float* dweight, float* dbias,
                       void* ws, void* stream) {
  RGBD_REQUIRE(dout && grad && mask && weight && bias && dweight && dbias && ws, RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && H > 0 && W > 0 && C > 0 && h > 0 && w > 0, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  TimerScope ts("dggm_bwd", s);
  const int ntiles = dggm_bwd_tiles(B, h, w);
  dim3 grid(ntiles, ceil_div(C, kFuseCh));
  float* partial = (float*)ws;
  if (dtype == RGBD_F32)
    k_dggm_fuse_bwd_partial<float><<<grid, 256, 0, s>>>((const float*)dout, grad, mask, pv_batch_stride,
                                                        B, H, W, C, h, w, weight, bias, partial);
  else if (dtype == RGBD_BF16)
    k_dggm_fuse_bwd_partial<bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)dout, grad, mask, pv_batch_stride,
                                                         B, H, W, C, h, w, weight, bias, partial);
  else
    return RGBD_E_DTYPE;
  k_dggm_fuse_bwd_final<<<C * 4, 256, 0, s>>>(partial, ntiles, C, dweight, dbias);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
