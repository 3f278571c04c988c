// K1 (DGGM-pre + 10-channel assembly) and K2 (DGGM gated fusion fwd/bwd) for gfx950.
//
// K1 follows calculate_gradient_features (reference mask2former/utils/data_process.py:1247-1305)
// as called by map_10channel_case2 (mask2former/utils/dataloader.py:386-425).  The Sobel sums
// of u8 depth are exact integers; sqrt and the normalising division use IEEE-rounded
// intrinsics, so the planes are bit-exact to the numpy/OpenCV float32 result.
//
// K2 follows DepthGradientInjectionResidual.forward (custom_model.py:1204-1269) fused with the
// final sum backbone_k = cp1_k + cp2_k (custom_model.py:355).  A workgroup computes the
// resampled gate (3 bilinear taps x 4 + 1 nearest) of a pixel tile once into LDS and streams 32
// channel planes of that tile with vector accesses (8 pixels per lane where h*w allows).
#include <cstdlib>

#include "common.hpp"
#include "timing.hpp"

using namespace rgbd;

namespace {

// image_mean / image_std of the reference's processor config
// (mask2former/checkpoints/standard/preprocessor_config.json), rounded to float32 as
// transformers' normalize does (np.array(mean, dtype=image.dtype)).  The config's std[1],
// 0.2239999920129776, is one float32 ulp below 0.224f.
__constant__ float kMean[3] = {0.48500001430511475f, 0.4560000002384186f, 0.4059999883174896f};
__constant__ float kStd[3] = {0.2290000021457672f, 0.2239999920129776f, 0.22499999403953552f};
constexpr double kRescale = 0.00392156862745098;  // rescale_factor of the same config

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
  // Mask2FormerImageProcessor (dataloader.py:405-410): transformers image_transforms.rescale
  // multiplies in float64 and rounds once to float32; normalize is (x - mean_c) / std_c in
  // float32, one rounding per op.
  const float x = (float)__dmul_rn((double)v, kRescale);
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

// Quad variants (W % 4 == 0, every NYUv2 / RealSense width): a thread owns 4 x-consecutive
// pixels — one 4-byte depth load per stencil row plus the two reflected edge bytes, three 4-byte
// RGB loads, and one 16-byte store per output plane — instead of 9 byte loads and 8 scalar
// stores per pixel.  Same arithmetic, same order per pixel, so the planes stay bit-exact.
__device__ __forceinline__ void row6(const uint8_t* __restrict__ row, int x0, int W, int (&v)[6]) {
  const uint32_t c = *reinterpret_cast<const uint32_t*>(row + x0);
  v[0] = row[reflect101(x0 - 1, W)];
  v[1] = c & 0xff;
  v[2] = (c >> 8) & 0xff;
  v[3] = (c >> 16) & 0xff;
  v[4] = c >> 24;
  v[5] = row[reflect101(x0 + 4, W)];
}

__global__ __launch_bounds__(256) void k_prep_pass1_q(const uint8_t* __restrict__ rgb,
                                                      const uint8_t* __restrict__ depth, int H, int W,
                                                      float* __restrict__ pv, float2* __restrict__ part) {
  const int b = blockIdx.y;
  const long long HW = (long long)H * W;
  const int WQ = W >> 2;
  const uint8_t* d = depth + b * HW;
  float* out = pv + b * 10 * HW;
  float vmax = 0.f, vmin = __uint_as_float(0x7f800000u);
  const int nq = (int)(HW >> 2);
  for (int q = blockIdx.x * 256 + threadIdx.x; q < nq; q += 256 * gridDim.x) {
    const int y = q / WQ, x0 = (q - y * WQ) * 4;
    const long long p = (long long)y * W + x0;
    int up[6], mid[6], dn[6];
    row6(d + (long long)reflect101(y - 1, H) * W, x0, W, up);
    row6(d + (long long)y * W, x0, W, mid);
    row6(d + (long long)reflect101(y + 1, H) * W, x0, W, dn);
    if (rgb) {
      const uint32_t* px = reinterpret_cast<const uint32_t*>(rgb + (b * HW + p) * 3);
      const uint32_t w0 = px[0], w1 = px[1], w2 = px[2];
      const uint8_t c[12] = {(uint8_t)w0, (uint8_t)(w0 >> 8), (uint8_t)(w0 >> 16), (uint8_t)(w0 >> 24),
                             (uint8_t)w1, (uint8_t)(w1 >> 8), (uint8_t)(w1 >> 16), (uint8_t)(w1 >> 24),
                             (uint8_t)w2, (uint8_t)(w2 >> 8), (uint8_t)(w2 >> 16), (uint8_t)(w2 >> 24)};
#pragma unroll
      for (int ch = 0; ch < 3; ++ch)
        *reinterpret_cast<float4*>(out + ch * HW + p) =
            make_float4(norm_u8(c[ch], ch), norm_u8(c[3 + ch], ch), norm_u8(c[6 + ch], ch), norm_u8(c[9 + ch], ch));
    }
#pragma unroll
    for (int ch = 0; ch < 3; ++ch)
      *reinterpret_cast<float4*>(out + (3 + ch) * HW + p) =
          make_float4(norm_u8(mid[1], ch), norm_u8(mid[2], ch), norm_u8(mid[3], ch), norm_u8(mid[4], ch));
    float mag[4], msk[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int l = i, c = i + 1, r = i + 2;
      const int gx = (up[r] - up[l]) + 2 * (mid[r] - mid[l]) + (dn[r] - dn[l]);
      const int gy = (dn[l] - up[l]) + 2 * (dn[c] - up[c]) + (dn[r] - up[r]);
      float m = sqrt_rn((float)(gx * gx + gy * gy));  // exact integer argument (< 2^24)
      if (mid[c] == 0) m = 0.f;                         // invalid depth (:1265, :1278)
      mag[i] = m;
      msk[i] = m > 0.f ? 1.f : 0.f;                     // valid-gradient mask (:1282)
      vmax = fmaxf(vmax, m);
      if (m > 0.f) vmin = fminf(vmin, m);
    }
    *reinterpret_cast<float4*>(out + 6 * HW + p) = make_float4(mag[0], mag[1], mag[2], mag[3]);  // scratch
    *reinterpret_cast<float4*>(out + 9 * HW + p) = make_float4(msk[0], msk[1], msk[2], msk[3]);
  }
  vmax = -wave_min(-vmax);
  vmin = wave_min(vmin);
  __shared__ float rmax[4], rmin[4];
  if ((threadIdx.x & 63) == 0) {
    rmax[threadIdx.x >> 6] = vmax;
    rmin[threadIdx.x >> 6] = vmin;
  }
  __syncthreads();
  // one (min, max) partial per block, reduced by pass 2 (no same-address atomics: 256 blocks of
  // one image serialising on one L2 line cost ~25 us)
  if (threadIdx.x == 0)
    part[(long long)b * gridDim.x + blockIdx.x] =
        make_float2(fminf(fminf(rmin[0], rmin[1]), fminf(rmin[2], rmin[3])),
                    fmaxf(fmaxf(rmax[0], rmax[1]), fmaxf(rmax[2], rmax[3])));
}

__global__ __launch_bounds__(256) void k_prep_pass2_q(int H, int W, float* __restrict__ pv,
                                                      const float2* __restrict__ part, int nparts) {
  const int b = blockIdx.y;
  const long long HW = (long long)H * W;
  float* out = pv + b * 10 * HW;
  float lmn = __uint_as_float(0x7f800000u), lmx = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) {
    const float2 v = part[(long long)b * nparts + i];
    lmn = fminf(lmn, v.x);
    lmx = fmaxf(lmx, v.y);
  }
  lmn = wave_min(lmn);
  lmx = -wave_min(-lmx);
  __shared__ float smn[4], smx[4];
  if ((threadIdx.x & 63) == 0) {
    smn[threadIdx.x >> 6] = lmn;
    smx[threadIdx.x >> 6] = lmx;
  }
  __syncthreads();
  const float mn = fminf(fminf(smn[0], smn[1]), fminf(smn[2], smn[3]));
  const float mx = fmaxf(fmaxf(smx[0], smx[1]), fmaxf(smx[2], smx[3]));
  const uint32_t mnb = __float_as_uint(mn);
  const bool scale = (mnb != 0x7f800000u) && (mx > mn);  // :1285-1293
  const float den = __fsub_rn(mx, mn);
  for (long long p = (blockIdx.x * 256ll + threadIdx.x) * 4; p < HW; p += 1024ll * gridDim.x) {
    const float4 m = *reinterpret_cast<const float4*>(out + 6 * HW + p);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (scale)
      v = make_float4(div_rn(__fsub_rn(m.x, mn), den), div_rn(__fsub_rn(m.y, mn), den),
                      div_rn(__fsub_rn(m.z, mn), den), div_rn(__fsub_rn(m.w, mn), den));
    *reinterpret_cast<float4*>(out + 6 * HW + p) = v;
    *reinterpret_cast<float4*>(out + 7 * HW + p) = v;
    *reinterpret_cast<float4*>(out + 8 * HW + p) = v;
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

// Block = a tile of 64*PX pixels of one image x 32 channels; the tile's gates are computed once
// into LDS, each wave then owns 8 channels and each lane PX consecutive pixels: one 16-B (PX=8),
// 8-B (PX=4) or 2-B (PX=1) access per bf16 channel plane, PX the largest of 8/4/1 dividing h*w
// (so a lane's pixels are all valid or all past the end).  All 8 channels' loads are issued
// before any arithmetic.
constexpr int kBlkCh = 32;
constexpr int kWaveCh = 8;
constexpr int kRedStride = 36;  // floats per lane row of the bwd wave reduction

template <typename T, int PX> struct PxN;
template <int PX> struct PxN<float, PX> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[PX]) {
    if constexpr (PX == 1) {
      v[0] = *p;
    } else {
#pragma unroll
      for (int q = 0; q < PX / 4; ++q) {
        const float4 a = ((const float4*)p)[q];
        v[4 * q] = a.x; v[4 * q + 1] = a.y; v[4 * q + 2] = a.z; v[4 * q + 3] = a.w;
      }
    }
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[PX]) {
    if constexpr (PX == 1) {
      *p = v[0];
    } else {
#pragma unroll
      for (int q = 0; q < PX / 4; ++q) ((float4*)p)[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    }
  }
};
template <int PX> struct PxN<bf16_t, PX> {
  static __device__ __forceinline__ void load(const bf16_t* p, float (&v)[PX]) {
    if constexpr (PX == 1) {
      v[0] = bf16_to_f32(*p);
    } else {
      uint32_t w[PX / 2];
      if constexpr (PX == 8) {
        const uint4 u = *(const uint4*)p;
        w[0] = u.x; w[1] = u.y; w[2] = u.z; w[3] = u.w;
      } else {
        const uint2 u = *(const uint2*)p;
        w[0] = u.x; w[1] = u.y;
      }
#pragma unroll
      for (int j = 0; j < PX / 2; ++j) {
        v[2 * j] = __uint_as_float(w[j] << 16);
        v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
      }
    }
  }
  static __device__ __forceinline__ void store(bf16_t* p, const float (&v)[PX]) {
    if constexpr (PX == 1) {
      *p = f32_to_bf16(v[0]);
    } else {
      uint32_t w[PX / 2];
#pragma unroll
      for (int j = 0; j < PX / 2; ++j) w[j] = (uint32_t)f32_to_bf16(v[2 * j]) | ((uint32_t)f32_to_bf16(v[2 * j + 1]) << 16);
      if constexpr (PX == 8)
        *(uint4*)p = make_uint4(w[0], w[1], w[2], w[3]);
      else
        *(uint2*)p = make_uint2(w[0], w[1]);
    }
  }
};


template <int PX>
struct TileGates {
  float g[3][PX];
  int p;       // first pixel of this lane within the image
  bool valid;  // the lane's PX pixels are inside the image
};

// Stage the tile's gates in LDS and return this lane's PX of them.
// Also stages the block's 32 channels of (w0, w1, w2, bias) into swb (clamped past C).
template <int PX>
__device__ __forceinline__ TileGates<PX> stage_gates(float (*sg)[512], float4* swb, const float* __restrict__ grad,
                                                     const float* __restrict__ mask, int H, int W, int h,
                                                     int w, int p0, const float* __restrict__ wt,
                                                     const float* __restrict__ bias, int C, int by) {
  constexpr int TP = 64 * PX;
  const int hw = h * w;
  if (threadIdx.x < kBlkCh) {
    const int c = min(by * kBlkCh + (int)threadIdx.x, C - 1);
    swb[threadIdx.x] = make_float4(wt[c * 3 + 0], wt[c * 3 + 1], wt[c * 3 + 2], bias[c]);
  }
#pragma unroll
  for (int i0 = 0; i0 < TP; i0 += 256) {
    const int i = i0 + threadIdx.x;
    const int p = p0 + i;
    if (i < TP) {
      Gate gt = {{0.f, 0.f, 0.f}};
      if (p < hw) gt = gate_at(grad, mask, H, W, h, w, p / w, p % w);
      sg[0][i] = gt.g[0];
      sg[1][i] = gt.g[1];
      sg[2][i] = gt.g[2];
    }
  }
  __syncthreads();
  TileGates<PX> t;
  const int lane = threadIdx.x & 63;
  t.p = p0 + PX * lane;
  t.valid = t.p < hw;
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int j = 0; j < PX; ++j) t.g[c][j] = sg[c][PX * lane + j];
  return t;
}

// One (pixel tile bx, 32-channel block by) of the fused forward; the kernels below map block
// indices onto it (one scale per launch, or all scales in one launch).
// One pixel's 8 channels [c0, c0+8) of an NHWC map -> v[cc][j] (cc < 8); C % 8 == 0.
template <typename T, int PX>
__device__ __forceinline__ void load_nhwc8(const T* p, float (&v)[kWaveCh][PX], int j) {
  if constexpr (sizeof(T) == 2) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[2 * q][j] = __uint_as_float(w[q] << 16);
      v[2 * q + 1][j] = __uint_as_float(w[q] & 0xffff0000u);
    }
  } else {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    v[0][j] = a.x; v[1][j] = a.y; v[2][j] = a.z; v[3][j] = a.w;
    v[4][j] = b.x; v[5][j] = b.y; v[6][j] = b.z; v[7][j] = b.w;
  }
}

template <typename T, int PX, bool HAS1, bool CP1_NHWC = false>
__device__ __forceinline__ void dggm_fwd_block(float (*sg)[512], float4* swb, int bx, int by,
                                               const T* __restrict__ cp1, const T* __restrict__ color,
                                               const float* __restrict__ grad, const float* __restrict__ mask,
                                               long long pvs, int H, int W, int C, int h, int w,
                                               const float* __restrict__ wt, const float* __restrict__ bias,
                                               T* __restrict__ out) {
  constexpr int TP = 64 * PX;
  const int hw = h * w, tpi = (hw + TP - 1) / TP;
  const int b = bx / tpi, p0 = (bx % tpi) * TP;
  const TileGates<PX> t = stage_gates<PX>(sg, swb, grad + b * pvs, mask + b * pvs, H, W, h, w, p0, wt, bias, C, by);
  const int cw = by * kBlkCh + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * kWaveCh;
  if (!t.valid || cw >= C) return;
  float col[kWaveCh][PX], y[kWaveCh][PX];
#pragma unroll
  for (int cc = 0; cc < kWaveCh; ++cc) {
    const long long o = ((long long)b * C + min(cw + cc, C - 1)) * hw + t.p;
    PxN<T, PX>::load(color + o, col[cc]);
    if constexpr (HAS1 && !CP1_NHWC) PxN<T, PX>::load(cp1 + o, y[cc]);
  }
  if constexpr (HAS1 && CP1_NHWC)  // cp1 NHWC (the DSAM cascade's layout): 8 channels per pixel load
#pragma unroll
    for (int j = 0; j < PX; ++j) load_nhwc8<T, PX>(cp1 + ((long long)b * hw + t.p + j) * C + cw, y, j);
  __builtin_amdgcn_sched_barrier(0);  // keep the whole load batch ahead of the first use
#pragma unroll
  for (int cc = 0; cc < kWaveCh; ++cc) {
    const int c = min(cw + cc, C - 1);
    const float4 wb = swb[c - by * kBlkCh];
    const float w0 = wb.x, w1 = wb.y, w2 = wb.z, bc = wb.w;
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      const float pre = bc + w0 * t.g[0][j] + w1 * t.g[1][j] + w2 * t.g[2][j];
      const float cp2 = col[cc][j] + (pre > 0.f ? pre : 0.f);  // color_feat + depth_enhancement (:1255)
      y[cc][j] = HAS1 ? y[cc][j] + cp2 : cp2;
    }
  }
  // stores after all arithmetic: a per-channel guard between loads and uses would let the
  // compiler sink each load into its guarded block (one load latency per channel)
  if (cw + kWaveCh <= C) {
#pragma unroll
    for (int cc = 0; cc < kWaveCh; ++cc) PxN<T, PX>::store(out + ((long long)b * C + cw + cc) * hw + t.p, y[cc]);
  } else {
#pragma unroll
    for (int cc = 0; cc < kWaveCh; ++cc)
      if (cw + cc < C) PxN<T, PX>::store(out + ((long long)b * C + cw + cc) * hw + t.p, y[cc]);
  }
}

template <typename T, int PX, bool HAS1>
__global__ __launch_bounds__(256) void k_dggm_fuse_fwd(const T* __restrict__ cp1, const T* __restrict__ color,
                                                       const float* __restrict__ grad,
                                                       const float* __restrict__ mask, long long pvs,
                                                       int H, int W, int C, int h, int w,
                                                       const float* __restrict__ wt,
                                                       const float* __restrict__ bias, T* __restrict__ out) {
  __shared__ float sg[3][512];
  __shared__ float4 swb[kBlkCh];
  dggm_fwd_block<T, PX, HAS1>(sg, swb, blockIdx.x, blockIdx.y, cp1, color, grad, mask, pvs, H, W, C, h, w, wt, bias,
                              out);
}

// partial[tile][c][4] = sum over the tile's pixels of dout*relu'(pre) * (1, g0, g1, g2).  Each
// lane sums its PX pixels for the wave's 8 channels (32 values), then the wave sums the 64
// lanes' values through LDS in fixed order (deterministic).
template <typename T, int PX>
__device__ __forceinline__ void dggm_bwd_block(float (*sg)[512], float4* swb, float (*sred)[64 * kRedStride], int bx,
                                               int by, const T* __restrict__ dout, const float* __restrict__ grad,
                                               const float* __restrict__ mask, long long pvs, int H, int W, int C,
                                               int h, int w, const float* __restrict__ wt,
                                               const float* __restrict__ bias, float* __restrict__ partial) {
  constexpr int TP = 64 * PX;
  const int hw = h * w, tpi = (hw + TP - 1) / TP;
  const int b = bx / tpi, p0 = (bx % tpi) * TP;
  const TileGates<PX> t = stage_gates<PX>(sg, swb, grad + b * pvs, mask + b * pvs, H, W, h, w, p0, wt, bias, C, by);
  const int lane = threadIdx.x & 63;
  const int cw = by * kBlkCh + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * kWaveCh;
  if (cw >= C) return;
  float d[kWaveCh][PX];
  if (t.valid) {
#pragma unroll
    for (int cc = 0; cc < kWaveCh; ++cc) PxN<T, PX>::load(dout + ((long long)b * C + min(cw + cc, C - 1)) * hw + t.p, d[cc]);
    __builtin_amdgcn_sched_barrier(0);  // keep the whole load batch ahead of the first use
  } else {
#pragma unroll
    for (int cc = 0; cc < kWaveCh; ++cc)
#pragma unroll
      for (int j = 0; j < PX; ++j) d[cc][j] = 0.f;
  }
  float v[4 * kWaveCh];
#pragma unroll
  for (int cc = 0; cc < kWaveCh; ++cc) {
    const int c = min(cw + cc, C - 1);
    const float4 wb = swb[c - by * kBlkCh];
    const float w0 = wb.x, w1 = wb.y, w2 = wb.z, bc = wb.w;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      const float pre = bc + w0 * t.g[0][j] + w1 * t.g[1][j] + w2 * t.g[2][j];
      const float dj = pre > 0.f ? d[cc][j] : 0.f;
      s0 += dj;
      s1 += dj * t.g[0][j];
      s2 += dj * t.g[1][j];
      s3 += dj * t.g[2][j];
    }
    v[4 * cc + 0] = s0;
    v[4 * cc + 1] = s1;
    v[4 * cc + 2] = s2;
    v[4 * cc + 3] = s3;
  }
  // wave reduction through LDS: row = lane (32 sums, stride 36 floats), then lane (idx, half)
  // adds rows half*32 .. half*32+31 of column idx; independent reads, fixed order
  float* red = sred[threadIdx.x >> 6];
#pragma unroll
  for (int q = 0; q < 8; ++q)
    *(float4*)&red[lane * kRedStride + 4 * q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int idx = lane & 31, half = lane >> 5;
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 32; ++r) s += red[(half * 32 + r) * kRedStride + idx];
  s += __shfl_xor(s, 32);
  const int c = cw + (idx >> 2);
  if (lane < 32 && c < C) partial[((long long)bx * C + c) * 4 + (idx & 3)] = s;
}

template <typename T, int PX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_dggm_fuse_bwd_partial(const T* __restrict__ dout,
                                                               const float* __restrict__ grad,
                                                               const float* __restrict__ mask,
                                                               long long pvs, int H, int W, int C, int h,
                                                               int w, const float* __restrict__ wt,
                                                               const float* __restrict__ bias,
                                                               float* __restrict__ partial) {
  __shared__ float sg[3][512];
  __shared__ float4 swb[kBlkCh];
  __shared__ __attribute__((aligned(16))) float sred[4][64 * kRedStride];
  dggm_bwd_block<T, PX>(sg, swb, sred, blockIdx.x, blockIdx.y, dout, grad, mask, pvs, H, W, C, h, w, wt, bias,
                        partial);
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

// ---- all scales in one launch (the four backbone scales of one step): a flat block index is
// mapped onto (scale, pixel tile, channel block); the vector width PX is per scale, uniform per
// block.  Cuts three launch/drain tails per direction on the small scales.
constexpr int DGGM_MAX_SCALES = 4;
struct DggmScaleArgs {
  const void* cp1;
  const void* color;  // fwd input / bwd: dout
  void* out;
  const float* wt;
  const float* bias;
  float* partial;     // bwd
  float* dw;          // bwd outputs
  float* db;
  int C, h, w, px, nbx, blk0, tiles;
  int cp1_nhwc;       // fwd: cp1 is NHWC [B][h][w][C] (C % 8 == 0)
};
struct DggmMulti {
  DggmScaleArgs s[DGGM_MAX_SCALES];
  int n, total;
};

__device__ __forceinline__ int dggm_scale_of(const DggmMulti& m, int blk) {
  int k = 0;
#pragma unroll
  for (int i = 1; i < DGGM_MAX_SCALES; ++i)
    if (i < m.n && blk >= m.s[i].blk0) k = i;
  return k;
}

template <typename T>
__global__ __launch_bounds__(256) void k_dggm_fuse_fwd_multi(DggmMulti m, const float* __restrict__ grad,
                                                             const float* __restrict__ mask, long long pvs, int H,
                                                             int W) {
  __shared__ float sg[3][512];
  __shared__ float4 swb[kBlkCh];
  const int k = dggm_scale_of(m, blockIdx.x);
  const DggmScaleArgs& d = m.s[k];
  const int local = blockIdx.x - d.blk0, bx = local % d.nbx, by = local / d.nbx;
  const T* cp1 = (const T*)d.cp1;
  if (cp1 && d.cp1_nhwc) {
    if (d.px == 8)
      dggm_fwd_block<T, 8, true, true>(sg, swb, bx, by, cp1, (const T*)d.color, grad, mask, pvs, H, W, d.C, d.h, d.w,
                                       d.wt, d.bias, (T*)d.out);
    else if (d.px == 4)
      dggm_fwd_block<T, 4, true, true>(sg, swb, bx, by, cp1, (const T*)d.color, grad, mask, pvs, H, W, d.C, d.h, d.w,
                                       d.wt, d.bias, (T*)d.out);
    else
      dggm_fwd_block<T, 1, true, true>(sg, swb, bx, by, cp1, (const T*)d.color, grad, mask, pvs, H, W, d.C, d.h, d.w,
                                       d.wt, d.bias, (T*)d.out);
  } else if (cp1) {
    if (d.px == 8)
      dggm_fwd_block<T, 8, true>(sg, swb, bx, by, cp1, (const T*)d.color, grad, mask, pvs, H, W, d.C, d.h, d.w, d.wt,
                                 d.bias, (T*)d.out);
    else if (d.px == 4)
      dggm_fwd_block<T, 4, true>(sg, swb, bx, by, cp1, (const T*)d.color, grad, mask, pvs, H, W, d.C, d.h, d.w, d.wt,
                                 d.bias, (T*)d.out);
    else
      dggm_fwd_block<T, 1, true>(sg, swb, bx, by, cp1, (const T*)d.color, grad, mask, pvs, H, W, d.C, d.h, d.w, d.wt,
                                 d.bias, (T*)d.out);
  } else {
    if (d.px == 8)
      dggm_fwd_block<T, 8, false>(sg, swb, bx, by, nullptr, (const T*)d.color, grad, mask, pvs, H, W, d.C, d.h, d.w,
                                  d.wt, d.bias, (T*)d.out);
    else if (d.px == 4)
      dggm_fwd_block<T, 4, false>(sg, swb, bx, by, nullptr, (const T*)d.color, grad, mask, pvs, H, W, d.C, d.h, d.w,
                                  d.wt, d.bias, (T*)d.out);
    else
      dggm_fwd_block<T, 1, false>(sg, swb, bx, by, nullptr, (const T*)d.color, grad, mask, pvs, H, W, d.C, d.h, d.w,
                                  d.wt, d.bias, (T*)d.out);
  }
}

template <typename T>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_dggm_fuse_bwd_multi(
    DggmMulti m, const float* __restrict__ grad, const float* __restrict__ mask, long long pvs, int H, int W) {
  __shared__ float sg[3][512];
  __shared__ float4 swb[kBlkCh];
  __shared__ __attribute__((aligned(16))) float sred[4][64 * kRedStride];
  const int k = dggm_scale_of(m, blockIdx.x);
  const DggmScaleArgs& d = m.s[k];
  const int local = blockIdx.x - d.blk0, bx = local % d.nbx, by = local / d.nbx;
  if (d.px == 8)
    dggm_bwd_block<T, 8>(sg, swb, sred, bx, by, (const T*)d.color, grad, mask, pvs, H, W, d.C, d.h, d.w, d.wt, d.bias,
                         d.partial);
  else if (d.px == 4)
    dggm_bwd_block<T, 4>(sg, swb, sred, bx, by, (const T*)d.color, grad, mask, pvs, H, W, d.C, d.h, d.w, d.wt, d.bias,
                         d.partial);
  else
    dggm_bwd_block<T, 1>(sg, swb, sred, bx, by, (const T*)d.color, grad, mask, pvs, H, W, d.C, d.h, d.w, d.wt, d.bias,
                         d.partial);
}

// the tile sums of every scale reduced in one launch: block = (scale, c, j), same fixed tree
__global__ __launch_bounds__(256) void k_dggm_fuse_bwd_final_multi(DggmMulti m) {
  __shared__ float red[256];
  int k = 0, t = blockIdx.x;
  while (k + 1 < m.n && t >= 4 * m.s[k].C) {
    t -= 4 * m.s[k].C;
    ++k;
  }
  const DggmScaleArgs& d = m.s[k];
  float s = 0.f;
  for (int i = threadIdx.x; i < d.tiles; i += 256) s += d.partial[(long long)i * d.C * 4 + t];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x) return;
  const int c = t >> 2, j = t & 3;
  if (j == 0)
    d.db[c] = red[0];
  else
    d.dw[c * 3 + (j - 1)] = red[0];
}


int dggm_px(int h, int w) {
  const long long hw = (long long)h * w;
  return hw % 8 == 0 ? 8 : (hw % 4 == 0 ? 4 : 1);
}

template <typename T, int PX>
void launch_fwd(const void* cp1, const void* color, const float* grad, const float* mask, long long pvs,
                       int B, int H, int W, int C, int h, int w, const float* wt, const float* bias, void* out,
                       hipStream_t s) {
  dim3 grid(B * ceil_div((long long)h * w, 64 * PX), ceil_div(C, kBlkCh));
  if (cp1)
    k_dggm_fuse_fwd<T, PX, true><<<grid, 256, 0, s>>>((const T*)cp1, (const T*)color, grad, mask, pvs, H, W, C, h, w,
                                                      wt, bias, (T*)out);
  else
    k_dggm_fuse_fwd<T, PX, false><<<grid, 256, 0, s>>>(nullptr, (const T*)color, grad, mask, pvs, H, W, C, h, w, wt,
                                                       bias, (T*)out);
}

template <typename T, int PX>
void launch_bwd(const void* dout, const float* grad, const float* mask, long long pvs, int B, int H, int W,
                       int C, int h, int w, const float* wt, const float* bias, float* partial, hipStream_t s) {
  dim3 grid(B * ceil_div((long long)h * w, 64 * PX), ceil_div(C, kBlkCh));
  k_dggm_fuse_bwd_partial<T, PX><<<grid, 256, 0, s>>>((const T*)dout, grad, mask, pvs, H, W, C, h, w, wt, bias,
                                                       partial);
}

#define RGBD_DGGM_DISPATCH(FN, T, PX, ...) \
  do {                                     \
    if ((PX) == 8)                         \
      FN<T, 8>(__VA_ARGS__);               \
    else if ((PX) == 4)                    \
      FN<T, 4>(__VA_ARGS__);               \
    else                                   \
      FN<T, 1>(__VA_ARGS__);               \
  } while (0)

}  // namespace

extern "C" {

constexpr int kPrepMaxParts = 1024;  // pass-1 blocks per image (quad path)
size_t rgbd_assemble_workspace_size(int B) {
  const size_t nb = (size_t)(B > 0 ? B : 1);
  return align256(sizeof(PrepWs) * nb) + align256(sizeof(float2) * kPrepMaxParts * nb);
}

int rgbd_assemble_pixel_values(const uint8_t* rgb_u8, const uint8_t* depth_u8, int B, int H, int W,
                               float* pv, void* ws, void* stream) {
  RGBD_REQUIRE(depth_u8 && pv && ws, RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && H > 0 && W > 0, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  PrepWs* w = (PrepWs*)ws;
  TimerScope ts("assemble", s);
  const long long HW = (long long)H * W;
  RGBD_REQUIRE(HW < (1ll << 31), RGBD_E_SHAPE);
  if (W % 4 == 0 && ((uintptr_t)pv & 15) == 0 && ((uintptr_t)depth_u8 & 3) == 0 && ((uintptr_t)rgb_u8 & 3) == 0) {
    const int nparts = (int)std::min<long long>(std::min<long long>(ceil_div(HW / 4, 256), std::max(2048 / B, 16)),
                                                kPrepMaxParts);
    float2* part = (float2*)((char*)ws + align256(sizeof(PrepWs) * (size_t)B));
    dim3 grid((unsigned)nparts, B);
    k_prep_pass1_q<<<grid, 256, 0, s>>>(rgb_u8, depth_u8, H, W, pv, part);
    k_prep_pass2_q<<<grid, 256, 0, s>>>(H, W, pv, part, nparts);
  } else {
    k_prep_init<<<ceil_div(B, 64), 64, 0, s>>>(w, B);
    dim3 grid((unsigned)std::min<long long>(ceil_div(HW, 256), 128), B);
    k_prep_pass1<<<grid, 256, 0, s>>>(rgb_u8, depth_u8, H, W, pv, w);
    k_prep_pass2<<<grid, 256, 0, s>>>(H, W, pv, w);
  }
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_dggm_fuse_fwd(int dtype, const void* cp1, const void* color, const float* grad,
                       const float* mask, long long pv_batch_stride, int B, int H, int W, int C,
                       int h, int w, const float* weight, const float* bias, void* out,
                       void* stream) {
  RGBD_REQUIRE(color && grad && mask && weight && bias && out, RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && H > 0 && W > 0 && C > 0 && h > 0 && w > 0, RGBD_E_ARG);
  RGBD_REQUIRE((long long)h * w < (1ll << 31), RGBD_E_SHAPE);
  hipStream_t s = (hipStream_t)stream;
  TimerScope ts("dggm_fwd", s);
  const int px = dggm_px(h, w);
  if (dtype == RGBD_F32)
    RGBD_DGGM_DISPATCH(launch_fwd, float, px, cp1, color, grad, mask, pv_batch_stride, B, H, W, C, h, w, weight,
                       bias, out, s);
  else if (dtype == RGBD_BF16)
    RGBD_DGGM_DISPATCH(launch_fwd, bf16_t, px, cp1, color, grad, mask, pv_batch_stride, B, H, W, C, h, w, weight,
                       bias, out, s);
  else
    return RGBD_E_DTYPE;
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

static int dggm_bwd_tiles(int B, int h, int w) { return B * ceil_div((long long)h * w, 64 * dggm_px(h, w)); }

size_t rgbd_dggm_fuse_bwd_workspace_size(int B, int C, int h, int w) {
  return align256(sizeof(float) * 4 * (size_t)C * dggm_bwd_tiles(B, h, w));
}

int rgbd_dggm_fuse_bwd(int dtype, const void* dout, const float* grad, const float* mask,
                       long long pv_batch_stride, int B, int H, int W, int C, int h, int w,
                       const float* weight, const float* bias, float* dweight, float* dbias,
                       void* ws, void* stream) {
  RGBD_REQUIRE(dout && grad && mask && weight && bias && dweight && dbias && ws, RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && H > 0 && W > 0 && C > 0 && h > 0 && w > 0, RGBD_E_ARG);
  RGBD_REQUIRE((long long)h * w < (1ll << 31), RGBD_E_SHAPE);
  hipStream_t s = (hipStream_t)stream;
  TimerScope ts("dggm_bwd", s);
  const int ntiles = dggm_bwd_tiles(B, h, w), px = dggm_px(h, w);
  float* partial = (float*)ws;
  if (dtype == RGBD_F32)
    RGBD_DGGM_DISPATCH(launch_bwd, float, px, dout, grad, mask, pv_batch_stride, B, H, W, C, h, w, weight, bias,
                       partial, s);
  else if (dtype == RGBD_BF16)
    RGBD_DGGM_DISPATCH(launch_bwd, bf16_t, px, dout, grad, mask, pv_batch_stride, B, H, W, C, h, w, weight, bias,
                       partial, s);
  else
    return RGBD_E_DTYPE;
  k_dggm_fuse_bwd_final<<<C * 4, 256, 0, s>>>(partial, ntiles, C, dweight, dbias);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}


// Multi-scale forms: scales given as host arrays (n <= 4), one launch (fwd) / two launches (bwd).
static int dggm_multi_setup(int n, const int* C, const int* h, const int* w, int B, DggmMulti& m) {
  RGBD_REQUIRE(n >= 1 && n <= DGGM_MAX_SCALES && C && h && w, RGBD_E_ARG);
  m.n = n;
  int blk = 0;
  for (int k = 0; k < n; ++k) {
    RGBD_REQUIRE(C[k] > 0 && h[k] > 0 && w[k] > 0 && (long long)h[k] * w[k] < (1ll << 31), RGBD_E_ARG);
    DggmScaleArgs& d = m.s[k];
    d.C = C[k];
    d.h = h[k];
    d.w = w[k];
    d.px = dggm_px(h[k], w[k]);
    d.nbx = B * ceil_div((long long)h[k] * w[k], 64 * d.px);
    d.tiles = d.nbx;
    d.blk0 = blk;
    blk += d.nbx * ceil_div(C[k], kBlkCh);
  }
  m.total = blk;
  return RGBD_OK;
}

size_t rgbd_dggm_fuse_bwd_multi_workspace_size(int n, const int* C_host, const int* h_host, const int* w_host,
                                               int B) {
  size_t tot = 0;
  for (int k = 0; k < n; ++k) tot += rgbd_dggm_fuse_bwd_workspace_size(B, C_host[k], h_host[k], w_host[k]);
  return tot;
}

int rgbd_dggm_fuse_fwd_multi(int dtype, int n, const void* const* cp1_host, const void* const* color_host,
                             void* const* out_host, const float* const* weight_host, const float* const* bias_host,
                             const int* C_host, const int* h_host, const int* w_host, const float* grad,
                             const float* mask, long long pv_batch_stride, int B, int H, int W, void* stream) {
  return rgbd_dggm_fuse_fwd_multi_mixed(dtype, n, cp1_host, 0, color_host, out_host, weight_host, bias_host, C_host,
                                        h_host, w_host, grad, mask, pv_batch_stride, B, H, W, stream);
}

int rgbd_dggm_fuse_fwd_multi_mixed(int dtype, int n, const void* const* cp1_host, int cp1_nhwc_mask,
                                   const void* const* color_host, void* const* out_host,
                                   const float* const* weight_host, const float* const* bias_host, const int* C_host,
                                   const int* h_host, const int* w_host, const float* grad, const float* mask,
                                   long long pv_batch_stride, int B, int H, int W, void* stream) {
  RGBD_REQUIRE(grad && mask && color_host && out_host && weight_host && bias_host && B > 0 && H > 0 && W > 0,
               RGBD_E_ARG);
  DggmMulti m;
  const int rc = dggm_multi_setup(n, C_host, h_host, w_host, B, m);
  if (rc) return rc;
  for (int k = 0; k < n; ++k) {
    RGBD_REQUIRE(color_host[k] && out_host[k] && weight_host[k] && bias_host[k], RGBD_E_ARG);
    m.s[k].cp1 = cp1_host ? cp1_host[k] : nullptr;
    m.s[k].cp1_nhwc = (cp1_nhwc_mask >> k) & 1;
    RGBD_REQUIRE(!m.s[k].cp1_nhwc || (C_host[k] % 8 == 0 && m.s[k].cp1), RGBD_E_SHAPE);
    m.s[k].color = color_host[k];
    m.s[k].out = out_host[k];
    m.s[k].wt = weight_host[k];
    m.s[k].bias = bias_host[k];
    m.s[k].partial = nullptr;
    m.s[k].dw = m.s[k].db = nullptr;
  }
  hipStream_t s = (hipStream_t)stream;
  TimerScope ts("dggm_fwd", s);
  if (dtype == RGBD_F32)
    k_dggm_fuse_fwd_multi<float><<<m.total, 256, 0, s>>>(m, grad, mask, pv_batch_stride, H, W);
  else if (dtype == RGBD_BF16)
    k_dggm_fuse_fwd_multi<bf16_t><<<m.total, 256, 0, s>>>(m, grad, mask, pv_batch_stride, H, W);
  else
    return RGBD_E_DTYPE;
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_dggm_fuse_bwd_multi(int dtype, int n, const void* const* dout_host, const float* const* weight_host,
                             const float* const* bias_host, float* const* dweight_host, float* const* dbias_host,
                             const int* C_host, const int* h_host, const int* w_host, const float* grad,
                             const float* mask, long long pv_batch_stride, int B, int H, int W, void* ws,
                             void* stream) {
  RGBD_REQUIRE(grad && mask && dout_host && weight_host && bias_host && dweight_host && dbias_host && ws && B > 0 &&
                   H > 0 && W > 0,
               RGBD_E_ARG);
  DggmMulti m;
  const int rc = dggm_multi_setup(n, C_host, h_host, w_host, B, m);
  if (rc) return rc;
  char* p = (char*)ws;
  int nfin = 0;
  for (int k = 0; k < n; ++k) {
    RGBD_REQUIRE(dout_host[k] && weight_host[k] && bias_host[k] && dweight_host[k] && dbias_host[k], RGBD_E_ARG);
    m.s[k].cp1 = nullptr;
    m.s[k].color = dout_host[k];
    m.s[k].out = nullptr;
    m.s[k].wt = weight_host[k];
    m.s[k].bias = bias_host[k];
    m.s[k].partial = (float*)p;
    m.s[k].dw = dweight_host[k];
    m.s[k].db = dbias_host[k];
    p += rgbd_dggm_fuse_bwd_workspace_size(B, C_host[k], h_host[k], w_host[k]);
    nfin += 4 * C_host[k];
  }
  hipStream_t s = (hipStream_t)stream;
  TimerScope ts("dggm_bwd", s);
  if (dtype == RGBD_F32)
    k_dggm_fuse_bwd_multi<float><<<m.total, 256, 0, s>>>(m, grad, mask, pv_batch_stride, H, W);
  else if (dtype == RGBD_BF16)
    k_dggm_fuse_bwd_multi<bf16_t><<<m.total, 256, 0, s>>>(m, grad, mask, pv_batch_stride, H, W);
  else
    return RGBD_E_DTYPE;
  k_dggm_fuse_bwd_final_multi<<<nfin, 256, 0, s>>>(m);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
