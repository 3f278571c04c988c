// f2: the pixel decoder's multi-scale deformable attention core on gfx950.
//
// Reference: multi_scale_deformable_attention (transformers 5.15 modeling_mask2former.py:798-837),
// called by Mask2FormerPixelDecoderEncoderMultiscaleDeformableAttention.forward (:1011) in each of
// the 6 pixel-decoder encoder layers.  The reference splits the value per level, runs one
// grid_sample per level over a [B*heads, D, H, W] re-layout of it (a transposed copy of the value
// per level), stacks the samples [B*heads, D, Q, L*P], multiplies by the attention weights and sums.
//
// Here one launch does all levels and points: a group of D / 8 lanes (D = head dim, 32 for the
// reference config) owns one (image, query, head); each lane keeps 8 channels.  Per (level, point) the
// group computes the bilinear source position once (grid = 2*loc - 1, ix = ((grid + 1) * W - 1) / 2,
// grid_sample's align_corners=False rule with zero padding), reads the four taps as D contiguous
// channels of the [B][S][heads][D] value (16 bytes per lane), and accumulates weight * sample in
// registers — no per-level copy, no [.., Q, L*P] intermediate.
// Backward in two launches: k_msda_bwd_query reduces, per (level, point), go . sample
// (attention-weight gradient) and go . d sample / d(ix, iy) (sampling-location gradient);
// k_msda_bwd_value gathers the value gradient into LDS tiles (no global atomics).  Bound: gather /
// L2 latency (the value of a level is at most a few MB per image) and LDS atomics.
#include <algorithm>

#include "common.hpp"

namespace rgbd {
namespace {

constexpr int MSDA_MAX_L = 4;

struct MsdaLevels {
  int L;
  int H[MSDA_MAX_L], W[MSDA_MAX_L], start[MSDA_MAX_L];
};

struct Tap {
  int idx[4];     // spatial index within the level, -1 when outside (zero padding)
  float w[4];     // bilinear weights (x0y0, x1y0, x0y1, x1y1)
  float lx, ly;   // fractional parts (for the location gradient)
};

__device__ __forceinline__ Tap msda_tap(float locx, float locy, int H, int W) {
  // grid_sample(align_corners=False): grid = 2*loc - 1 (computed by the reference in the tensor
  // op), unnormalised with ((grid + 1) * size - 1) / 2
  const float gx = 2.f * locx - 1.f, gy = 2.f * locy - 1.f;
  // clamped into [-2, size + 1]: beyond that all four taps are padding either way, and the
  // float -> int conversion stays defined
  const float ix = fminf(fmaxf(((gx + 1.f) * (float)W - 1.f) / 2.f, -2.f), (float)W + 1.f);
  const float iy = fminf(fmaxf(((gy + 1.f) * (float)H - 1.f) / 2.f, -2.f), (float)H + 1.f);
  const float fx = floorf(ix), fy = floorf(iy);
  const int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
  Tap t;
  t.lx = ix - fx;
  t.ly = iy - fy;
  const float wx0 = 1.f - t.lx, wy0 = 1.f - t.ly;
  t.w[0] = wx0 * wy0;
  t.w[1] = t.lx * wy0;
  t.w[2] = wx0 * t.ly;
  t.w[3] = t.lx * t.ly;
  const bool vx0 = x0 >= 0 && x0 < W, vx1 = x1 >= 0 && x1 < W, vy0 = y0 >= 0 && y0 < H, vy1 = y1 >= 0 && y1 < H;
  t.idx[0] = vx0 && vy0 ? y0 * W + x0 : -1;
  t.idx[1] = vx1 && vy0 ? y0 * W + x1 : -1;
  t.idx[2] = vx0 && vy1 ? y1 * W + x0 : -1;
  t.idx[3] = vx1 && vy1 ? y1 * W + x1 : -1;
  return t;
}

// 8 consecutive channels of a value row, widened to float (16 B of bf16 or 32 B of float)
__device__ __forceinline__ void ld8(const bf16_t* p, float (&v)[8]) {
  const uint4 w = *reinterpret_cast<const uint4*>(p);
  const uint32_t x[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(x[i] << 16);
    v[2 * i + 1] = __uint_as_float(x[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void ld8(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void st8(bf16_t* p, const float (&v)[8]) {
  *reinterpret_cast<uint4*>(p) =
      make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
}
__device__ __forceinline__ void st8(float* p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// Forward: a group of G = D / 8 lanes owns one (image, query, head); lane j of the group keeps
// channels 8j..8j+7, so every tap is one 16-byte (bf16) load per lane and a wave-instruction
// gathers 64 / G value rows at once.
template <typename T, int D>
__global__ __launch_bounds__(256) void k_msda_fwd(const T* __restrict__ value, MsdaLevels lv, int S, int Q, int NH,
                                                  int P, const float* __restrict__ loc, const float* __restrict__ attw,
                                                  long long nqh, T* __restrict__ out) {
  constexpr int G = D / 8;
  const int j = threadIdx.x % G;
  const long long qh = (long long)blockIdx.x * (256 / G) + threadIdx.x / G;
  if (qh >= nqh) return;
  const int h = (int)(qh % NH);
  const long long b = (qh / NH) / Q;
  const float* lq = loc + qh * lv.L * P * 2;
  const float* wq = attw + qh * lv.L * P;
  const T* vb = value + b * S * NH * D + (long long)h * D + 8 * j;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int l = 0; l < lv.L; ++l) {
    const int H = lv.H[l], W = lv.W[l];
    const T* vl = vb + (long long)lv.start[l] * NH * D;
    for (int p = 0; p < P; ++p) {
      const int k = l * P + p;
      const Tap t = msda_tap(lq[2 * k], lq[2 * k + 1], H, W);
      float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (t.idx[e] >= 0) {
          float v[8];
          ld8(vl + (long long)t.idx[e] * NH * D, v);
#pragma unroll
          for (int c = 0; c < 8; ++c) s[c] += t.w[e] * v[c];
        }
      const float a = wq[k];
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[c] += a * s[c];
    }
  }
  st8(out + qh * D + 8 * j, acc);
}

template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Backward, per query: the attention-weight gradient go . sample and the sampling-location
// gradient go . d sample / d(ix, iy), the forward's lane groups reducing over their 8-channel
// slices with shuffles.  No atomics: the value gradient is k_msda_bwd_value's.
template <typename T, int D>
__global__ __launch_bounds__(256) void k_msda_bwd_query(const T* __restrict__ value, MsdaLevels lv, int S, int Q,
                                                        int NH, int P, const float* __restrict__ loc,
                                                        const float* __restrict__ attw, const T* __restrict__ gout,
                                                        long long nqh, float* __restrict__ gloc,
                                                        float* __restrict__ gattw) {
  constexpr int G = D / 8;
  const int j = threadIdx.x % G;
  const long long qh = (long long)blockIdx.x * (256 / G) + threadIdx.x / G;
  // every lane of a group takes part in the shuffles: out-of-range groups run with zero weight
  const bool live = qh < nqh;
  const long long q0 = live ? qh : 0;
  const int h = (int)(q0 % NH);
  const long long b = (q0 / NH) / Q;
  const float* lq = loc + q0 * lv.L * P * 2;
  const float* wq = attw + q0 * lv.L * P;
  const T* vb = value + b * S * NH * D + (long long)h * D + 8 * j;
  float go[8];
  ld8(gout + q0 * D + 8 * j, go);
  if (!live)
#pragma unroll
    for (int c = 0; c < 8; ++c) go[c] = 0.f;
  for (int l = 0; l < lv.L; ++l) {
    const int H = lv.H[l], W = lv.W[l];
    const T* vl = vb + (long long)lv.start[l] * NH * D;
    for (int p = 0; p < P; ++p) {
      const int k = l * P + p;
      const Tap t = msda_tap(lq[2 * k], lq[2 * k + 1], H, W);
      float v[4][8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (t.idx[e] >= 0) {
          ld8(vl + (long long)t.idx[e] * NH * D, v[e]);
        } else {
#pragma unroll
          for (int c = 0; c < 8; ++c) v[e][c] = 0.f;
        }
      }
      float gw = 0.f, gx = 0.f, gy = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float smp = t.w[0] * v[0][c] + t.w[1] * v[1][c] + t.w[2] * v[2][c] + t.w[3] * v[3][c];
        // d sample / d ix, d iy (zero-padded taps are zeros)
        const float dsx = (1.f - t.ly) * (v[1][c] - v[0][c]) + t.ly * (v[3][c] - v[2][c]);
        const float dsy = (1.f - t.lx) * (v[2][c] - v[0][c]) + t.lx * (v[3][c] - v[1][c]);
        gw += go[c] * smp;
        gx += go[c] * dsx;
        gy += go[c] * dsy;
      }
      gw = group_sum<G>(gw);
      gx = group_sum<G>(gx);
      gy = group_sum<G>(gy);
      if (live && j == 0) {
        const float a = wq[k];
        gattw[q0 * lv.L * P + k] = gw;
        // ix = loc * W - 1/2 through grid = 2 loc - 1: d ix / d loc = W
        gloc[(q0 * lv.L * P + k) * 2] = a * gx * (float)W;
        gloc[(q0 * lv.L * P + k) * 2 + 1] = a * gy * (float)H;
      }
    }
  }
}

// Backward, value gradient, gathered per value band instead of scattered per query: a workgroup
// owns (image, head, level, 8-channel chunk, band of MSDA_BAND pixels of the level) as a float32
// tile in LDS, runs over every query of its image, and adds a * w_tap * go into the tile for each
// tap that falls in its band (LDS atomics); then writes the tile once.  Every element of the
// value gradient belongs to exactly one workgroup: plain stores, no memset, no global atomics
// (grid_sample's backward scatters with global atomics; at the C2 shape those were 2.5 GB of
// atomic traffic per call).  Thread = (query, channel pair); 128 queries per pass, 8 waves per
// workgroup (the tile is the only LDS user: one workgroup per CU, so it brings its own waves);
// each thread keeps the loads of 4 queries in flight (the scan is latency-bound: per query 48
// scattered bytes of locations / weights / gradient).
constexpr int MSDA_C = 8;                                         // channels per workgroup
constexpr int MSDA_BAND = 163840 / (MSDA_C * (int)sizeof(float));  // pixels per LDS tile (160 KiB)

struct MsdaBands {
  int nb[MSDA_MAX_L];     // bands per level
  int first[MSDA_MAX_L];  // first work index of the level (levels in order, largest first in grid)
};

template <typename T, int D>
__global__ __launch_bounds__(512) void k_msda_bwd_value(MsdaLevels lv, MsdaBands bd, int S, int Q, int NH, int P,
                                                        const float* __restrict__ loc, const float* __restrict__ attw,
                                                        const T* __restrict__ gout, int BNH, int vec4,
                                                        float* __restrict__ gvalue) {
  extern __shared__ float tile[];  // [band px][MSDA_C]
  constexpr int NCH = D / MSDA_C;
  // work index -> (level, band, chunk, b * NH + h); within a level: bh fastest
  int w = blockIdx.x, l = 0;
  while (l + 1 < lv.L && w >= bd.first[l + 1]) ++l;
  w -= bd.first[l];
  const int bh = w % BNH;
  const int chunk = (w / BNH) % NCH;
  const int band = w / (BNH * NCH);
  const int h = bh % NH, b = bh / NH;
  const int H = lv.H[l], W = lv.W[l], HW = H * W;
  const int lo = band * MSDA_BAND, hi = min(HW, lo + MSDA_BAND), n = hi - lo;
  for (int i = threadIdx.x; i < n * MSDA_C; i += 512) tile[i] = 0.f;
  __syncthreads();
  const int cp = threadIdx.x & 3;  // channel pair 2cp, 2cp+1 of the chunk
  const int c0 = chunk * MSDA_C + 2 * cp;
  auto add_point = [&](float lx, float ly, float a, float g0, float g1) {
    const Tap t = msda_tap(lx, ly, H, W);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ix = t.idx[e] - lo;
      if (t.idx[e] >= 0 && ix >= 0 && ix < n) {
        const float f = a * t.w[e];
        atomicAdd(&tile[ix * MSDA_C + 2 * cp], f * g0);
        atomicAdd(&tile[ix * MSDA_C + 2 * cp + 1], f * g1);
      }
    }
  };
  constexpr int U = 4;  // queries per thread in flight: their loads issue together (latency-bound)
  if (vec4) {  // P == 4, locations / weights 16-byte aligned
    for (int q0 = threadIdx.x >> 2; q0 < Q; q0 += 128 * U) {
      float4 la[U], lb[U], wa[U];
      float ga[U], gb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = q0 + 128 * u;
        if (q < Q) {
          const long long qh = ((long long)b * Q + q) * NH + h;
          const float* lq = loc + (qh * lv.L + l) * 8;  // 4 points x (x, y): 32 B, 32-B aligned
          la[u] = *reinterpret_cast<const float4*>(lq);
          lb[u] = *reinterpret_cast<const float4*>(lq + 4);
          wa[u] = *reinterpret_cast<const float4*>(attw + (qh * lv.L + l) * 4);
          ga[u] = Num<T>::to_f(gout[qh * D + c0]);
          gb[u] = Num<T>::to_f(gout[qh * D + c0 + 1]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (q0 + 128 * u >= Q) break;
        add_point(la[u].x, la[u].y, wa[u].x, ga[u], gb[u]);
        add_point(la[u].z, la[u].w, wa[u].y, ga[u], gb[u]);
        add_point(lb[u].x, lb[u].y, wa[u].z, ga[u], gb[u]);
        add_point(lb[u].z, lb[u].w, wa[u].w, ga[u], gb[u]);
      }
    }
  } else {
    for (int q = threadIdx.x >> 2; q < Q; q += 128) {
      const long long qh = ((long long)b * Q + q) * NH + h;
      const float* lq = loc + (qh * lv.L + l) * P * 2;
      const float* wq = attw + (qh * lv.L + l) * P;
      const float g0 = Num<T>::to_f(gout[qh * D + c0]), g1 = Num<T>::to_f(gout[qh * D + c0 + 1]);
      for (int p = 0; p < P; ++p) add_point(lq[2 * p], lq[2 * p + 1], wq[p], g0, g1);
    }
  }
  __syncthreads();
  float* gv = gvalue + (((long long)b * S + lv.start[l] + lo) * NH + h) * D + chunk * MSDA_C;
  for (int i = threadIdx.x; i < n * 2; i += 512) {  // 16 B (4 channels) per store
    const int px = i >> 1, half = i & 1;
    *reinterpret_cast<float4*>(gv + (long long)px * NH * D + 4 * half) =
        *reinterpret_cast<const float4*>(&tile[px * MSDA_C + 4 * half]);
  }
}

int msda_levels(int L, const int* shapes_host, MsdaLevels& lv, int& S) {
  if (L < 1 || L > MSDA_MAX_L || !shapes_host) return RGBD_E_SHAPE;
  lv.L = L;
  S = 0;
  for (int l = 0; l < L; ++l) {
    lv.H[l] = shapes_host[2 * l];
    lv.W[l] = shapes_host[2 * l + 1];
    if (lv.H[l] <= 0 || lv.W[l] <= 0) return RGBD_E_SHAPE;
    lv.start[l] = S;
    S += lv.H[l] * lv.W[l];
  }
  return RGBD_OK;
}

template <typename T, int D>
void launch_fwd(const void* value, const MsdaLevels& lv, int S, int Q, int NH, int P, const float* loc,
                const float* attw, long long nqh, void* out, hipStream_t s) {
  const dim3 grid((unsigned)ceil_div(nqh, 256 / (D / 8)));
  k_msda_fwd<T, D><<<grid, 256, 0, s>>>((const T*)value, lv, S, Q, NH, P, loc, attw, nqh, (T*)out);
}

template <typename T, int D>
int launch_bwd(const void* value, const MsdaLevels& lv, int B, int S, int Q, int NH, int P, const float* loc,
               const float* attw, const void* gout, float* gvalue, float* gloc, float* gattw, hipStream_t s) {
  const long long nqh = (long long)B * Q * NH;
  k_msda_bwd_query<T, D><<<(unsigned)ceil_div(nqh, 256 / (D / 8)), 256, 0, s>>>(
      (const T*)value, lv, S, Q, NH, P, loc, attw, (const T*)gout, nqh, gloc, gattw);
  MsdaBands bd;
  int work = 0, max_px = 0;
  for (int l = 0; l < lv.L; ++l) {
    const int hw = lv.H[l] * lv.W[l];
    bd.nb[l] = (hw + MSDA_BAND - 1) / MSDA_BAND;
    bd.first[l] = work;
    work += bd.nb[l] * (D / MSDA_C) * B * NH;
    max_px = std::max(max_px, std::min(hw, MSDA_BAND));
  }
  const size_t lds = (size_t)max_px * MSDA_C * sizeof(float);
  static const hipError_t attr = hipFuncSetAttribute((const void*)k_msda_bwd_value<T, D>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  if (attr != hipSuccess) return (int)attr;
  const int vec4 = P == 4 && ((uintptr_t)loc & 15) == 0 && ((uintptr_t)attw & 15) == 0;
  k_msda_bwd_value<T, D><<<work, 512, lds, s>>>(lv, bd, S, Q, NH, P, loc, attw, (const T*)gout, B * NH, vec4, gvalue);
  return RGBD_OK;
}

}  // namespace
}  // namespace rgbd

using namespace rgbd;

extern "C" int rgbd_msda_fwd(int dtype, const void* value, int B, int L, const int* shapes_host, int NH, int D,
                             int Q, int P, const float* loc, const float* attw, void* out, void* stream) {
  RGBD_REQUIRE(value && loc && attw && out && B > 0 && NH > 0 && Q > 0 && P > 0, RGBD_E_ARG);
  RGBD_REQUIRE(D == 16 || D == 32 || D == 64, RGBD_E_SHAPE);
  RGBD_REQUIRE(dtype == RGBD_F32 || dtype == RGBD_BF16, RGBD_E_DTYPE);
  RGBD_REQUIRE(((uintptr_t)value & 15) == 0 && ((uintptr_t)out & 15) == 0, RGBD_E_SHAPE);  // 16-byte lane loads
  MsdaLevels lv;
  int S = 0;
  const int rc = msda_levels(L, shapes_host, lv, S);
  if (rc) return rc;
  const long long nqh = (long long)B * Q * NH;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_F32) {
    if (D == 32) launch_fwd<float, 32>(value, lv, S, Q, NH, P, loc, attw, nqh, out, s);
    else if (D == 64) launch_fwd<float, 64>(value, lv, S, Q, NH, P, loc, attw, nqh, out, s);
    else launch_fwd<float, 16>(value, lv, S, Q, NH, P, loc, attw, nqh, out, s);
  } else {
    if (D == 32) launch_fwd<bf16_t, 32>(value, lv, S, Q, NH, P, loc, attw, nqh, out, s);
    else if (D == 64) launch_fwd<bf16_t, 64>(value, lv, S, Q, NH, P, loc, attw, nqh, out, s);
    else launch_fwd<bf16_t, 16>(value, lv, S, Q, NH, P, loc, attw, nqh, out, s);
  }
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

extern "C" int rgbd_msda_bwd(int dtype, const void* value, int B, int L, const int* shapes_host, int NH, int D,
                             int Q, int P, const float* loc, const float* attw, const void* gout, float* gvalue,
                             float* gloc, float* gattw, void* stream) {
  RGBD_REQUIRE(value && loc && attw && gout && gvalue && gloc && gattw && B > 0 && NH > 0 && Q > 0 && P > 0,
               RGBD_E_ARG);
  RGBD_REQUIRE(D == 16 || D == 32 || D == 64, RGBD_E_SHAPE);
  RGBD_REQUIRE(dtype == RGBD_F32 || dtype == RGBD_BF16, RGBD_E_DTYPE);
  RGBD_REQUIRE(((uintptr_t)value & 15) == 0 && ((uintptr_t)gout & 15) == 0 && ((uintptr_t)gvalue & 15) == 0,
               RGBD_E_SHAPE);
  MsdaLevels lv;
  int S = 0;
  const int rc = msda_levels(L, shapes_host, lv, S);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  int r;
  if (dtype == RGBD_F32) {
    if (D == 32) r = launch_bwd<float, 32>(value, lv, B, S, Q, NH, P, loc, attw, gout, gvalue, gloc, gattw, s);
    else if (D == 64) r = launch_bwd<float, 64>(value, lv, B, S, Q, NH, P, loc, attw, gout, gvalue, gloc, gattw, s);
    else r = launch_bwd<float, 16>(value, lv, B, S, Q, NH, P, loc, attw, gout, gvalue, gloc, gattw, s);
  } else {
    if (D == 32) r = launch_bwd<bf16_t, 32>(value, lv, B, S, Q, NH, P, loc, attw, gout, gvalue, gloc, gattw, s);
    else if (D == 64) r = launch_bwd<bf16_t, 64>(value, lv, B, S, Q, NH, P, loc, attw, gout, gvalue, gloc, gattw, s);
    else r = launch_bwd<bf16_t, 16>(value, lv, B, S, Q, NH, P, loc, attw, gout, gvalue, gloc, gattw, s);
  }
  if (r != RGBD_OK) return r;
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}
