// f3: the point-sampled mask terms of the Mask2Former loss and matcher (gfx950).
//
// Reference (third-party, called by the model the reference trains, custom_model.py:37-53 via
// finetuning.py's Trainer): transformers 5.15 modeling_mask2former.py
//   sample_point                          :245-275  (grid_sample, bilinear, align_corners=False, zeros)
//   pair_wise_sigmoid_cross_entropy_loss  :350-375  } the matcher's point-sampled costs (:445-470)
//   pair_wise_dice_loss                   :328-347  }
//   sigmoid_cross_entropy_loss / dice_loss :278-325   the matched-pair mask losses (loss_masks, :580-630)
// The random point coordinates, the uncertainty top-k and the index gathers stay torch calls in
// the wrapper (rgbd_amd/point_loss.py) so the RNG stream and the selected points are the
// reference's own; these kernels do the sampling and the reductions over the 12 544 points.
//
//   k_point_sample      one thread per (map, point): the four-tap bilinear sample, ATen's
//                       grid_sampler formula and tap order
//   k_point_sample_bwd  the transposed scatter (f32 atomics into the map gradient, as ATen's
//                       grid_sampler_2d_backward does)
//   k_match_cost        one workgroup per (image, query): per point the positive / negative BCE
//                       and the sigmoid of the query's logit, reduced against every target's
//                       labels in one pass over the points (T targets in registers per chunk)
//   k_point_losses      one workgroup per matched pair: BCE mean and the dice term of the row;
//                       the backward forms d/dlogit of both from the same sums
#include <cmath>

#include "common.hpp"

using namespace rgbd;

namespace {

// ATen grid_sampler_compute_source_index (align_corners=False): ((g + 1) * size - 1) / 2, with
// g = 2 * c - 1 as sample_point forms it.
__device__ __forceinline__ float src_index(float c, int size) {
  const float g = __fsub_rn(__fmul_rn(2.f, c), 1.f);  // two torch elementwise ops in sample_point
  // ATen's kernel is built with FMA contraction: ((g + 1) * size - 1) / 2 as fma(g + 1, size, -1) / 2
  return __fdiv_rn(__builtin_fmaf(__fadd_rn(g, 1.f), (float)size, -1.f), 2.f);
}

struct Taps {
  int x0, y0;
  float nw, ne, sw, se;
};
__device__ __forceinline__ Taps taps(float cx, float cy, int h, int w) {
  const float ix = src_index(cx, w), iy = src_index(cy, h);
  Taps t;
  const float fx = floorf(ix), fy = floorf(iy);
  t.x0 = (int)fx;
  t.y0 = (int)fy;
  const float x1 = fx + 1.f, y1 = fy + 1.f;
  t.nw = __fmul_rn(__fsub_rn(x1, ix), __fsub_rn(y1, iy));
  t.ne = __fmul_rn(__fsub_rn(ix, fx), __fsub_rn(y1, iy));
  t.sw = __fmul_rn(__fsub_rn(x1, ix), __fsub_rn(iy, fy));
  t.se = __fmul_rn(__fsub_rn(ix, fx), __fsub_rn(iy, fy));
  return t;
}

// out[m][p] = bilinear sample of map m at coords[m / per][p] (x = width, y = height): a point set
// per group of `per` consecutive maps
template <typename T>
__global__ __launch_bounds__(256) void k_point_sample(const T* __restrict__ maps, int nmaps, int h, int w,
                                                      const float* __restrict__ coords, int per, int P,
                                                      float* __restrict__ out) {
  const long long i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= (long long)nmaps * P) return;
  const int m = (int)(i / P), p = (int)(i % P);
  const float2 c = reinterpret_cast<const float2*>(coords)[(long long)(m / per) * P + p];
  const Taps t = taps(c.x, c.y, h, w);
  const T* mp = maps + (long long)m * h * w;
  auto in = [&](int y, int x) { return x >= 0 && x < w && y >= 0 && y < h; };
  // the four taps loaded unconditionally (an outside tap reads element 0 and is not added), so
  // they are in flight together instead of one branch and one memory round trip each
  auto at = [&](int y, int x) { return Num<T>::to_f(mp[in(y, x) ? y * w + x : 0]); };  // bf16 widens exactly
  const float a0 = at(t.y0, t.x0), a1 = at(t.y0, t.x0 + 1), a2 = at(t.y0 + 1, t.x0), a3 = at(t.y0 + 1, t.x0 + 1);
  float v = 0.f;  // ATen accumulates nw, ne, sw, se in that order (contracted to FMAs)
  v = in(t.y0, t.x0) ? __builtin_fmaf(a0, t.nw, v) : v;
  v = in(t.y0, t.x0 + 1) ? __builtin_fmaf(a1, t.ne, v) : v;
  v = in(t.y0 + 1, t.x0) ? __builtin_fmaf(a2, t.sw, v) : v;
  v = in(t.y0 + 1, t.x0 + 1) ? __builtin_fmaf(a3, t.se, v) : v;
  out[i] = v;
}

__global__ __launch_bounds__(256) void k_point_sample_bwd(const float* __restrict__ gout, int nmaps, int h, int w,
                                                          const float* __restrict__ coords, int per, int P,
                                                          float* __restrict__ gmaps) {
  const long long i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= (long long)nmaps * P) return;
  const int m = (int)(i / P), p = (int)(i % P);
  const float g = gout[i];
  if (g == 0.f) return;
  const float2 c = reinterpret_cast<const float2*>(coords)[(long long)(m / per) * P + p];
  const Taps t = taps(c.x, c.y, h, w);
  float* mp = gmaps + (long long)m * h * w;
  auto in = [&](int y, int x) { return x >= 0 && x < w && y >= 0 && y < h; };
  if (in(t.y0, t.x0)) atomicAdd(mp + t.y0 * w + t.x0, g * t.nw);
  if (in(t.y0, t.x0 + 1)) atomicAdd(mp + t.y0 * w + t.x0 + 1, g * t.ne);
  if (in(t.y0 + 1, t.x0)) atomicAdd(mp + (t.y0 + 1) * w + t.x0, g * t.sw);
  if (in(t.y0 + 1, t.x0 + 1)) atomicAdd(mp + (t.y0 + 1) * w + t.x0 + 1, g * t.se);
}

// BCEWithLogits (ATen binary_cross_entropy_with_logits, no weights): with m = max(-x, 0),
// log-sum = log(exp(-m) + exp(-x - m)); target 1: m + ls; target 0: x + m + ls.
__device__ __forceinline__ void bce_pair(float x, float& pos, float& neg) {
  const float m = fmaxf(-x, 0.f);
  const float ls = logf(expf(-m) + expf(-x - m));
  pos = m + ls;
  neg = x + m + ls;
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red) {  // 256 threads, fixed order
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// cost[b][q][t] = w_mask * CE(q, t) + w_class * class_cost[b][q][t] + w_dice * DICE(q, t), then
// clamped to [-1e10, 1e10] and NaN -> 0 (the reference's post-processing of the matrix).
// pred [B][Q][P], tgt rows of image b at tgt + toff[b] * P ([T_b][P]); class_cost / cost of image b
// at coff[b] ([Q][T_b]).  Grid (Q, B); T is processed in chunks of 8 targets.
constexpr int MC_TC = 8;
__global__ __launch_bounds__(256) void k_match_cost(const float* __restrict__ pred, int Q, int P,
                                                    const float* __restrict__ tgt, const int* __restrict__ toff,
                                                    const float* __restrict__ class_cost, const long long* __restrict__ coff,
                                                    float w_mask, float w_class, float w_dice, float* __restrict__ cost) {
  __shared__ float red[4];
  const int q = blockIdx.x, b = blockIdx.y;
  const int t0 = toff[b], T = toff[b + 1] - t0;
  if (T <= 0) return;
  const float* x = pred + ((long long)b * Q + q) * P;
  const float* y = tgt + (long long)t0 * P;
  float ssig = 0.f;
  for (int p = threadIdx.x; p < P; p += 256) ssig += sigmoidf_(x[p]);
  const float S = block_sum(ssig, red);
  for (int tc = 0; tc < T; tc += MC_TC) {
    float apos[MC_TC], aneg[MC_TC], asig[MC_TC], ay[MC_TC];
#pragma unroll
    for (int k = 0; k < MC_TC; ++k) apos[k] = aneg[k] = asig[k] = ay[k] = 0.f;
    for (int p = threadIdx.x; p < P; p += 256) {
      const float xv = x[p];
      float pos, neg;
      bce_pair(xv, pos, neg);
      const float sg = sigmoidf_(xv);
#pragma unroll
      for (int k = 0; k < MC_TC; ++k) {
        if (tc + k >= T) break;
        const float yv = y[(long long)(tc + k) * P + p];
        apos[k] += pos * yv;
        aneg[k] += neg * (1.f - yv);
        asig[k] += sg * yv;
        ay[k] += yv;
      }
    }
#pragma unroll
    for (int k = 0; k < MC_TC; ++k) {
      if (tc + k >= T) break;
      const float cp = block_sum(apos[k], red), cn = block_sum(aneg[k], red);
      const float cs = block_sum(asig[k], red), cy = block_sum(ay[k], red);
      if (threadIdx.x == 0) {
        const float ce = cp / (float)P + cn / (float)P;
        const float dice = 1.f - (2.f * cs + 1.f) / (S + cy + 1.f);
        const long long o = coff[b] + (long long)q * T + tc + k;
        float c = w_mask * ce + w_class * class_cost[o] + w_dice * dice;
        // torch.minimum / maximum propagate NaN, then nan_to_num(., 0) zeroes it
        cost[o] = isnan(c) ? 0.f : fmaxf(fminf(c, 1e10f), -1e10f);
      }
    }
  }
}

// Per matched pair n: ce[n] = mean_p BCE(x, y), dice[n] = 1 - (2 sum sig*y + 1) / (sum sig + sum y + 1);
// sums[n] = (sum sig*y, sum sig, sum y) kept for the backward.
__global__ __launch_bounds__(256) void k_point_losses(const float* __restrict__ x, const float* __restrict__ y, int P,
                                                      float* __restrict__ ce, float* __restrict__ dice,
                                                      float* __restrict__ sums) {
  __shared__ float red[4];
  const int n = blockIdx.x;
  const float* xr = x + (long long)n * P;
  const float* yr = y + (long long)n * P;
  float sbce = 0.f, ssy = 0.f, ss = 0.f, sy = 0.f;
  for (int p = threadIdx.x; p < P; p += 256) {
    const float xv = xr[p], yv = yr[p];
    float pos, neg;
    bce_pair(xv, pos, neg);
    sbce += yv * pos + (1.f - yv) * neg;  // (1 - y) x + m + ls for y in [0, 1]
    const float sg = sigmoidf_(xv);
    ssy += sg * yv;
    ss += sg;
    sy += yv;
  }
  sbce = block_sum(sbce, red);
  ssy = block_sum(ssy, red);
  ss = block_sum(ss, red);
  sy = block_sum(sy, red);
  if (threadIdx.x == 0) {
    ce[n] = sbce / (float)P;
    dice[n] = 1.f - (2.f * ssy + 1.f) / (ss + sy + 1.f);
    sums[3 * n] = ssy;
    sums[3 * n + 1] = ss;
    sums[3 * n + 2] = sy;
  }
}

// gx[n][p] = g_ce[n] * (sig - y) / P + g_dice[n] * d dice / dx with dice = 1 - (2A + 1) / D,
// A = sum sig*y, D = sum sig + sum y + 1: d dice / d sig_p = -(2 y_p D - (2A + 1)) / D^2.
__global__ __launch_bounds__(256) void k_point_losses_bwd(const float* __restrict__ x, const float* __restrict__ y, int N,
                                                          int P, const float* __restrict__ sums,
                                                          const float* __restrict__ g_ce,
                                                          const float* __restrict__ g_dice, float* __restrict__ gx) {
  const long long i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= (long long)N * P) return;
  const int n = (int)(i / P);
  const float xv = x[i], yv = y[i], sg = sigmoidf_(xv);
  const float A = sums[3 * n], D = sums[3 * n + 1] + sums[3 * n + 2] + 1.f;
  const float ddice = -(2.f * yv * D - (2.f * A + 1.f)) / (D * D) * (sg * (1.f - sg));
  gx[i] = g_ce[n] * (sg - yv) / (float)P + g_dice[n] * ddice;
}

}  // namespace

extern "C" {

int rgbd_point_sample(const float* maps, int nmaps, int h, int w, const float* coords, int maps_per_coord, int P,
                      float* out, void* stream) {
  // nothing to sample (empty tensors carry null data pointers): checked before the pointers
  RGBD_REQUIRE(nmaps >= 0 && h > 0 && w > 0 && P >= 0 && maps_per_coord > 0, RGBD_E_ARG);
  const long long n = (long long)nmaps * P;
  if (n == 0) return RGBD_OK;
  RGBD_REQUIRE(maps && coords && out, RGBD_E_ARG);
  k_point_sample<float><<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(maps, nmaps, h, w, coords,
                                                                                      maps_per_coord, P, out);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_point_sample_t(int dtype, const void* maps, int nmaps, int h, int w, const float* coords, int maps_per_coord,
                        int P, float* out, void* stream) {
  if (dtype == RGBD_F32)
    return rgbd_point_sample((const float*)maps, nmaps, h, w, coords, maps_per_coord, P, out, stream);
  RGBD_REQUIRE(dtype == RGBD_BF16, RGBD_E_DTYPE);
  RGBD_REQUIRE(nmaps >= 0 && h > 0 && w > 0 && P >= 0 && maps_per_coord > 0, RGBD_E_ARG);
  const long long n = (long long)nmaps * P;
  if (n == 0) return RGBD_OK;
  RGBD_REQUIRE(maps && coords && out, RGBD_E_ARG);
  k_point_sample<bf16_t><<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      (const bf16_t*)maps, nmaps, h, w, coords, maps_per_coord, P, out);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_point_sample_bwd(const float* gout, int nmaps, int h, int w, const float* coords, int maps_per_coord, int P,
                          float* gmaps, void* stream) {
  RGBD_REQUIRE(nmaps >= 0 && h > 0 && w > 0 && P >= 0 && maps_per_coord > 0, RGBD_E_ARG);
  const long long n = (long long)nmaps * P;
  if (n == 0) return RGBD_OK;
  RGBD_REQUIRE(gout && coords && gmaps, RGBD_E_ARG);
  k_point_sample_bwd<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(gout, nmaps, h, w, coords,
                                                                                   maps_per_coord, P, gmaps);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_match_cost(const float* pred, int B, int Q, int P, const float* tgt, const int* toff,
                    const float* class_cost, const long long* coff, float w_mask, float w_class, float w_dice,
                    float* cost, void* stream) {
  RGBD_REQUIRE(pred && tgt && toff && class_cost && coff && cost && B > 0 && Q > 0 && P > 0, RGBD_E_ARG);
  k_match_cost<<<dim3(Q, B), 256, 0, (hipStream_t)stream>>>(pred, Q, P, tgt, toff, class_cost, coff, w_mask, w_class,
                                                            w_dice, cost);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_point_losses(const float* logits, const float* labels, int N, int P, float* ce, float* dice, float* sums,
                      void* stream) {
  // N == 0 (a batch without target instances): empty tensors, null pointers, nothing to do
  RGBD_REQUIRE(N >= 0 && P > 0, RGBD_E_ARG);
  if (N == 0) return RGBD_OK;
  RGBD_REQUIRE(logits && labels && ce && dice && sums, RGBD_E_ARG);
  k_point_losses<<<N, 256, 0, (hipStream_t)stream>>>(logits, labels, P, ce, dice, sums);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_point_losses_bwd(const float* logits, const float* labels, int N, int P, const float* sums,
                          const float* g_ce, const float* g_dice, float* glogits, void* stream) {
  RGBD_REQUIRE(N >= 0 && P > 0, RGBD_E_ARG);
  const long long n = (long long)N * P;
  if (n == 0) return RGBD_OK;
  RGBD_REQUIRE(logits && labels && sums && g_ce && g_dice && glogits, RGBD_E_ARG);
  k_point_losses_bwd<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(logits, labels, N, P, sums, g_ce,
                                                                                   g_dice, glogits);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
