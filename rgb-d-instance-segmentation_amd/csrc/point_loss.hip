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
// per group of `per` consecutive maps, or per map the set set_of_map[m] when that is given
template <typename T>
__global__ __launch_bounds__(256) void k_point_sample(const T* __restrict__ maps, int nmaps, int h, int w,
                                                      const float* __restrict__ coords, int per,
                                                      const int* __restrict__ set_of_map, int P,
                                                      float* __restrict__ out) {
  const long long i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= (long long)nmaps * P) return;
  const int m = (int)(i / P), p = (int)(i % P);
  const int set = set_of_map ? set_of_map[m] : m / per;
  const float2 c = reinterpret_cast<const float2*>(coords)[(long long)set * P + p];
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
// at coff[b] ([Q][T_b]).  Grid (Q, B); T is processed in chunks of 8 targets.  With probs set, the
// class cost is read as -probs[b][q][labels[toff[b] + t]] (probs [B][Q][C], the matcher's softmax)
// instead of from class_cost.
constexpr int MC_TC = 8;
__global__ __launch_bounds__(256) void k_match_cost(const float* __restrict__ pred, int Q, int P,
                                                    const float* __restrict__ tgt, const int* __restrict__ toff,
                                                    const float* __restrict__ class_cost, const long long* __restrict__ coff,
                                                    const float* __restrict__ probs, int C,
                                                    const long long* __restrict__ labels, float w_mask,
                                                    float w_class, float w_dice, float* __restrict__ cost) {
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
        const float cc = probs ? -probs[((long long)b * Q + q) * C + labels[t0 + tc + k]] : class_cost[o];
        float c = w_mask * ce + w_class * cc + w_dice * dice;
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

// The k largest of every row (loss_masks' uncertainty selection, torch.topk(unc, k, dim=1,
// sorted=False) :711): one workgroup per row, the row's order-preserving keys resident in LDS
// (torch's TopKTypeConfig<float>: x ^ (sign ? ~0 : 0x80000000), NaN the largest), a 4-pass
// 8-bit radix select of the k-th key T (per-wave histograms), then every key > T and the
// lowest-index keys == T up to k, written in index order.
constexpr int TK_THR = 512;
constexpr int TK_HIST = (TK_THR / 64) * 256;
constexpr int TK_MAXN = (163840 - (TK_HIST + 2 * TK_THR + 8) * 4) / 4;
__device__ __forceinline__ uint32_t tk_key(float v) {
  const uint32_t x = __float_as_uint(v);
  return v == v ? (x ^ ((x & 0x80000000u) ? 0xffffffffu : 0x80000000u)) : 0xffffffffu;
}
// exclusive prefix sum of v over the workgroup's 512 threads (Hillis-Steele in LDS); total in *tot
__device__ __forceinline__ uint32_t tk_scan(uint32_t v, uint32_t* buf, uint32_t* tot) {
  const int t = threadIdx.x;
  buf[t] = v;
  __syncthreads();
  for (int o = 1; o < TK_THR; o <<= 1) {
    const uint32_t a = t >= o ? buf[t - o] : 0u;
    __syncthreads();
    buf[t] += a;
    __syncthreads();
  }
  const uint32_t incl = buf[t];
  if (tot) *tot = buf[TK_THR - 1];
  __syncthreads();
  return incl - v;
}
__global__ __launch_bounds__(TK_THR) void k_topk_rows(const float* __restrict__ x, int n, int k,
                                                      long long* __restrict__ out) {
  extern __shared__ uint32_t tk_sm[];
  uint32_t* keys = tk_sm;
  uint32_t* hist = tk_sm + n;               // [8 waves][256]
  uint32_t* buf = hist + TK_HIST;           // scan buffer [512]
  uint32_t* misc = buf + TK_THR;            // [0] digit, [1] remaining
  const int t = threadIdx.x, wave = t >> 6;
  const float* xr = x + (long long)blockIdx.x * n;
  for (int i = t; i < n; i += TK_THR) keys[i] = tk_key(xr[i]);
  uint32_t prefix = 0u, pmask = 0u;
  int kr = k;  // keys still to take among those matching the prefix
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int i = t; i < TK_HIST; i += TK_THR) hist[i] = 0u;
    __syncthreads();
    for (int i = t; i < n; i += TK_THR) {
      const uint32_t kv = keys[i];
      if ((kv & pmask) == prefix) atomicAdd(&hist[wave * 256 + ((kv >> shift) & 255u)], 1u);
    }
    __syncthreads();
    // suffix counts over the digits, high digit first: thread t < 256 owns digit 255 - t
    uint32_t c = 0u;
    if (t < 256) {
#pragma unroll
      for (int w = 0; w < TK_THR / 64; ++w) c += hist[w * 256 + (255 - t)];
    }
    const uint32_t before = tk_scan(c, buf, nullptr);  // keys with a larger digit
    if (t < 256 && before < (uint32_t)kr && before + c >= (uint32_t)kr) {
      misc[0] = 255u - t;
      misc[1] = (uint32_t)kr - before;
    }
    __syncthreads();
    prefix |= misc[0] << shift;
    pmask |= 255u << shift;
    kr = (int)misc[1];
    __syncthreads();
  }
  // every key > prefix, then the first kr keys == prefix in index order
  const int chunk = (n + TK_THR - 1) / TK_THR, c0 = min(n, t * chunk), c1 = min(n, c0 + chunk);
  uint32_t gt = 0u, eq = 0u;
  for (int i = c0; i < c1; ++i) {
    const uint32_t kv = keys[i];
    gt += kv > prefix;
    eq += kv == prefix;
  }
  const uint32_t eq_before = tk_scan(eq, buf, nullptr);
  const uint32_t take_eq = (uint32_t)kr > eq_before ? min(eq, (uint32_t)kr - eq_before) : 0u;
  uint32_t pos = tk_scan(gt + take_eq, buf, nullptr);
  long long* o = out + (long long)blockIdx.x * k;
  uint32_t eq_seen = 0u;
  for (int i = c0; i < c1; ++i) {
    const uint32_t kv = keys[i];
    if (kv > prefix || (kv == prefix && eq_seen++ < take_eq)) o[pos++] = i;
  }
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
                                                                                      maps_per_coord, nullptr, P, out);
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
      (const bf16_t*)maps, nmaps, h, w, coords, maps_per_coord, nullptr, P, out);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_point_sample_sets(int dtype, const void* maps, int nmaps, int h, int w, const float* coords,
                           const int* set_of_map, int P, float* out, void* stream) {
  RGBD_REQUIRE(dtype == RGBD_F32 || dtype == RGBD_BF16, RGBD_E_DTYPE);
  RGBD_REQUIRE(nmaps >= 0 && h > 0 && w > 0 && P >= 0, RGBD_E_ARG);
  const long long n = (long long)nmaps * P;
  if (n == 0) return RGBD_OK;
  RGBD_REQUIRE(maps && coords && set_of_map && out, RGBD_E_ARG);
  const unsigned grid = (unsigned)((n + 255) / 256);
  if (dtype == RGBD_F32)
    k_point_sample<float><<<grid, 256, 0, (hipStream_t)stream>>>((const float*)maps, nmaps, h, w, coords, 1,
                                                                 set_of_map, P, out);
  else
    k_point_sample<bf16_t><<<grid, 256, 0, (hipStream_t)stream>>>((const bf16_t*)maps, nmaps, h, w, coords, 1,
                                                                  set_of_map, P, out);
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
  k_match_cost<<<dim3(Q, B), 256, 0, (hipStream_t)stream>>>(pred, Q, P, tgt, toff, class_cost, coff, nullptr, 0,
                                                            nullptr, w_mask, w_class, w_dice, cost);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

size_t rgbd_topk_rows_max_n() { return (size_t)TK_MAXN; }

int rgbd_topk_rows(const float* x, int rows, int n, int k, long long* idx, void* stream) {
  RGBD_REQUIRE(rows >= 0 && n > 0 && k > 0 && k <= n, RGBD_E_ARG);
  RGBD_REQUIRE(n <= TK_MAXN, RGBD_E_SHAPE);
  if (rows == 0) return RGBD_OK;
  RGBD_REQUIRE(x && idx, RGBD_E_ARG);
  const size_t smem = ((size_t)n + TK_HIST + TK_THR + 8) * 4;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)k_topk_rows, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  if (attr != hipSuccess) return (int)attr;
  k_topk_rows<<<rows, TK_THR, smem, (hipStream_t)stream>>>(x, n, k, idx);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_match_cost_probs(const float* pred, int B, int Q, int P, const float* tgt, const int* toff,
                          const float* probs, int C, const long long* labels, const long long* coff, float w_mask,
                          float w_class, float w_dice, float* cost, void* stream) {
  RGBD_REQUIRE(pred && tgt && toff && probs && labels && coff && cost && B > 0 && Q > 0 && P > 0 && C > 0,
               RGBD_E_ARG);
  k_match_cost<<<dim3(Q, B), 256, 0, (hipStream_t)stream>>>(pred, Q, P, tgt, toff, nullptr, coff, probs, C, labels,
                                                            w_mask, w_class, w_dice, cost);
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
