// f2: nn.GroupNorm(32, 256) of the Mask2Former pixel decoder (transformers 5.15
// modeling_mask2former.py Mask2FormerPixelDecoder: the three input projections, the FPN lateral
// adapter and the FPN output layer, whose ReLU is fused here), forward and backward, NCHW.
//
// A group's channels are contiguous in NCHW, and everything the normalisation needs reduces per
// channel first: the forward's per-channel (mean, M2) (Welford per thread, Chan's combination in a
// fixed order), combined per group in the apply pass; the backward's per-channel
// (sum dy', sum dy' x^) with dy' = dy (* [y > 0] with the fused ReLU), from which both the group
// terms of dx (gamma_c times those sums) and the parameter gradients follow.  Two launches each
// way, HBM-bound (x read twice forward, x and dy read twice backward), deterministic.
#include "common.hpp"

#include <algorithm>

namespace rgbd {
namespace {

constexpr int GN_THREADS = 256;

template <typename T>
__device__ __forceinline__ float gn_ld(const T* p, long long i) {
  return Num<T>::to_f(p[i]);
}

// Chan's combination of (n, mean, M2) partials
__device__ __forceinline__ void chan_combine(float& n, float& mean, float& m2, float nb, float meanb, float m2b) {
  if (nb == 0.f) return;
  const float nt = n + nb, d = meanb - mean;
  mean += d * (nb / nt);
  m2 += m2b + d * d * (n * nb / nt);
  n = nt;
}

// block (b * C + c): the channel's HW values -> (mean, M2) in stat[b * C + c][2]
template <typename T>
__global__ __launch_bounds__(GN_THREADS) void k_gn_chan_stats(const T* __restrict__ x, int HW, float* __restrict__ stat) {
  __shared__ float sn[GN_THREADS], sm[GN_THREADS], s2[GN_THREADS];
  const T* xc = x + (long long)blockIdx.x * HW;
  float n = 0.f, mean = 0.f, m2 = 0.f;
  for (int i = threadIdx.x; i < HW; i += GN_THREADS) {  // Welford
    const float v = gn_ld(xc, i);
    n += 1.f;
    const float d = v - mean;
    mean += d / n;
    m2 += d * (v - mean);
  }
  sn[threadIdx.x] = n;
  sm[threadIdx.x] = mean;
  s2[threadIdx.x] = m2;
  __syncthreads();
  for (int o = GN_THREADS / 2; o > 0; o >>= 1) {  // fixed-shape tree
    if (threadIdx.x < o) {
      float a = sn[threadIdx.x], b = sm[threadIdx.x], c = s2[threadIdx.x];
      chan_combine(a, b, c, sn[threadIdx.x + o], sm[threadIdx.x + o], s2[threadIdx.x + o]);
      sn[threadIdx.x] = a;
      sm[threadIdx.x] = b;
      s2[threadIdx.x] = c;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    stat[2 * blockIdx.x] = sm[0];
    stat[2 * blockIdx.x + 1] = s2[0];
  }
}

// the group's (mean, rstd) from its channels' (mean, M2), channels in order
__device__ __forceinline__ void gn_group(const float* __restrict__ stat, int b, int g, int C, int cpg, int HW, float eps,
                                         float& mean, float& rstd) {
  float n = 0.f, m2 = 0.f;
  mean = 0.f;
  for (int k = 0; k < cpg; ++k) {
    const int c = g * cpg + k;
    chan_combine(n, mean, m2, (float)HW, stat[2 * (b * C + c)], stat[2 * (b * C + c) + 1]);
  }
  rstd = 1.f / sqrtf(m2 / n + eps);  // biased variance, as torch.nn.GroupNorm
}

// grid (B * C, chunks): y = (x - mean) * rstd * gamma + beta (, ReLU); block (b, c, 0) of channel
// g * cpg also stores the group's (mean, rstd)
template <typename TX, typename TY>
__global__ __launch_bounds__(GN_THREADS) void k_gn_apply(const TX* __restrict__ x, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, const float* __restrict__ stat,
                                                         int C, int G, int HW, int chunk, float eps, int relu,
                                                         TY* __restrict__ y, float* __restrict__ mr) {
  const int bc = blockIdx.x, b = bc / C, c = bc % C, cpg = C / G, g = c / cpg;
  float mean, rstd;
  gn_group(stat, b, g, C, cpg, HW, eps, mean, rstd);
  const float sc = rstd * (gamma ? gamma[c] : 1.f), sh = (beta ? beta[c] : 0.f) - mean * sc;
  const long long base = (long long)bc * HW;
  const int i0 = blockIdx.y * chunk, i1 = min(HW, i0 + chunk);
  for (int i = i0 + threadIdx.x; i < i1; i += GN_THREADS) {
    float v = __builtin_fmaf(gn_ld(x, base + i), sc, sh);
    if (relu) v = fmaxf(v, 0.f);
    y[base + i] = Num<TY>::from_f(v);
  }
  if (blockIdx.y == 0 && c % cpg == 0 && threadIdx.x == 0) {
    mr[2 * (b * G + g)] = mean;
    mr[2 * (b * G + g) + 1] = rstd;
  }
}

// backward pass 1, block (b * C + c): (sum dy', sum dy' x^) of the channel, dy' = dy (* [y > 0])
template <typename TX, typename TD>
__global__ __launch_bounds__(GN_THREADS) void k_gn_bwd_chan(const TX* __restrict__ x, const TD* __restrict__ dy,
                                                            const float* __restrict__ gamma, const float* __restrict__ beta,
                                                            const float* __restrict__ mr, int C, int G, int HW, int relu,
                                                            float* __restrict__ part) {
  __shared__ float sa[GN_THREADS], sb[GN_THREADS];
  const int bc = blockIdx.x, b = bc / C, c = bc % C, g = c / (C / G);
  const float mean = mr[2 * (b * G + g)], rstd = mr[2 * (b * G + g) + 1];
  const float ga = gamma ? gamma[c] : 1.f, be = beta ? beta[c] : 0.f;
  const float sc = rstd * ga, sh = be - mean * sc;  // the forward's affine: the same ReLU mask
  const long long base = (long long)bc * HW;
  float a = 0.f, q = 0.f;
  for (int i = threadIdx.x; i < HW; i += GN_THREADS) {
    const float xv = gn_ld(x, base + i);
    const float xh = (xv - mean) * rstd;
    float d = gn_ld(dy, base + i);
    if (relu && __builtin_fmaf(xv, sc, sh) <= 0.f) d = 0.f;
    a += d;
    q += d * xh;
  }
  sa[threadIdx.x] = a;
  sb[threadIdx.x] = q;
  __syncthreads();
  for (int o = GN_THREADS / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      sa[threadIdx.x] += sa[threadIdx.x + o];
      sb[threadIdx.x] += sb[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * bc] = sa[0];
    part[2 * bc + 1] = sb[0];
  }
}

// backward pass 2, grid (B * C, chunks): dx = rstd (gamma dy' - mean_g(gamma dy') - x^ mean_g(gamma dy' x^));
// blocks (0, c, 0) also form dgamma[c] = sum_b part[b][c][1], dbeta[c] = sum_b part[b][c][0]
template <typename TX, typename TD>
__global__ __launch_bounds__(GN_THREADS) void k_gn_bwd_apply(const TX* __restrict__ x, const TD* __restrict__ dy,
                                                             const float* __restrict__ gamma, const float* __restrict__ beta,
                                                             const float* __restrict__ mr, const float* __restrict__ part,
                                                             int B, int C, int G, int HW, int chunk, int relu,
                                                             TX* __restrict__ dx, float* __restrict__ dgamma,
                                                             float* __restrict__ dbeta) {
  const int bc = blockIdx.x, b = bc / C, c = bc % C, cpg = C / G, g = c / cpg;
  const float mean = mr[2 * (b * G + g)], rstd = mr[2 * (b * G + g) + 1];
  float s1 = 0.f, s2 = 0.f;
  for (int k = 0; k < cpg; ++k) {
    const int cc = g * cpg + k;
    const float gk = gamma ? gamma[cc] : 1.f;
    s1 += gk * part[2 * (b * C + cc)];
    s2 += gk * part[2 * (b * C + cc) + 1];
  }
  const float inv_n = 1.f / ((float)cpg * (float)HW);
  const float m1 = s1 * inv_n, m2 = s2 * inv_n;
  const float ga = gamma ? gamma[c] : 1.f, be = beta ? beta[c] : 0.f;
  const float sc = rstd * ga, sh = be - mean * sc;
  const long long base = (long long)bc * HW;
  const int i0 = blockIdx.y * chunk, i1 = min(HW, i0 + chunk);
  for (int i = i0 + threadIdx.x; i < i1; i += GN_THREADS) {
    const float xv = gn_ld(x, base + i);
    const float xh = (xv - mean) * rstd;
    float d = gn_ld(dy, base + i);
    if (relu && __builtin_fmaf(xv, sc, sh) <= 0.f) d = 0.f;
    dx[base + i] = Num<TX>::from_f(rstd * (ga * d - m1 - xh * m2));
  }
  if (b == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    float dg = 0.f, db = 0.f;
    for (int bb = 0; bb < B; ++bb) {
      db += part[2 * (bb * C + c)];
      dg += part[2 * (bb * C + c) + 1];
    }
    if (dgamma) dgamma[c] = dg;
    if (dbeta) dbeta[c] = db;
  }
}

inline int gn_chunk(int HW) { return std::max(GN_THREADS * 8, (HW + 7) / 8); }

template <typename TX, typename TY>
void gn_fwd_t(const void* x, const float* gamma, const float* beta, int B, int C, int G, int HW, float eps, int relu,
              void* y, float* mr, float* stat, hipStream_t s) {
  hipLaunchKernelGGL(k_gn_chan_stats<TX>, dim3(B * C), dim3(GN_THREADS), 0, s, (const TX*)x, HW, stat);
  const int chunk = gn_chunk(HW);
  hipLaunchKernelGGL((k_gn_apply<TX, TY>), dim3(B * C, ceil_div(HW, chunk)), dim3(GN_THREADS), 0, s, (const TX*)x, gamma,
                     beta, stat, C, G, HW, chunk, eps, relu, (TY*)y, mr);
}

template <typename TX, typename TD>
void gn_bwd_t(const void* x, const void* dy, const float* gamma, const float* beta, const float* mr, int B, int C,
              int G, int HW, int relu, void* dx, float* dgamma, float* dbeta, float* part, hipStream_t s) {
  hipLaunchKernelGGL((k_gn_bwd_chan<TX, TD>), dim3(B * C), dim3(GN_THREADS), 0, s, (const TX*)x, (const TD*)dy, gamma,
                     beta, mr, C, G, HW, relu, part);
  const int chunk = gn_chunk(HW);
  hipLaunchKernelGGL((k_gn_bwd_apply<TX, TD>), dim3(B * C, ceil_div(HW, chunk)), dim3(GN_THREADS), 0, s, (const TX*)x,
                     (const TD*)dy, gamma, beta, mr, part, B, C, G, HW, chunk, relu, (TX*)dx, dgamma, dbeta);
}

}  // namespace
}  // namespace rgbd

using namespace rgbd;

extern "C" {

size_t rgbd_groupnorm_workspace_size(int B, int C) { return (size_t)std::max(1, B * C) * 2 * sizeof(float); }

int rgbd_groupnorm_fwd(int x_dtype, const void* x, const float* gamma, const float* beta, int B, int C, int G, int HW,
                       float eps, int relu, int y_dtype, void* y, float* mean_rstd, void* ws, void* stream) {
  RGBD_REQUIRE(x && y && mean_rstd && ws && B > 0 && C > 0 && G > 0 && HW > 0, RGBD_E_ARG);
  RGBD_REQUIRE(C % G == 0, RGBD_E_SHAPE);
  RGBD_REQUIRE((x_dtype == RGBD_F32 || x_dtype == RGBD_BF16) && (y_dtype == RGBD_F32 || y_dtype == RGBD_BF16),
               RGBD_E_DTYPE);
  hipStream_t s = (hipStream_t)stream;
  float* stat = (float*)ws;
  if (x_dtype == RGBD_BF16) {
    if (y_dtype == RGBD_BF16) gn_fwd_t<bf16_t, bf16_t>(x, gamma, beta, B, C, G, HW, eps, relu, y, mean_rstd, stat, s);
    else gn_fwd_t<bf16_t, float>(x, gamma, beta, B, C, G, HW, eps, relu, y, mean_rstd, stat, s);
  } else {
    if (y_dtype == RGBD_BF16) gn_fwd_t<float, bf16_t>(x, gamma, beta, B, C, G, HW, eps, relu, y, mean_rstd, stat, s);
    else gn_fwd_t<float, float>(x, gamma, beta, B, C, G, HW, eps, relu, y, mean_rstd, stat, s);
  }
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_groupnorm_bwd(int x_dtype, const void* x, int dy_dtype, const void* dy, const float* gamma, const float* beta,
                       const float* mean_rstd, int B, int C, int G, int HW, int relu, void* dx, float* dgamma,
                       float* dbeta, void* ws, void* stream) {
  RGBD_REQUIRE(x && dy && mean_rstd && dx && ws && B > 0 && C > 0 && G > 0 && HW > 0, RGBD_E_ARG);
  RGBD_REQUIRE(C % G == 0, RGBD_E_SHAPE);
  RGBD_REQUIRE(!relu || gamma, RGBD_E_ARG);
  RGBD_REQUIRE((x_dtype == RGBD_F32 || x_dtype == RGBD_BF16) && (dy_dtype == RGBD_F32 || dy_dtype == RGBD_BF16),
               RGBD_E_DTYPE);
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)ws;
  if (x_dtype == RGBD_BF16) {
    if (dy_dtype == RGBD_BF16)
      gn_bwd_t<bf16_t, bf16_t>(x, dy, gamma, beta, mean_rstd, B, C, G, HW, relu, dx, dgamma, dbeta, part, s);
    else
      gn_bwd_t<bf16_t, float>(x, dy, gamma, beta, mean_rstd, B, C, G, HW, relu, dx, dgamma, dbeta, part, s);
  } else {
    if (dy_dtype == RGBD_BF16)
      gn_bwd_t<float, bf16_t>(x, dy, gamma, beta, mean_rstd, B, C, G, HW, relu, dx, dgamma, dbeta, part, s);
    else
      gn_bwd_t<float, float>(x, dy, gamma, beta, mean_rstd, B, C, G, HW, relu, dx, dgamma, dbeta, part, s);
  }
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
