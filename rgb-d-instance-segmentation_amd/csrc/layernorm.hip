// f1 / f2: nn.LayerNorm of the Mask2Former decoder layers (transformers 5.15
// modeling_mask2former.py:1700-1719, 9 layers x 3 norms + the decoder's final norm :1894),
// the pixel decoder's encoder layers (:1022-1040, 6 layers x 2) and Swin-T (modeling_swin.py
// layernorm_before / layernorm_after :542, :570, patch merging :330, stage outputs), forward
// and backward.  HBM-bound: one wave per row, the row register-resident (C <= 1536: lane l
// holds columns l + 64 i), statistics in float32 by two passes over the registers (mean, then
// the mean squared deviation — no cancellation), 1 / sqrt(var + eps).
#include "common.hpp"

#include <algorithm>

namespace rgbd {
namespace {

constexpr int LN_MAXI = 24;   // C <= 64 * 24 (Swin patch merging: 4 x 384)
constexpr int LN_RB = 64;     // minimum rows per backward block (its dgamma / dbeta partial)
constexpr int LN_MAXBLK = 256;  // at most this many partials: the final reduction stays short

inline int ln_rows_per_block(int rows) { return std::max(LN_RB, (rows + LN_MAXBLK - 1) / LN_MAXBLK); }

template <typename T>
__device__ __forceinline__ float ld_f(const void* p, long long i) {
  return Num<T>::to_f(reinterpret_cast<const T*>(p)[i]);
}
template <typename T>
__device__ __forceinline__ void st_f(void* p, long long i, float v) {
  reinterpret_cast<T*>(p)[i] = Num<T>::from_f(v);
}

template <typename TX, typename TY>
__global__ __launch_bounds__(256) void k_ln_fwd(const void* __restrict__ x, const float* __restrict__ gamma,
                                                const float* __restrict__ beta, int rows, int C, float eps,
                                                void* __restrict__ y, float* __restrict__ mean, float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const long long base = (long long)row * C;
  float v[LN_MAXI];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXI; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < C ? ld_f<TX>(x, base + c) : 0.f;
    s += v[i];
  }
  const float mu = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXI; ++i) {
    const int c = lane + 64 * i;
    const float d = c < C ? v[i] - mu : 0.f;
    q += d * d;
  }
  const float var = wave_sum(q) / (float)C;
  const float rs = 1.f / sqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < LN_MAXI; ++i) {
    const int c = lane + 64 * i;
    if (c < C) st_f<TY>(y, base + c, (v[i] - mu) * rs * (gamma ? gamma[c] : 1.f) + (beta ? beta[c] : 0.f));
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// dx per row; dgamma / dbeta partials per block of LN_RB rows: part[blk][2][C]
template <typename TX, typename TD>
__global__ __launch_bounds__(256) void k_ln_bwd(const void* __restrict__ x, const void* __restrict__ dy,
                                                const float* __restrict__ gamma, const float* __restrict__ mean,
                                                const float* __restrict__ rstd, int rows, int C, int rb,
                                                void* __restrict__ dx, float* __restrict__ part) {
  __shared__ float red[4][2][64 * LN_MAXI];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float pg[LN_MAXI], pb[LN_MAXI];
#pragma unroll
  for (int i = 0; i < LN_MAXI; ++i) pg[i] = pb[i] = 0.f;
  const int r0 = blockIdx.x * rb;
  for (int row = r0 + wave; row < min(rows, r0 + rb); row += 4) {
    const long long base = (long long)row * C;
    const float mu = mean[row], rs = rstd[row];
    float xh[LN_MAXI], g[LN_MAXI];
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAXI; ++i) {
      const int c = lane + 64 * i;
      xh[i] = g[i] = 0.f;
      if (c < C) {
        const float d = ld_f<TD>(dy, base + c);
        xh[i] = (ld_f<TX>(x, base + c) - mu) * rs;
        g[i] = d * (gamma ? gamma[c] : 1.f);
        pg[i] += d * xh[i];
        pb[i] += d;
      }
      sa += g[i];
      sb += g[i] * xh[i];
    }
    const float ma = wave_sum(sa) / (float)C, mb = wave_sum(sb) / (float)C;
#pragma unroll
    for (int i = 0; i < LN_MAXI; ++i) {
      const int c = lane + 64 * i;
      if (c < C) st_f<TX>(dx, base + c, rs * (g[i] - ma - xh[i] * mb));
    }
  }
#pragma unroll
  for (int i = 0; i < LN_MAXI; ++i) {
    red[wave][0][lane + 64 * i] = pg[i];
    red[wave][1][lane + 64 * i] = pb[i];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * C; i += 256) {
    const int w = i / C, c = i % C;
    part[((long long)blockIdx.x * 2 + w) * C + c] = ((red[0][w][c] + red[1][w][c]) + red[2][w][c]) + red[3][w][c];
  }
}

__global__ __launch_bounds__(256) void k_ln_param_reduce(const float* __restrict__ part, int nblk, int C,
                                                         float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= 2 * C) return;
  const int w = i / C, c = i % C;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += part[((long long)b * 2 + w) * C + c];
  (w ? dbeta : dgamma)[c] = s;
}

template <typename TX>
void ln_fwd_t(int y_dtype, const void* x, const float* gamma, const float* beta, int rows, int C, float eps, void* y,
              float* mean, float* rstd, hipStream_t s) {
  dim3 grid(ceil_div(rows, 4));
  if (y_dtype == RGBD_BF16)
    hipLaunchKernelGGL((k_ln_fwd<TX, bf16_t>), grid, dim3(256), 0, s, x, gamma, beta, rows, C, eps, y, mean, rstd);
  else
    hipLaunchKernelGGL((k_ln_fwd<TX, float>), grid, dim3(256), 0, s, x, gamma, beta, rows, C, eps, y, mean, rstd);
}

template <typename TX>
void ln_bwd_t(int dy_dtype, const void* x, const void* dy, const float* gamma, const float* mean, const float* rstd,
              int rows, int C, void* dx, float* part, hipStream_t s) {
  const int rb = ln_rows_per_block(rows);
  dim3 grid(ceil_div(rows, rb));
  if (dy_dtype == RGBD_BF16)
    hipLaunchKernelGGL((k_ln_bwd<TX, bf16_t>), grid, dim3(256), 0, s, x, dy, gamma, mean, rstd, rows, C, rb, dx, part);
  else
    hipLaunchKernelGGL((k_ln_bwd<TX, float>), grid, dim3(256), 0, s, x, dy, gamma, mean, rstd, rows, C, rb, dx, part);
}

}  // namespace
}  // namespace rgbd

using namespace rgbd;

extern "C" {

int rgbd_layernorm_fwd(int x_dtype, const void* x, const float* gamma, const float* beta, int rows, int C,
                       float eps, int y_dtype, void* y, float* mean, float* rstd, void* stream) {
  RGBD_REQUIRE(x && y && mean && rstd && rows > 0 && C > 0, RGBD_E_ARG);
  RGBD_REQUIRE(C <= 64 * LN_MAXI, RGBD_E_SHAPE);
  RGBD_REQUIRE((x_dtype == RGBD_F32 || x_dtype == RGBD_BF16) && (y_dtype == RGBD_F32 || y_dtype == RGBD_BF16),
               RGBD_E_DTYPE);
  hipStream_t s = (hipStream_t)stream;
  if (x_dtype == RGBD_BF16)
    ln_fwd_t<bf16_t>(y_dtype, x, gamma, beta, rows, C, eps, y, mean, rstd, s);
  else
    ln_fwd_t<float>(y_dtype, x, gamma, beta, rows, C, eps, y, mean, rstd, s);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

size_t rgbd_layernorm_bwd_workspace_size(int rows, int C) {
  return (size_t)ceil_div(rows, ln_rows_per_block(rows)) * 2 * C * sizeof(float);
}

int rgbd_layernorm_bwd(int x_dtype, const void* x, int dy_dtype, const void* dy, const float* gamma,
                       const float* mean, const float* rstd, int rows, int C, void* dx, float* dgamma,
                       float* dbeta, void* ws, void* stream) {
  RGBD_REQUIRE(x && dy && mean && rstd && dx && dgamma && dbeta && ws && rows > 0 && C > 0, RGBD_E_ARG);
  RGBD_REQUIRE(C <= 64 * LN_MAXI, RGBD_E_SHAPE);
  RGBD_REQUIRE((x_dtype == RGBD_F32 || x_dtype == RGBD_BF16) && (dy_dtype == RGBD_F32 || dy_dtype == RGBD_BF16),
               RGBD_E_DTYPE);
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)ws;
  if (x_dtype == RGBD_BF16)
    ln_bwd_t<bf16_t>(dy_dtype, x, dy, gamma, mean, rstd, rows, C, dx, part, s);
  else
    ln_bwd_t<float>(dy_dtype, x, dy, gamma, mean, rstd, rows, C, dx, part, s);
  RGBD_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_ln_param_reduce, dim3(ceil_div(2 * C, 256)), dim3(256), 0, s, part,
                     ceil_div(rows, ln_rows_per_block(rows)), C, dgamma, dbeta);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
