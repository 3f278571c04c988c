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

// ---- vectorised rows (C % 4 == 0, the shapes of the model: 96 .. 1536): a row belongs to a group
// of T lanes (T = the power of two >= C / 4, at most 64; 64 / T rows per wave), lane j of the group
// holds the 4-column chunks j + T k (k < NCH), loaded as one 16-byte (f32) or 8-byte (bf16) access;
// the row statistics are group shuffle sums.  Many rows per wave-instruction keep enough loads in
// flight for small C (the one-wave-per-row kernels above ran at ~1 TB/s on Swin's C = 96 rows).
template <typename T>
__device__ __forceinline__ void ld4(const void* p, long long i, float (&v)[4]);
template <>
__device__ __forceinline__ void ld4<float>(const void* p, long long i, float (&v)[4]) {
  const float4 q = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + i);
  v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
}
template <>
__device__ __forceinline__ void ld4<bf16_t>(const void* p, long long i, float (&v)[4]) {
  const uint2 q = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(p) + i);
  v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
  v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
}
template <typename T>
__device__ __forceinline__ void st4(void* p, long long i, const float (&v)[4]);
template <>
__device__ __forceinline__ void st4<float>(void* p, long long i, const float (&v)[4]) {
  *reinterpret_cast<float4*>(reinterpret_cast<float*>(p) + i) = make_float4(v[0], v[1], v[2], v[3]);
}
template <>
__device__ __forceinline__ void st4<bf16_t>(void* p, long long i, const float (&v)[4]) {
  *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p) + i) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
}
template <int T>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = T / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <typename TX, typename TY, int T, int NCH>
__global__ __launch_bounds__(256) void k_ln_fwd_v(const void* __restrict__ x, const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, int rows, int C, float eps,
                                                  void* __restrict__ y, float* __restrict__ mean,
                                                  float* __restrict__ rstd) {
  const int j = threadIdx.x % T;
  const int row = blockIdx.x * (256 / T) + threadIdx.x / T;
  const bool live = row < rows;  // every lane of a group takes part in the shuffles
  const long long base = (long long)(live ? row : 0) * C;
  float v[NCH][4];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * (j + T * k);
    if (c < C) {
      ld4<TX>(x, base + c, v[k]);
    } else {
      v[k][0] = v[k][1] = v[k][2] = v[k][3] = 0.f;
    }
    s += (v[k][0] + v[k][1]) + (v[k][2] + v[k][3]);
  }
  const float mu = group_sum<T>(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k)
    if (4 * (j + T * k) < C)
#pragma unroll
      for (int e = 0; e < 4; ++e) q += (v[k][e] - mu) * (v[k][e] - mu);
  const float var = group_sum<T>(q) / (float)C;
  const float rs = 1.f / sqrtf(var + eps);
  if (!live) return;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * (j + T * k);
    if (c < C) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[e] = (v[k][e] - mu) * rs * (gamma ? gamma[c + e] : 1.f) + (beta ? beta[c + e] : 0.f);
      st4<TY>(y, base + c, o);
    }
  }
  if (j == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// The post-norm residual of the decoder / pixel-decoder encoder layers in one pass:
//   s = x + r (float32 arithmetic, rounded to s's dtype, as torch's add of the two), y = LN(s);
// s is written for the backward (rgbd_layernorm_bwd on s).  Same row grouping as k_ln_fwd_v.
template <typename TX, typename TR, typename TS, typename TY, int T, int NCH>
__global__ __launch_bounds__(256) void k_add_ln_fwd_v(const void* __restrict__ x, const void* __restrict__ r,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      int rows, int C, float eps, float clampc,
                                                      void* __restrict__ s_out, void* __restrict__ y,
                                                      bf16_t* __restrict__ y2, float* __restrict__ mean,
                                                      float* __restrict__ rstd) {
  const int j = threadIdx.x % T;
  const int row = blockIdx.x * (256 / T) + threadIdx.x / T;
  const bool live = row < rows;
  const long long base = (long long)(live ? row : 0) * C;
  float v[NCH][4];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * (j + T * k);
    if (c < C) {
      float a[4], b[4];
      ld4<TX>(x, base + c, a);
      ld4<TR>(r, base + c, b);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[k][e] = a[e] + b[e];
      if constexpr (sizeof(TS) == 2) {  // the bf16 sum is what the norm sees
#pragma unroll
        for (int e = 0; e < 4; ++e) v[k][e] = bf16_to_f32(f32_to_bf16(v[k][e]));
      }
    } else {
      v[k][0] = v[k][1] = v[k][2] = v[k][3] = 0.f;
    }
    s += (v[k][0] + v[k][1]) + (v[k][2] + v[k][3]);
  }
  const float mu = group_sum<T>(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k)
    if (4 * (j + T * k) < C)
#pragma unroll
      for (int e = 0; e < 4; ++e) q += (v[k][e] - mu) * (v[k][e] - mu);
  const float var = group_sum<T>(q) / (float)C;
  const float rs = 1.f / sqrtf(var + eps);
  if (!live) return;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * (j + T * k);
    if (c < C) {
      st4<TS>(s_out, base + c, v[k]);
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[e] = (v[k][e] - mu) * rs * (gamma ? gamma[c + e] : 1.f) + (beta ? beta[c + e] : 0.f);
      if (clampc > 0.f) {  // torch.clamp(y, -c, c): NaN stays NaN
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = o[e] < -clampc ? -clampc : (o[e] > clampc ? clampc : o[e]);
      }
      st4<TY>(y, base + c, o);
      if (y2) st4<bf16_t>(y2, base + c, o);
    }
  }
  if (j == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// dx per row; dgamma / dbeta partials per block: part[blk][2][C].  A block's groups take rows
// r0 + g, r0 + g + G, ... (G = groups per block), two rows per group in flight; the groups'
// partials are summed in a fixed order through LDS: deterministic for a given shape.
// Ext (rgbd_add_layernorm_bwd): with clampc > 0 the upstream gradient is masked where the
// forward's clamp(y, -c, c) was not the identity (y recomputed from x, mean, rstd, gamma, beta in
// the forward's operation order: the same bits); dx2 (optional) receives dx rounded to bf16.
struct LnBwdExt {
  const float* beta;
  float clampc;
  bf16_t* dx2;
};
template <typename TX, typename TD, int T, int NCH>
__global__ __launch_bounds__(256) void k_ln_bwd_v(const void* __restrict__ x, const void* __restrict__ dy,
                                                  const float* __restrict__ gamma, const float* __restrict__ mean,
                                                  const float* __restrict__ rstd, int rows, int C, int rb,
                                                  void* __restrict__ dx, float* __restrict__ part, LnBwdExt ext) {
  constexpr int G = 256 / T;
  extern __shared__ float red[];  // [G][2][C]
  const int j = threadIdx.x % T, grp = threadIdx.x / T;
  float pg[NCH][4], pb[NCH][4], gm[NCH][4];
#pragma unroll
  for (int k = 0; k < NCH; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      pg[k][e] = pb[k][e] = 0.f;
      const int c = 4 * (j + T * k) + e;
      gm[k][e] = c < C ? (gamma ? gamma[c] : 1.f) : 0.f;
    }
  const int r0 = blockIdx.x * rb, r1 = min(rows, r0 + rb);
  for (int rowa = r0 + grp; rowa < r1; rowa += 2 * G) {
    int rw[2] = {rowa, rowa + G};
    float xv[2][NCH][4], dv[2][NCH][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {  // both rows' loads in flight together
      const bool ok = rw[u] < r1;
      const long long base = (long long)(ok ? rw[u] : rowa) * C;
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int c = 4 * (j + T * k);
        if (c < C) {
          ld4<TX>(x, base + c, xv[u][k]);
          ld4<TD>(dy, base + c, dv[u][k]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) xv[u][k][e] = dv[u][k][e] = 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool ok = rw[u] < r1;  // group-uniform
      const int row = ok ? rw[u] : rowa;
      const float mu = mean[row], rs = rstd[row];
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int k = 0; k < NCH; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xh = (xv[u][k][e] - mu) * rs;
          if (ext.clampc > 0.f) {  // torch.clamp's backward: the gradient where min <= y <= max
            const int c = 4 * (j + T * k) + e;
            const float yv = xh * gm[k][e] + (c < C && ext.beta ? ext.beta[c] : 0.f);
            if (!(yv >= -ext.clampc && yv <= ext.clampc)) dv[u][k][e] = 0.f;
          }
          const float g = dv[u][k][e] * gm[k][e];
          xv[u][k][e] = xh;
          if (ok) {
            pg[k][e] += dv[u][k][e] * xh;
            pb[k][e] += dv[u][k][e];
          }
          sa += g;
          sb += g * xh;
        }
      const float ma = group_sum<T>(sa) / (float)C, mb = group_sum<T>(sb) / (float)C;
      if (!ok) continue;
      const long long base = (long long)row * C;
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int c = 4 * (j + T * k);
        if (c < C) {
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = rs * (dv[u][k][e] * gm[k][e] - ma - xv[u][k][e] * mb);
          st4<TX>(dx, base + c, o);
          if (ext.dx2) st4<bf16_t>(ext.dx2, base + c, o);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * (j + T * k);
    if (c < C)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        red[(grp * 2) * C + c + e] = pg[k][e];
        red[(grp * 2 + 1) * C + c + e] = pb[k][e];
      }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * C; i += 256) {
    const int w = i / C, c = i % C;
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < G; ++q) t += red[(q * 2 + w) * C + c];
    part[((long long)blockIdx.x * 2 + w) * C + c] = t;
  }
}

// the blocks' dgamma / dbeta partials: 64 columns x 16 block ranges per workgroup, four
// independent accumulators per thread (loads in flight together), the range sums added in a
// fixed order: deterministic for a given shape
__global__ __launch_bounds__(1024) void k_ln_param_reduce_v(const float* __restrict__ part, int nblk, int C,
                                                            float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float sq[16][64];
  const int lane = threadIdx.x & 63, qr = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (col < 2 * C) {
    const int w = col / C, c = col % C;
    const int b0 = (int)((long long)nblk * qr / 16), b1 = (int)((long long)nblk * (qr + 1) / 16);
    const float* p = part + (long long)w * C + c;
    const long long st = 2ll * C;
    int b = b0;
    for (; b + 4 <= b1; b += 4)
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += p[(b + u) * st];
    for (; b < b1; ++b) a[0] += p[b * st];
  }
  sq[qr][lane] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (qr == 0 && col < 2 * C) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += sq[q][lane];
    const int w = col / C, c = col % C;
    (w ? dbeta : dgamma)[c] = t;
  }
}

constexpr int LNV_MAXBLK = 1024;  // backward blocks (partials) of the vectorised path
inline int lnv_rows_per_block(int rows) { return std::max(16, (rows + LNV_MAXBLK - 1) / LNV_MAXBLK); }
inline bool lnv_ok(int C) { return C % 4 == 0 && C <= 64 * 4 * 6; }
inline int lnv_group(int C) {
  const int ch = C / 4;
  return ch <= 16 ? 16 : (ch <= 32 ? 32 : 64);
}

template <typename TX, typename TY, int T, int NCH>
void lnv_fwd_launch(const void* x, const float* gamma, const float* beta, int rows, int C, float eps, void* y,
                    float* mean, float* rstd, hipStream_t s) {
  hipLaunchKernelGGL((k_ln_fwd_v<TX, TY, T, NCH>), dim3(ceil_div(rows, 256 / T)), dim3(256), 0, s, x, gamma, beta,
                     rows, C, eps, y, mean, rstd);
}
template <typename TX, typename TY>
void lnv_fwd(const void* x, const float* gamma, const float* beta, int rows, int C, float eps, void* y, float* mean,
             float* rstd, hipStream_t s) {
  const int T = lnv_group(C), nch = ceil_div(C / 4, T);
  if (T == 16) lnv_fwd_launch<TX, TY, 16, 1>(x, gamma, beta, rows, C, eps, y, mean, rstd, s);
  else if (T == 32) lnv_fwd_launch<TX, TY, 32, 1>(x, gamma, beta, rows, C, eps, y, mean, rstd, s);
  else if (nch == 1) lnv_fwd_launch<TX, TY, 64, 1>(x, gamma, beta, rows, C, eps, y, mean, rstd, s);
  else if (nch == 2) lnv_fwd_launch<TX, TY, 64, 2>(x, gamma, beta, rows, C, eps, y, mean, rstd, s);
  else if (nch == 3) lnv_fwd_launch<TX, TY, 64, 3>(x, gamma, beta, rows, C, eps, y, mean, rstd, s);
  else if (nch == 4) lnv_fwd_launch<TX, TY, 64, 4>(x, gamma, beta, rows, C, eps, y, mean, rstd, s);
  else if (nch == 5) lnv_fwd_launch<TX, TY, 64, 5>(x, gamma, beta, rows, C, eps, y, mean, rstd, s);
  else lnv_fwd_launch<TX, TY, 64, 6>(x, gamma, beta, rows, C, eps, y, mean, rstd, s);
}
template <typename TX, typename TD, int T, int NCH>
void lnv_bwd_launch(const void* x, const void* dy, const float* gamma, const float* mean, const float* rstd, int rows,
                    int C, void* dx, float* part, hipStream_t s, LnBwdExt ext = LnBwdExt{nullptr, 0.f, nullptr}) {
  const int rb = lnv_rows_per_block(rows);
  const size_t smem = (size_t)(256 / T) * 2 * C * sizeof(float);
  hipLaunchKernelGGL((k_ln_bwd_v<TX, TD, T, NCH>), dim3(ceil_div(rows, rb)), dim3(256), smem, s, x, dy, gamma, mean,
                     rstd, rows, C, rb, dx, part, ext);
}
template <typename TX, typename TD>
void lnv_bwd(const void* x, const void* dy, const float* gamma, const float* mean, const float* rstd, int rows, int C,
             void* dx, float* part, hipStream_t s, LnBwdExt ext = LnBwdExt{nullptr, 0.f, nullptr}) {
  const int T = lnv_group(C), nch = ceil_div(C / 4, T);
  if (T == 16) lnv_bwd_launch<TX, TD, 16, 1>(x, dy, gamma, mean, rstd, rows, C, dx, part, s, ext);
  else if (T == 32) lnv_bwd_launch<TX, TD, 32, 1>(x, dy, gamma, mean, rstd, rows, C, dx, part, s, ext);
  else if (nch == 1) lnv_bwd_launch<TX, TD, 64, 1>(x, dy, gamma, mean, rstd, rows, C, dx, part, s, ext);
  else if (nch == 2) lnv_bwd_launch<TX, TD, 64, 2>(x, dy, gamma, mean, rstd, rows, C, dx, part, s, ext);
  else if (nch == 3) lnv_bwd_launch<TX, TD, 64, 3>(x, dy, gamma, mean, rstd, rows, C, dx, part, s, ext);
  else if (nch == 4) lnv_bwd_launch<TX, TD, 64, 4>(x, dy, gamma, mean, rstd, rows, C, dx, part, s, ext);
  else if (nch == 5) lnv_bwd_launch<TX, TD, 64, 5>(x, dy, gamma, mean, rstd, rows, C, dx, part, s, ext);
  else lnv_bwd_launch<TX, TD, 64, 6>(x, dy, gamma, mean, rstd, rows, C, dx, part, s, ext);
}

template <typename TX, typename TR, typename TS, typename TY, int T, int NCH>
void add_lnv_launch(const void* x, const void* r, const float* gamma, const float* beta, int rows, int C, float eps,
                    float clampc, void* s_out, void* y, bf16_t* y2, float* mean, float* rstd, hipStream_t s) {
  hipLaunchKernelGGL((k_add_ln_fwd_v<TX, TR, TS, TY, T, NCH>), dim3(ceil_div(rows, 256 / T)), dim3(256), 0, s, x, r,
                     gamma, beta, rows, C, eps, clampc, s_out, y, y2, mean, rstd);
}
template <typename TX, typename TR, typename TS, typename TY>
void add_lnv(const void* x, const void* r, const float* gamma, const float* beta, int rows, int C, float eps,
             float clampc, void* s_out, void* y, bf16_t* y2, float* mean, float* rstd, hipStream_t s) {
  const int T = lnv_group(C), nch = ceil_div(C / 4, T);
#define ADD_LNV(TT, NN) \
  add_lnv_launch<TX, TR, TS, TY, TT, NN>(x, r, gamma, beta, rows, C, eps, clampc, s_out, y, y2, mean, rstd, s)
  if (T == 16) ADD_LNV(16, 1);
  else if (T == 32) ADD_LNV(32, 1);
  else if (nch == 1) ADD_LNV(64, 1);
  else if (nch == 2) ADD_LNV(64, 2);
  else if (nch == 3) ADD_LNV(64, 3);
  else if (nch == 4) ADD_LNV(64, 4);
  else if (nch == 5) ADD_LNV(64, 5);
  else ADD_LNV(64, 6);
#undef ADD_LNV
}

template <typename TX>
void ln_fwd_t(int y_dtype, const void* x, const float* gamma, const float* beta, int rows, int C, float eps, void* y,
              float* mean, float* rstd, hipStream_t s) {
  if (lnv_ok(C) && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
    if (y_dtype == RGBD_BF16) lnv_fwd<TX, bf16_t>(x, gamma, beta, rows, C, eps, y, mean, rstd, s);
    else lnv_fwd<TX, float>(x, gamma, beta, rows, C, eps, y, mean, rstd, s);
    return;
  }
  dim3 grid(ceil_div(rows, 4));
  if (y_dtype == RGBD_BF16)
    hipLaunchKernelGGL((k_ln_fwd<TX, bf16_t>), grid, dim3(256), 0, s, x, gamma, beta, rows, C, eps, y, mean, rstd);
  else
    hipLaunchKernelGGL((k_ln_fwd<TX, float>), grid, dim3(256), 0, s, x, gamma, beta, rows, C, eps, y, mean, rstd);
}

template <typename TX>
void ln_bwd_t(int dy_dtype, const void* x, const void* dy, const float* gamma, const float* mean, const float* rstd,
              int rows, int C, void* dx, float* part, hipStream_t s) {
  if (lnv_ok(C) && ((uintptr_t)x & 15) == 0 && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)dx & 15) == 0) {
    if (dy_dtype == RGBD_BF16) lnv_bwd<TX, bf16_t>(x, dy, gamma, mean, rstd, rows, C, dx, part, s);
    else lnv_bwd<TX, float>(x, dy, gamma, mean, rstd, rows, C, dx, part, s);
    return;
  }
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

int rgbd_add_layernorm_fwd(int x_dtype, const void* x, int r_dtype, const void* r, const float* gamma,
                           const float* beta, int rows, int C, float eps, float clamp, int y_dtype, void* s_out,
                           void* y, void* y2, float* mean, float* rstd, void* stream) {
  RGBD_REQUIRE(x && r && s_out && y && mean && rstd && rows > 0 && C > 0, RGBD_E_ARG);
  RGBD_REQUIRE(lnv_ok(C), RGBD_E_SHAPE);
  RGBD_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)r & 15) == 0 && ((uintptr_t)s_out & 15) == 0 &&
                   ((uintptr_t)y & 15) == 0 && ((uintptr_t)y2 & 15) == 0,
               RGBD_E_SHAPE);
  RGBD_REQUIRE((x_dtype == RGBD_F32 || x_dtype == RGBD_BF16) && (r_dtype == RGBD_F32 || r_dtype == RGBD_BF16) &&
                   (y_dtype == RGBD_F32 || y_dtype == RGBD_BF16),
               RGBD_E_DTYPE);
  hipStream_t s = (hipStream_t)stream;
  // s in the promoted dtype of x + r: float32 when either is
#define ADD_LN(TX, TR, TS)                                                                      \
  do {                                                                                          \
    if (y_dtype == RGBD_BF16)                                                                   \
      add_lnv<TX, TR, TS, bf16_t>(x, r, gamma, beta, rows, C, eps, clamp, s_out, y, (bf16_t*)y2, mean, rstd, s); \
    else                                                                                        \
      add_lnv<TX, TR, TS, float>(x, r, gamma, beta, rows, C, eps, clamp, s_out, y, (bf16_t*)y2, mean, rstd, s);  \
  } while (0)
  if (x_dtype == RGBD_F32 && r_dtype == RGBD_F32) ADD_LN(float, float, float);
  else if (x_dtype == RGBD_F32) ADD_LN(float, bf16_t, float);
  else if (r_dtype == RGBD_F32) ADD_LN(bf16_t, float, float);
  else ADD_LN(bf16_t, bf16_t, bf16_t);
#undef ADD_LN
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_add_layernorm_bwd(int s_dtype, const void* s_in, int dy_dtype, const void* dy, const float* gamma,
                           const float* beta, const float* mean, const float* rstd, int rows, int C, float clamp,
                           void* ds, void* ds_bf16, float* dgamma, float* dbeta, void* ws, void* stream) {
  RGBD_REQUIRE(s_in && dy && mean && rstd && ds && dgamma && dbeta && ws && rows > 0 && C > 0, RGBD_E_ARG);
  RGBD_REQUIRE(lnv_ok(C), RGBD_E_SHAPE);
  RGBD_REQUIRE(((uintptr_t)s_in & 15) == 0 && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)ds & 15) == 0 &&
                   ((uintptr_t)ds_bf16 & 15) == 0,
               RGBD_E_SHAPE);
  RGBD_REQUIRE((s_dtype == RGBD_F32 || s_dtype == RGBD_BF16) && (dy_dtype == RGBD_F32 || dy_dtype == RGBD_BF16),
               RGBD_E_DTYPE);
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)ws;
  const LnBwdExt ext{beta, clamp, (bf16_t*)ds_bf16};
  if (s_dtype == RGBD_BF16) {
    if (dy_dtype == RGBD_BF16) lnv_bwd<bf16_t, bf16_t>(s_in, dy, gamma, mean, rstd, rows, C, ds, part, s, ext);
    else lnv_bwd<bf16_t, float>(s_in, dy, gamma, mean, rstd, rows, C, ds, part, s, ext);
  } else {
    if (dy_dtype == RGBD_BF16) lnv_bwd<float, bf16_t>(s_in, dy, gamma, mean, rstd, rows, C, ds, part, s, ext);
    else lnv_bwd<float, float>(s_in, dy, gamma, mean, rstd, rows, C, ds, part, s, ext);
  }
  RGBD_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_ln_param_reduce_v, dim3(ceil_div(2 * C, 64)), dim3(1024), 0, s, part,
                     ceil_div(rows, lnv_rows_per_block(rows)), C, dgamma, dbeta);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

size_t rgbd_layernorm_bwd_workspace_size(int rows, int C) {
  if (rows <= 0 || C <= 0) return 256;
  const int nblk = std::max(ceil_div(rows, ln_rows_per_block(rows)), ceil_div(rows, lnv_rows_per_block(rows)));
  return (size_t)nblk * 2 * C * sizeof(float);
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
  const bool vec = lnv_ok(C) && ((uintptr_t)x & 15) == 0 && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)dx & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(k_ln_param_reduce_v, dim3(ceil_div(2 * C, 64)), dim3(1024), 0, s, part,
                       ceil_div(rows, lnv_rows_per_block(rows)), C, dgamma, dbeta);
  else
    hipLaunchKernelGGL(k_ln_param_reduce, dim3(ceil_div(2 * C, 256)), dim3(256), 0, s, part,
                       ceil_div(rows, ln_rows_per_block(rows)), C, dgamma, dbeta);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
