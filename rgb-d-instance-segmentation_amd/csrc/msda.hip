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
// Backward (k_msda_bwd): per (level, point) the group reduces go . sample (attention-weight
// gradient) and go . d sample / d(ix, iy) (sampling-location gradient) with shuffles, and
// scatters weight * tap weight * go into the value gradient with float atomics (as
// grid_sample's backward does).  Bound: the atomic byte rate.
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
      // the four taps loaded unconditionally (a padding tap reads cell 0 and is not added), so the
      // loads issue together instead of one branch and one memory round trip per tap
      float v[4][8];
#pragma unroll
      for (int e = 0; e < 4; ++e) ld8(vl + (long long)max(t.idx[e], 0) * NH * D, v[e]);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int c = 0; c < 8; ++c) s[c] = t.idx[e] >= 0 ? s[c] + t.w[e] * v[e][c] : s[c];
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

// Backward: one group of D lanes per (image, query, head), lane c = channel c (a tap's value
// row is one 128-byte line in f32): per (level, point) the group reduces go . sample (attention-
// weight gradient) and go . d sample / d(ix, iy) (sampling-location gradient) with shuffles and
// scatters a * w_tap * go into the value gradient with float atomics, each wave-instruction two
// 128-byte row segments (MI355X_MICROARCH "Global float atomics": the full-rate shape).  Bound:
// the atomic byte rate (~1.3 TB/s; 2.5 GB at the C2 pixel decoder).  Measured alternative
// (r03): the value gradient gathered into a float32 LDS tile per (image, head, level, 8
// channels) with ds_add_f32 — 1.4x SLOWER (2.7 vs 1.9 ms at C2): LDS float atomics ran at about
// a tenth of plain LDS read-modify-write (same kernel with racy plain adds: 0.27 ms), with or
// without same-address conflicts.
template <typename T, int D>
__global__ __launch_bounds__(256) void k_msda_bwd(const T* __restrict__ value, MsdaLevels lv, int S, int Q, int NH,
                                                  int P, const float* __restrict__ loc, const float* __restrict__ attw,
                                                  const T* __restrict__ gout, long long nqh, float* __restrict__ gvalue,
                                                  float* __restrict__ gloc, float* __restrict__ gattw) {
  const int c = threadIdx.x % D;
  const long long qh = (long long)blockIdx.x * (256 / D) + threadIdx.x / D;
  // every lane of a group takes part in the shuffles: out-of-range groups run with zero weight
  const bool live = qh < nqh;
  const long long q0 = live ? qh : 0;
  const int h = (int)(q0 % NH);
  const long long b = (q0 / NH) / Q;
  const float* lq = loc + q0 * lv.L * P * 2;
  const float* wq = attw + q0 * lv.L * P;
  const long long voff = b * S * NH * D + (long long)h * D + c;
  const T* vb = value + voff;
  float* gvb = gvalue + voff;
  const float go = live ? Num<T>::to_f(gout[q0 * D + c]) : 0.f;
  for (int l = 0; l < lv.L; ++l) {
    const int H = lv.H[l], W = lv.W[l];
    const long long lo = (long long)lv.start[l] * NH * D;
    for (int p = 0; p < P; ++p) {
      const int k = l * P + p;
      const Tap t = msda_tap(lq[2 * k], lq[2 * k + 1], H, W);
      const float a = wq[k];
      float v[4];  // unconditional loads (padding taps read cell 0, then count as zero)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = Num<T>::to_f(vb[lo + (long long)max(t.idx[e], 0) * NH * D]);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = t.idx[e] >= 0 ? v[e] : 0.f;
      const float s = t.w[0] * v[0] + t.w[1] * v[1] + t.w[2] * v[2] + t.w[3] * v[3];
      // d sample / d ix, d iy (zero-padded taps are zeros)
      const float dsx = (1.f - t.ly) * (v[1] - v[0]) + t.ly * (v[3] - v[2]);
      const float dsy = (1.f - t.lx) * (v[2] - v[0]) + t.lx * (v[3] - v[1]);
      const float gw = group_sum<D>(go * s);
      const float gx = group_sum<D>(go * dsx);
      const float gy = group_sum<D>(go * dsy);
      if (live) {
        if (c == 0) {
          gattw[q0 * lv.L * P + k] = gw;
          // ix = loc * W - 1/2 through grid = 2 loc - 1: d ix / d loc = W
          gloc[(q0 * lv.L * P + k) * 2] = a * gx * (float)W;
          gloc[(q0 * lv.L * P + k) * 2 + 1] = a * gy * (float)H;
        }
        const float ga = a * go;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (t.idx[e] >= 0) atomicAdd(gvb + lo + (long long)t.idx[e] * NH * D, ga * t.w[e]);
      }
    }
  }
}

// Backward over runs of R consecutive queries of one (image, head), per group of D lanes (lane c =
// channel c), for the reference configuration's L levels x P points (compile-time, so the
// per-slot state lives in registers).  Neighbouring queries sample neighbouring places: a query
// one pixel further right samples, per (level, point), the same bilinear cells shifted by one
// cell on its own level and by half / a quarter of a cell on the coarser ones, so two or all four
// of its taps are cells the previous query also scattered into.  Each (level, point) slot keeps
// the previous query's four (cell, a * w_tap * go) contributions in registers; a new query's tap
// on one of those cells adds the held value to its own, and only contributions whose cell the
// next query does not touch are flushed with a float atomic (same full-rate shape: two 128-byte
// row segments per wave-instruction).  The sums are the same (float addition order aside: the
// atomics already leave it unspecified); how many atomics are saved depends on how smoothly the
// sampling offsets vary across neighbouring queries (spatially constant at the pixel decoder's
// initialisation: about 60 % fewer at C2).
// one value element through a buffer descriptor: a 32-bit byte offset per lane instead of a 64-bit
// address (the run's 32 tap loads in flight at once would otherwise hold 64 address registers)
__device__ __forceinline__ bf16_t buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t e, bf16_t*) {
  return (bf16_t)__builtin_amdgcn_raw_buffer_load_b16(r, e * 2u, 0, 0);
}
__device__ __forceinline__ float buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t e, float*) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, e * 4u, 0, 0));
}

template <typename T, int D, int L, int P, int R>
__global__ __launch_bounds__(256) void k_msda_bwd_runs(const T* __restrict__ value, int vbytes, MsdaLevels lv, int S,
                                                       int Q, int NH, const float* __restrict__ loc,
                                                       const float* __restrict__ attw, const T* __restrict__ gout,
                                                       long long ngroups, int nrun, float* __restrict__ gvalue,
                                                       float* __restrict__ gloc, float* __restrict__ gattw) {
  constexpr int LP = L * P;
  const int c = threadIdx.x % D;
  const long long gid = (long long)blockIdx.x * (256 / D) + threadIdx.x / D;
  // every lane of a group takes part in the shuffles: out-of-range groups run with zero weight
  const bool glive = gid < ngroups;
  const long long g0 = glive ? gid : 0;
  const int h = (int)(g0 % NH);
  const long long br = g0 / NH;
  const int run = (int)(br % nrun);
  const long long b = br / nrun;
  const int qa = run * R, qn = min(R, Q - qa);
  const long long voff = b * S * NH * D + (long long)h * D + c;
  float* gvb = gvalue + voff;
  const __amdgpu_buffer_rsrc_t vrs = wt_rsrc(value, vbytes);  // the host checks vbytes < 2^31
  float gos[R];  // unconditional loads (a query past the run's end reads the run's first)
#pragma unroll
  for (int i = 0; i < R; ++i) gos[i] = Num<T>::to_f(gout[((b * Q + qa + (i < qn ? i : 0)) * NH + h) * D + c]);
#pragma unroll
  for (int i = 0; i < R; ++i) gos[i] = glive && i < qn ? gos[i] : 0.f;
  // slot-major: one (level, point) slot over the run's queries, its held taps in 8 registers
  for (int k = 0; k < LP; ++k) {
    const int l = k / P;
    const int H = lv.H[l], W = lv.W[l];
    const long long lo = (long long)lv.start[l] * NH * D;
    int pidx[4] = {-1, -1, -1, -1};
    float pval[4] = {0.f, 0.f, 0.f, 0.f};
    // the slot's locations and attention weights for the whole run, loaded together up front
    float2 lq[R];
    float aq[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const long long q0 = glive && i < qn ? (b * Q + qa + i) * NH + h : 0;
      lq[i] = *reinterpret_cast<const float2*>(loc + (q0 * LP + k) * 2);
      aq[i] = attw[q0 * LP + k];
    }
    // every tap value of the slot's run, issued together before any of the slot's stores and
    // atomics: those count in the same vmcnt, so a load issued after them would wait for them
    // too (unconditional: padding taps read cell 0, then count as zero)
    T vr[R][4];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const Tap t = msda_tap(lq[i].x, lq[i].y, H, W);
#pragma unroll
      for (int e = 0; e < 4; ++e) vr[i][e] = buf_ld(vrs, (uint32_t)(voff + lo + (long long)max(t.idx[e], 0) * NH * D), (T*)nullptr);
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const bool live = glive && i < qn;  // group-uniform
      const long long q0 = live ? (b * Q + qa + i) * NH + h : 0;
      const float go = gos[i];
      const Tap t = msda_tap(lq[i].x, lq[i].y, H, W);
      const float a = live ? aq[i] : 0.f;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = t.idx[e] >= 0 ? Num<T>::to_f(vr[i][e]) : 0.f;
      const float s = t.w[0] * v[0] + t.w[1] * v[1] + t.w[2] * v[2] + t.w[3] * v[3];
      const float dsx = (1.f - t.ly) * (v[1] - v[0]) + t.ly * (v[3] - v[2]);
      const float dsy = (1.f - t.lx) * (v[2] - v[0]) + t.lx * (v[3] - v[1]);
      const float gw = group_sum<D>(go * s);
      const float gx = group_sum<D>(go * dsx);
      const float gy = group_sum<D>(go * dsy);
      if (live && c == 0) {
        gattw[q0 * LP + k] = gw;
        gloc[(q0 * LP + k) * 2] = a * gx * (float)W;
        gloc[(q0 * LP + k) * 2 + 1] = a * gy * (float)H;
      }
      const float ga = a * go;
      int nidx[4];
      float nv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        nidx[e] = live ? t.idx[e] : -1;
        nv[e] = nidx[e] >= 0 ? ga * t.w[e] : 0.f;
      }
      // the held contributions: carried into a tap on the same cell, else flushed
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bool carried = false;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (pidx[j] >= 0 && nidx[e] == pidx[j]) {
            nv[e] += pval[j];
            carried = true;
          }
        if (pidx[j] >= 0 && !carried) atomicAdd(gvb + lo + (long long)pidx[j] * NH * D, pval[j]);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pidx[e] = nidx[e];
        pval[e] = nv[e];
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (pidx[e] >= 0) atomicAdd(gvb + lo + (long long)pidx[e] * NH * D, pval[e]);
  }
}

// queries per run of k_msda_bwd_runs: longer runs carry more taps but hold more registers
// (measured at C2, bf16, tools/micro_msda_bwd.py: R = 2/3/4/5/6/8/16 -> 1398/1084/1003/973/938/
// 1107/2077 us; 6 is the longest run at 3 waves per SIMD without spills; forcing the taps to be
// recomputed after the loads instead of held saves ~30 registers but measured slower at R = 4-8)
constexpr int MSDA_RUN = 6;

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
  // the value gradient is accumulated with atomics: zero it first (stream-ordered)
  const hipError_t e = hipMemsetAsync(gvalue, 0, sizeof(float) * (size_t)B * S * NH * D, s);
  if (e != hipSuccess) return (int)e;
  const long long vbytes = (long long)B * S * NH * D * (long long)sizeof(T);
  if (lv.L == 3 && P == 4 && vbytes < (1ll << 31)) {  // the reference configuration (3 levels x 4 points)
    const int nrun = ceil_div(Q, MSDA_RUN);
    const long long ngroups = (long long)B * nrun * NH;
    k_msda_bwd_runs<T, D, 3, 4, MSDA_RUN><<<(unsigned)ceil_div(ngroups, 256 / D), 256, 0, s>>>(
        (const T*)value, (int)vbytes, lv, S, Q, NH, loc, attw, (const T*)gout, ngroups, nrun, gvalue, gloc, gattw);
    return RGBD_OK;
  }
  k_msda_bwd<T, D><<<(unsigned)ceil_div(nqh, 256 / D), 256, 0, s>>>((const T*)value, lv, S, Q, NH, P, loc, attw,
                                                                   (const T*)gout, nqh, gvalue, gloc, gattw);
  return RGBD_OK;
}

// Sampling locations of the two-coordinate reference points (:990-994):
//   loc[b][q][h][l][p][c] = ref[b][q][l][c] + (off[b][q][h][l][p][c] / norm[l][c])
// with the division in the offsets' dtype (torch: bf16 / int64 -> bf16, computed in float and
// rounded), the sum in float32; backward: goff = (float(round(gloc)) / norm) rounded to the offsets'
// dtype (the add's gradient cast to that dtype, then the division's).
template <typename T>
__global__ __launch_bounds__(256) void k_msda_loc(const float* __restrict__ ref, const T* __restrict__ off,
                                                  const float* __restrict__ norm, long long n, int NH, int L, int P,
                                                  float* __restrict__ loc) {
  const long long i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i & 1);
  const long long j = i >> 1;                        // (b, q, h, l, p)
  const int l = (int)((j / P) % L);
  const long long bq = j / ((long long)P * L * NH);
  const float q = Num<T>::to_f(Num<T>::from_f(Num<T>::to_f(off[i]) / norm[2 * l + c]));
  loc[i] = ref[(bq * L + l) * 2 + c] + q;
}
template <typename T>
__global__ __launch_bounds__(256) void k_msda_loc_bwd(const float* __restrict__ gloc, const float* __restrict__ norm,
                                                      long long n, int L, int P, T* __restrict__ goff) {
  const long long i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i & 1);
  const int l = (int)(((i >> 1) / P) % L);
  const float g = Num<T>::to_f(Num<T>::from_f(gloc[i]));
  goff[i] = Num<T>::from_f(g / norm[2 * l + c]);
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

extern "C" int rgbd_msda_locations(int dtype, const float* ref, const void* off, const float* norm, int B, int Q,
                                   int NH, int L, int P, float* loc, void* stream) {
  RGBD_REQUIRE(ref && off && norm && loc && B > 0 && Q > 0 && NH > 0 && L > 0 && P > 0, RGBD_E_ARG);
  RGBD_REQUIRE(dtype == RGBD_F32 || dtype == RGBD_BF16, RGBD_E_DTYPE);
  const long long n = (long long)B * Q * NH * L * P * 2;
  const unsigned grid = (unsigned)((n + 255) / 256);
  if (dtype == RGBD_F32)
    k_msda_loc<float><<<grid, 256, 0, (hipStream_t)stream>>>(ref, (const float*)off, norm, n, NH, L, P, loc);
  else
    k_msda_loc<bf16_t><<<grid, 256, 0, (hipStream_t)stream>>>(ref, (const bf16_t*)off, norm, n, NH, L, P, loc);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

extern "C" int rgbd_msda_locations_bwd(int dtype, const float* gloc, const float* norm, int B, int Q, int NH, int L,
                                       int P, void* goff, void* stream) {
  RGBD_REQUIRE(gloc && norm && goff && B > 0 && Q > 0 && NH > 0 && L > 0 && P > 0, RGBD_E_ARG);
  RGBD_REQUIRE(dtype == RGBD_F32 || dtype == RGBD_BF16, RGBD_E_DTYPE);
  const long long n = (long long)B * Q * NH * L * P * 2;
  const unsigned grid = (unsigned)((n + 255) / 256);
  if (dtype == RGBD_F32)
    k_msda_loc_bwd<float><<<grid, 256, 0, (hipStream_t)stream>>>(gloc, norm, n, L, P, (float*)goff);
  else
    k_msda_loc_bwd<bf16_t><<<grid, 256, 0, (hipStream_t)stream>>>(gloc, norm, n, L, P, (bf16_t*)goff);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}
