// K3: E-DSAM depth decomposition on device, once per image for all three DSAMs.
//
// Reference: DSAModule (mask2former/utils/custom_model.py:622-798), which per sample and per
// DSAM copies the grey depth to the host, runs np.histogram(512) + scipy find_peaks, builds
// full-resolution numpy masks and copies them back.  Here the same discrete decisions are
// made on device in stream-ordered launches (no host sync), split in two phases:
//  phase A, rgbd_edsam_modes (does not depend on the ratio: runs beside the ratio predictor)
//   1. k_grey_minmax : grey = 0.299 d0 + 0.587 d1 + 0.114 d2 (f32, one rounding per op,
//                      :466-480), written once to the workspace (4 B/px), and nanmin/nanmax via
//                      order-preserving uint keys (:715)
//   2. k_hist        : numpy's uniform-bin fast path over the grey plane (index =
//                      int((x-first)/(last-first)*512) with the +-1 edge corrections),
//                      LDS-privatised 512-bin histogram
//   3. k_modes       : one 512-thread workgroup per image: plateau-aware local maxima
//                      (scipy _local_maxima_1d), wave-cooperative prominence search
//                      (scipy _peak_prominences, wlen = whole signal), threshold
//                      0.01*max(hist) in float64, top-3 by (count, centre) and the centres
//  phase B, rgbd_edsam_codes (after the ratio): one launch
//   4. k_codes_pyramid / k_codes_pool: the windows from the centres and the ratio (:754-772),
//                      then the per-pixel 4-bit region code (bit i <-> conv_layers[i],
//                      :774-798) of the grey plane OR-pooled over the adaptive_max_pool2d bins
//                      of each DSAM input resolution (:687)
// Every float op that feeds a discrete decision uses an explicitly rounded intrinsic, so the
// result is bit-exact to the numpy 2.2 / scipy 1.15 reference.
#include "common.hpp"
#include "timing.hpp"

using namespace rgbd;

namespace {

struct DecWs {
  uint32_t min_key, max_key;
};
constexpr int kDecParts = 128;  // blocks per image of the min/max and histogram passes

__device__ __forceinline__ float grey_at(const float* __restrict__ d, long long HW, long long p, int nch) {
  if (nch == 1) return d[p];  // already grey (DSAModule called with a 1-channel depth map)
  const float a = __fmul_rn(0.299f, d[p]);
  const float b = __fmul_rn(0.587f, d[HW + p]);
  const float c = __fmul_rn(0.114f, d[2 * HW + p]);
  return __fadd_rn(__fadd_rn(a, b), c);
}

struct Range {
  float first, last, step, denom;
  int status;  // 0 ok, 1 non-finite / empty, 2 too many bins
};

__device__ __forceinline__ Range make_range(const DecWs& w) {
  Range r;
  r.status = 0;
  if (w.min_key == 0xffffffffu && w.max_key == 0u) {  // every value NaN
    r.status = 1;
    r.first = r.last = 0.f;
  } else {
    r.first = key_f32(w.min_key);
    r.last = key_f32(w.max_key);
  }
  if (r.status == 0 && (isinf(r.first) || isinf(r.last))) r.status = 1;
  if (r.status == 0 && r.first == r.last) {  // numpy _get_outer_edges: expand by +-0.5
    r.first = __fsub_rn(r.first, 0.5f);
    r.last = __fadd_rn(r.last, 0.5f);
  }
  r.denom = __fsub_rn(r.last, r.first);
  r.step = div_rn(r.denom, 512.f);  // linspace: (stop - start) / 512
  if (r.status == 0 && r.step == 0.f) r.status = 2;
  return r;
}

// np.linspace(first, last, 513, dtype=f32)[i] = i*step + first, last edge forced to `last`.
__device__ __forceinline__ float edge_at(const Range& r, int i) {
  return i == RGBD_NBINS ? r.last : __fadd_rn(__fmul_rn((float)i, r.step), r.first);
}

// One (min, max) key pair per block into part[b][blockIdx.x]; k_hist reduces them (the 96
// blocks x 8 images of same-line atomics this replaced serialised for ~20 us).
__global__ __launch_bounds__(256) void k_grey_minmax(const float* __restrict__ depth3, long long bstride,
                                                     long long HW, int nch, uint2* __restrict__ part,
                                                     rgbd_decomp_info* __restrict__ info, float* __restrict__ grey) {
  const int b = blockIdx.y;
  if (blockIdx.x == 0)  // k_hist adds into the histogram
    for (int i = threadIdx.x; i < RGBD_NBINS; i += 256) info[b].hist[i] = 0;
  const float* d = depth3 + b * bstride;
  float* gout = grey ? grey + b * HW : nullptr;
  uint32_t kmin = 0xffffffffu, kmax = 0u;
  for (long long p = blockIdx.x * 256ll + threadIdx.x; p < HW; p += 256ll * gridDim.x) {
    const float g = grey_at(d, HW, p, nch);
    if (gout) gout[p] = g;
    if (!isnan(g)) {  // np.nanmin / np.nanmax
      const uint32_t k = f32_key(g);
      kmin = min(kmin, k);
      kmax = max(kmax, k);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o));
    kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
  }
  __shared__ uint32_t rmin[4], rmax[4];
  if ((threadIdx.x & 63) == 0) {
    rmin[threadIdx.x >> 6] = kmin;
    rmax[threadIdx.x >> 6] = kmax;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    part[(long long)b * gridDim.x + blockIdx.x] =
        make_uint2(min(min(rmin[0], rmin[1]), min(rmin[2], rmin[3])), max(max(rmax[0], rmax[1]), max(rmax[2], rmax[3])));
}

// Block-level reduction of an image's min/max partials (every k_hist block needs the range).
__device__ __forceinline__ DecWs reduce_parts(const uint2* __restrict__ part, int nparts) {
  uint32_t kmin = 0xffffffffu, kmax = 0u;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    const uint2 v = part[i];
    kmin = min(kmin, v.x);
    kmax = max(kmax, v.y);
  }
  for (int o = 32; o > 0; o >>= 1) {
    kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o));
    kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
  }
  __shared__ uint32_t rmin[4], rmax[4];
  if ((threadIdx.x & 63) == 0) {
    rmin[threadIdx.x >> 6] = kmin;
    rmax[threadIdx.x >> 6] = kmax;
  }
  __syncthreads();
  DecWs w;
  w.min_key = min(min(rmin[0], rmin[1]), min(rmin[2], rmin[3]));
  w.max_key = max(max(rmax[0], rmax[1]), max(rmax[2], rmax[3]));
  return w;
}

__global__ __launch_bounds__(256) void k_hist(const float* __restrict__ depth3, long long bstride,
                                              long long HW, int nch, const uint2* __restrict__ part, DecWs* ws,
                                              rgbd_decomp_info* info) {
  __shared__ uint32_t h[RGBD_NBINS];
  const int b = blockIdx.y;
  const DecWs mm = reduce_parts(part + (long long)b * gridDim.x, gridDim.x);
  if (blockIdx.x == 0 && threadIdx.x == 0) ws[b] = mm;  // for k_modes
  const Range r = make_range(mm);
  if (r.status != 0) return;  // uniform per block
  for (int i = threadIdx.x; i < RGBD_NBINS; i += 256) h[i] = 0;
  __syncthreads();
  const float* d = depth3 + b * bstride;
  for (long long p = blockIdx.x * 256ll + threadIdx.x; p < HW; p += 256ll * gridDim.x) {
    const float g = grey_at(d, HW, p, nch);
    if (!(g >= r.first && g <= r.last)) continue;  // `keep` mask (drops NaN)
    const float f = __fmul_rn(div_rn(__fsub_rn(g, r.first), r.denom), 512.f);
    int idx = (int)f;
    if (idx == RGBD_NBINS) idx -= 1;
    if (g < edge_at(r, idx)) idx -= 1;
    if (g >= edge_at(r, idx + 1) && idx != RGBD_NBINS - 1) idx += 1;
    atomicAdd(&h[idx], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < RGBD_NBINS; i += 256)
    if (h[i]) atomicAdd((uint32_t*)&info[b].hist[i], h[i]);
}

__device__ __forceinline__ long long wave_max_i64(long long v) {
  for (int o = 32; o > 0; o >>= 1) {
    const int lo = __shfl_xor((int)(v & 0xffffffff), o);
    const int hi = __shfl_xor((int)(v >> 32), o);
    const long long u = ((long long)hi << 32) | (uint32_t)lo;
    v = u > v ? u : v;
  }
  return v;
}

__global__ __launch_bounds__(512) void k_modes(const DecWs* ws, rgbd_decomp_info* info, uint32_t* __restrict__ cmask,
                                               int ncmask) {
  __shared__ int x[RGBD_NBINS];
  __shared__ int peaks[RGBD_NBINS];
  __shared__ int is_kept[RGBD_NBINS];
  __shared__ int npeaks, bad;
  __shared__ long long red[8];
  __shared__ int sel[RGBD_MAX_MODES];
  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (b == 0 && cmask && t < ncmask) cmask[t] = 0u;  // phase B ORs the code-presence masks into it
  rgbd_decomp_info* out = info + b;
  Range r = make_range(ws[b]);
  x[t] = out->hist[t];
  is_kept[t] = 0;
  if (t == 0) {
    npeaks = 0;
    bad = 0;
  }
  __syncthreads();
  // linspace monotonicity check (numpy raises "Too many bins for data range")
  if (r.status == 0 && !(edge_at(r, t) < edge_at(r, t + 1))) atomicOr(&bad, 1);
  __syncthreads();
  if (r.status == 0 && bad) r.status = 2;
  if (r.status != 0) {
    if (t == 0) {
      out->status = r.status;
      out->n_modes = 0;
      out->n_masks = RGBD_MAX_MODES + 1;
      out->first_edge = r.first;
      out->last_edge = r.last;
    }
    return;
  }
  // --- local maxima (scipy _local_maxima_1d): plateau starts are x[i-1] < x[i]
  if (t >= 1 && t < RGBD_NBINS - 1 && x[t - 1] < x[t]) {
    int j = t + 1;
    while (j < RGBD_NBINS - 1 && x[j] == x[t]) ++j;
    if (x[j] < x[t]) peaks[atomicAdd(&npeaks, 1)] = (t + j - 1) >> 1;
  }
  // --- max(hist)
  long long mv = wave_max_i64((long long)x[t]);
  if (lane == 0) red[wave] = mv;
  __syncthreads();
  long long hmax = red[0];
  for (int i = 1; i < 8; ++i) hmax = red[i] > hmax ? red[i] : hmax;
  const double pmin = 0.01 * (double)hmax;  // prominence threshold, float64 (:738)
  const int np_ = npeaks;
  // --- prominences, one wave per peak (scipy _peak_prominences, wlen=-1)
  for (int k = wave; k < np_; k += 8) {
    const int p = peaks[k];
    const int v = x[p];
    int lmin = v;
    for (int base = p - 1; base >= 0; base -= 64) {
      const int idx = base - lane;
      const bool in = idx >= 0;
      const int xv = in ? x[idx] : 0;
      const unsigned long long hm = __ballot(in && xv > v);
      const int stop = hm ? __ffsll((long long)hm) - 1 : 64;  // first higher bin (closest to p)
      int cand = (in && lane < stop) ? xv : v;
      for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o));
      lmin = min(lmin, cand);
      if (hm) break;
    }
    int rmin = v;
    for (int base = p + 1; base < RGBD_NBINS; base += 64) {
      const int idx = base + lane;
      const bool in = idx < RGBD_NBINS;
      const int xv = in ? x[idx] : 0;
      const unsigned long long hm = __ballot(in && xv > v);
      const int stop = hm ? __ffsll((long long)hm) - 1 : 64;
      int cand = (in && lane < stop) ? xv : v;
      for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o));
      rmin = min(rmin, cand);
      if (hm) break;
    }
    const int prom = v - max(lmin, rmin);
    if (lane == 0 && pmin <= (double)prom) is_kept[p] = 1;
  }
  __syncthreads();
  // --- top-3 by (count, centre) == (count, bin) descending (:744-750)
  for (int m = 0; m < RGBD_MAX_MODES; ++m) {
    long long key = is_kept[t] ? (((long long)x[t] << 10) | t) : -1ll;
    key = wave_max_i64(key);
    if (lane == 0) red[wave] = key;
    __syncthreads();
    if (t == 0) {
      long long best = red[0];
      for (int i = 1; i < 8; ++i) best = red[i] > best ? red[i] : best;
      sel[m] = best < 0 ? -1 : (int)(best & 1023);
      if (best >= 0) is_kept[best & 1023] = 0;
    }
    __syncthreads();
  }
  if (t == 0) {
    int n = 0;
    for (int m = 0; m < RGBD_MAX_MODES; ++m) {
      const int p = sel[m];
      if (p < 0) break;
      const float e0 = edge_at(r, p), e1 = edge_at(r, p + 1);
      out->peak_bin[m] = p;
      out->center[m] = __fadd_rn(e0, __fmul_rn(__fsub_rn(e1, e0), 0.5f));  // edge + diff/2 (:745)
      out->lo[m] = out->hi[m] = 0.f;                                       // phase B (the ratio)
      ++n;
    }
    for (int m = n; m < RGBD_MAX_MODES; ++m) {
      out->peak_bin[m] = -1;
      out->center[m] = out->lo[m] = out->hi[m] = 0.f;
    }
    out->status = 0;
    out->n_modes = n;
    out->n_masks = n ? n + 1 : RGBD_MAX_MODES + 1;
    out->first_edge = r.first;
    out->last_edge = r.last;
  }
}

// The depth-interval windows of an image (custom_model.py:754-772) from its centres and ratio:
// half = c * r / 2 in f32, lo = max(0, c - half) (0 when clamped), hi = c + half.  Every block of
// a codes launch computes them; ``publish`` (one thread of the launch) also stores them in the
// image's record.
struct Windows {
  int n;
  float lo[RGBD_MAX_MODES], hi[RGBD_MAX_MODES];
};
__device__ __forceinline__ Windows windows_of(rgbd_decomp_info* info, const float* __restrict__ ratio, int b,
                                              bool publish) {
  Windows w;
  w.n = info[b].n_modes;
  const float rr = ratio[b];
  float cen[RGBD_MAX_MODES];  // loaded unconditionally: one round trip, not one per mode
#pragma unroll
  for (int m = 0; m < RGBD_MAX_MODES; ++m) cen[m] = info[b].center[m];
#pragma unroll
  for (int m = 0; m < RGBD_MAX_MODES; ++m) {
    float lo = 0.f, hi = 0.f;
    if (m < w.n) {
      const float c = cen[m];
      const float half = __fmul_rn(__fmul_rn(c, rr), 0.5f);  // c * r / 2 (:768)
      lo = __fsub_rn(c, half);
      if (!(lo > 0.f)) lo = 0.f;                             // max(0, .) (:769)
      hi = __fadd_rn(c, half);                               // (:770)
    }
    w.lo[m] = lo;
    w.hi[m] = hi;
  }
  if (publish)
    for (int m = 0; m < RGBD_MAX_MODES; ++m) {
      info[b].lo[m] = w.lo[m];
      info[b].hi[m] = w.hi[m];
    }
  return w;
}

// The window loop runs to the fixed RGBD_MAX_MODES (t < n predicated) so lo / hi stay in
// registers: a loop to the run-time n indexed them dynamically, which put the two arrays in LDS
// and cost two dependent LDS reads per window per pixel.
__device__ __forceinline__ uint32_t pixel_code(float g, int n, const float* lo, const float* hi) {
  if (n == 0) return 0u;  // no mode: four all-zero masks (:676-678)
  uint32_t c = 0u;
#pragma unroll
  for (int t = 0; t < RGBD_MAX_MODES; ++t)
    if (t < n && g >= lo[t] && g <= hi[t]) c |= 1u << t;  // (d >= lo) & (d <= hi) (:790)
  if (c == 0u) c = 1u << n;                      // remaining region ~union (:795)
  return c;
}

__global__ __launch_bounds__(256) void k_codes_pool(const float* __restrict__ depth3, long long bstride,
                                                    int H, int W, int nch, int oh, int ow, rgbd_decomp_info* info,
                                                    const float* __restrict__ ratio, int publish,
                                                    uint8_t* __restrict__ code) {
  const int b = blockIdx.y;
  const int q = blockIdx.x * 256 + threadIdx.x;
  const Windows win = windows_of(info, ratio, b, publish && blockIdx.x == 0 && threadIdx.x == 0);
  if (q >= oh * ow) return;
  const int i = q / ow, j = q % ow;
  const int n = win.n;
  const float* lo = win.lo;
  const float* hi = win.hi;
  // adaptive_max_pool2d bins: [floor(i*H/oh), ceil((i+1)*H/oh))
  const int y0 = (i * H) / oh, y1 = ((i + 1) * H + oh - 1) / oh;
  const int x0 = (j * W) / ow, x1 = ((j + 1) * W + ow - 1) / ow;
  const long long HW = (long long)H * W;
  const float* d = depth3 + b * bstride;
  uint32_t c = 0u;
  if (n > 0)
    for (int y = y0; y < y1; ++y)
      for (int x = x0; x < x1; ++x) c |= pixel_code(grey_at(d, HW, (long long)y * W + x, nch), n, lo, hi);
  code[(long long)b * oh * ow + q] = (uint8_t)c;
}

// The three-level code pyramid of the Swin input resolutions in one pass, for the common case
// where each level halves the previous one and the first pools whole f0y x f0x pixel blocks:
// a 256-thread block owns 16 x 16 level-0 cells (whole level-1 / level-2 cells: tile origins are
// multiples of 4 cells and level 0 has exactly 4x the level-2 cells), computes each level-0 code
// from its pixels, OR-pools 2 x 2 cells twice through LDS (exactly adaptive_max_pool2d of the
// full-resolution masks, bins nesting), and ORs 1 << code into the per-level presence masks.
template <bool kF4>
__global__ __launch_bounds__(256) void k_codes_pyramid(const float* __restrict__ depth3, long long bstride, int H, int W,
                                                       int nch, int oh0, int ow0, rgbd_decomp_info* info,
                                                       const float* __restrict__ ratio,
                                                       uint8_t* __restrict__ c0, uint8_t* __restrict__ c1,
                                                       uint8_t* __restrict__ c2, uint32_t* __restrict__ cmask) {
  __shared__ uint8_t s0[16][17], s1[8][9];
  __shared__ uint32_t smask[3];
  const int b = blockIdx.z, tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int i = blockIdx.y * 16 + ty, j = blockIdx.x * 16 + tx;
  const int fy = H / oh0, fx = W / ow0;
  const long long HW = (long long)H * W;
  const float* d = depth3 + b * bstride;
  const bool in0 = i < oh0 && j < ow0;
  // the cell's grey rows are loaded before the windows are known (they do not depend on them),
  // so the loads and the windows' record reads are in flight together
  float4 v[4];
  if (kF4 && in0)
#pragma unroll
    for (int y = 0; y < 4; ++y) v[y] = *reinterpret_cast<const float4*>(d + (long long)(4 * i + y) * W + 4 * j);
  const Windows win =
      windows_of(info, ratio, b, blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0);
  const int n = win.n;
  const float* lo = win.lo;
  const float* hi = win.hi;
  if (threadIdx.x < 3) smask[threadIdx.x] = 0u;
  uint32_t c = 0u;
  if (kF4) {  // the grey plane, 4 x 4-pixel cells (the Swin stride): one 16-byte load per cell row
    if (in0 && n > 0) {
#pragma unroll
      for (int y = 0; y < 4; ++y)
        c |= pixel_code(v[y].x, n, lo, hi) | pixel_code(v[y].y, n, lo, hi) | pixel_code(v[y].z, n, lo, hi) |
             pixel_code(v[y].w, n, lo, hi);
    }
  } else if (in0 && n > 0) {
    for (int y = i * fy; y < (i + 1) * fy; ++y)
      for (int x = j * fx; x < (j + 1) * fx; ++x) c |= pixel_code(grey_at(d, HW, (long long)y * W + x, nch), n, lo, hi);
  }
  s0[ty][tx] = (uint8_t)c;
  __syncthreads();
  if (in0) {
    c0[((long long)b * oh0 + i) * ow0 + j] = (uint8_t)c;
    atomicOr(&smask[0], 1u << c);
  }
  const int oh1 = oh0 / 2, ow1 = ow0 / 2, oh2 = oh1 / 2, ow2 = ow1 / 2;
  if (ty < 8 && tx < 8) {
    const uint32_t v = s0[2 * ty][2 * tx] | s0[2 * ty][2 * tx + 1] | s0[2 * ty + 1][2 * tx] | s0[2 * ty + 1][2 * tx + 1];
    s1[ty][tx] = (uint8_t)v;
    const int i1 = blockIdx.y * 8 + ty, j1 = blockIdx.x * 8 + tx;
    if (i1 < oh1 && j1 < ow1) {
      c1[((long long)b * oh1 + i1) * ow1 + j1] = (uint8_t)v;
      atomicOr(&smask[1], 1u << v);
    }
  }
  __syncthreads();
  if (ty < 4 && tx < 4) {
    const uint32_t v = s1[2 * ty][2 * tx] | s1[2 * ty][2 * tx + 1] | s1[2 * ty + 1][2 * tx] | s1[2 * ty + 1][2 * tx + 1];
    const int i2 = blockIdx.y * 4 + ty, j2 = blockIdx.x * 4 + tx;
    if (i2 < oh2 && j2 < ow2) {
      c2[((long long)b * oh2 + i2) * ow2 + j2] = (uint8_t)v;
      atomicOr(&smask[2], 1u << v);
    }
  }
  __syncthreads();
  // every block ORs into the same three words: skip the atomic when the bits are already there
  // (the words only gain bits during the launch, so a stale read can only cause an extra atomic)
  if (cmask && threadIdx.x < 3 && smask[threadIdx.x]) {
    const uint32_t seen = __hip_atomic_load(cmask + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((seen | smask[threadIdx.x]) != seen) atomicOr(cmask + threadIdx.x, smask[threadIdx.x]);
  }
}

// Presence masks of code planes the pyramid kernel did not build (the general path).
__global__ __launch_bounds__(256) void k_codes_presence(const uint8_t* __restrict__ code, long long n,
                                                        uint32_t* __restrict__ cmask) {
  uint32_t m = 0u;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) m |= 1u << (code[i] & 15);
  for (int o = 1; o < 64; o <<= 1) m |= (uint32_t)__shfl_xor((int)m, o);
  if ((threadIdx.x & 63) == 0 && m) atomicOr(cmask, m);
}

// OR-pool a finer code plane into a coarser one when the adaptive bins nest exactly
// (H_in % H_out == 0, W_in % W_out == 0): identical to pooling the full-resolution masks.
__global__ __launch_bounds__(256) void k_codes_or_pool(const uint8_t* __restrict__ fine, int fh, int fw,
                                                       int oh, int ow, uint8_t* __restrict__ code) {
  const int b = blockIdx.y;
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= oh * ow) return;
  const int i = q / ow, j = q % ow, sy = fh / oh, sx = fw / ow;
  uint32_t c = 0u;
  for (int y = i * sy; y < (i + 1) * sy; ++y)
    for (int x = j * sx; x < (j + 1) * sx; ++x) c |= fine[((long long)b * fh + y) * fw + x];
  code[(long long)b * oh * ow + q] = (uint8_t)c;
}

// Windows only (a codes call without output planes): one thread per image.
__global__ void k_windows(rgbd_decomp_info* info, const float* __restrict__ ratio, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) (void)windows_of(info, ratio, b, true);
}

size_t ws_head(int B) {
  const size_t nb = (size_t)(B > 0 ? B : 1);
  return align256(sizeof(DecWs) * nb) + align256(sizeof(uint2) * kDecParts * nb);
}

// phase A: grey (into ``grey`` when given), min/max, histogram, modes
int modes_impl(const float* depth3, long long batch_stride, int nch, int B, int H, int W, rgbd_decomp_info* info,
               void* ws, float* grey, uint32_t* code_masks, int n_scales, hipStream_t st) {
  DecWs* w = (DecWs*)ws;
  const long long HW = (long long)H * W;
  dim3 grid((unsigned)std::min<long long>(ceil_div(HW, 256), kDecParts), B);
  uint2* part = (uint2*)((char*)ws + align256(sizeof(DecWs) * (size_t)B));
  k_grey_minmax<<<grid, 256, 0, st>>>(depth3, batch_stride, HW, nch, part, info, grey);
  if (grey)
    k_hist<<<grid, 256, 0, st>>>(grey, HW, HW, 1, part, w, info);
  else
    k_hist<<<grid, 256, 0, st>>>(depth3, batch_stride, HW, nch, part, w, info);
  k_modes<<<B, 512, 0, st>>>(w, info, code_masks, n_scales);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

// phase B: windows + region codes of the (grey or 3-plane) depth at the given resolutions
int codes_impl(const float* src, long long sstride, int nch, int B, int H, int W, const float* ratio, int n_scales,
               const int* out_h_host, const int* out_w_host, uint8_t* const* codes_host, rgbd_decomp_info* info,
               uint32_t* code_masks, hipStream_t st) {
  TimerScope ts("decompose", st);
  if (n_scales == 0) {
    k_windows<<<ceil_div(B, 64), 64, 0, st>>>(info, ratio, B);
    RGBD_CHECK_LAUNCH();
    return RGBD_OK;
  }
  // the Swin pyramid (each level half the previous, level 0 whole pixel blocks): one launch
  const bool pyramid = n_scales == 3 && H % out_h_host[0] == 0 && W % out_w_host[0] == 0 && out_h_host[0] % 4 == 0 &&
                       out_w_host[0] % 4 == 0 && out_h_host[1] * 2 == out_h_host[0] &&
                       out_w_host[1] * 2 == out_w_host[0] && out_h_host[2] * 2 == out_h_host[1] &&
                       out_w_host[2] * 2 == out_w_host[1];
  if (pyramid) {
    dim3 g3(ceil_div(out_w_host[0], 16), ceil_div(out_h_host[0], 16), B);
    // 16-byte loads: one grey plane (nch 1), 4 x 4 cells, rows 16-byte aligned
    const bool f4 = nch == 1 && H == 4 * out_h_host[0] && W == 4 * out_w_host[0] && W % 4 == 0 && sstride % 4 == 0 &&
                    ((uintptr_t)src & 15) == 0;
    if (f4)
      k_codes_pyramid<true><<<g3, 256, 0, st>>>(src, sstride, H, W, nch, out_h_host[0], out_w_host[0], info, ratio,
                                                codes_host[0], codes_host[1], codes_host[2], code_masks);
    else
      k_codes_pyramid<false><<<g3, 256, 0, st>>>(src, sstride, H, W, nch, out_h_host[0], out_w_host[0], info, ratio,
                                                 codes_host[0], codes_host[1], codes_host[2], code_masks);
    RGBD_CHECK_LAUNCH();
    return RGBD_OK;
  }
  for (int s = 0; s < n_scales; ++s) {
    const int oh = out_h_host[s], ow = out_w_host[s];
    dim3 g2(ceil_div((long long)oh * ow, 256), B);
    // a previous (finer) scale whose bins nest exactly into this one's: pool its codes
    int srcs = -1;
    for (int t = 0; t < s; ++t) {
      const int fh = out_h_host[t], fw = out_w_host[t];
      if (fh >= oh && fw >= ow && fh % oh == 0 && fw % ow == 0 && H % fh == 0 && W % fw == 0) srcs = t;
    }
    if (srcs >= 0)
      k_codes_or_pool<<<g2, 256, 0, st>>>(codes_host[srcs], out_h_host[srcs], out_w_host[srcs], oh, ow,
                                          codes_host[s]);
    else  // scale 0 always pools the pixels: its launch also publishes the windows
      k_codes_pool<<<g2, 256, 0, st>>>(src, sstride, H, W, nch, oh, ow, info, ratio, s == 0, codes_host[s]);
    if (code_masks) {
      const long long nb = (long long)B * oh * ow;
      k_codes_presence<<<(unsigned)std::min<long long>(ceil_div(nb, 256 * 8), 256), 256, 0, st>>>(codes_host[s], nb,
                                                                                              code_masks + s);
    }
  }
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int check_scales(int B, int H, int W, int n_scales, const int* out_h_host, const int* out_w_host,
                 uint8_t* const* codes_host) {
  RGBD_REQUIRE(B > 0 && H > 0 && W > 0 && n_scales >= 0 && n_scales <= 8, RGBD_E_ARG);
  for (int s = 0; s < n_scales; ++s) {
    RGBD_REQUIRE(out_h_host && out_w_host && codes_host && codes_host[s], RGBD_E_ARG);
    RGBD_REQUIRE(out_h_host[s] > 0 && out_w_host[s] > 0 && out_h_host[s] <= H && out_w_host[s] <= W, RGBD_E_SHAPE);
  }
  return RGBD_OK;
}

}  // namespace

extern "C" {

size_t rgbd_edsam_decompose_workspace_size(int B) { return ws_head(B); }

size_t rgbd_edsam_modes_workspace_size(int B, int H, int W) {
  return ws_head(B) + align256(sizeof(float) * (size_t)(B > 0 ? B : 1) * (H > 0 ? H : 1) * (W > 0 ? W : 1));
}

static int decompose(const float* depth3, long long batch_stride, int depth_channels, int B, int H, int W,
                     const float* ratio, int n_scales, const int* out_h_host, const int* out_w_host,
                     uint8_t* const* codes_host, rgbd_decomp_info* info, uint32_t* code_masks, void* ws,
                     void* stream) {
  RGBD_REQUIRE(depth3 && ratio && info && ws, RGBD_E_ARG);
  RGBD_REQUIRE(depth_channels == 1 || depth_channels == 3, RGBD_E_SHAPE);
  const int rc = check_scales(B, H, W, n_scales, out_h_host, out_w_host, codes_host);
  if (rc != RGBD_OK) return rc;
  hipStream_t st = (hipStream_t)stream;
  const int ra = modes_impl(depth3, batch_stride, depth_channels, B, H, W, info, ws, nullptr, code_masks, n_scales, st);
  if (ra != RGBD_OK) return ra;
  return codes_impl(depth3, batch_stride, depth_channels, B, H, W, ratio, n_scales, out_h_host, out_w_host, codes_host,
                    info, code_masks, st);
}

int rgbd_edsam_decompose(const float* depth3, long long batch_stride, int depth_channels, int B, int H, int W,
                         const float* ratio, int n_scales, const int* out_h_host,
                         const int* out_w_host, uint8_t* const* codes_host, rgbd_decomp_info* info,
                         void* ws, void* stream) {
  return decompose(depth3, batch_stride, depth_channels, B, H, W, ratio, n_scales, out_h_host, out_w_host, codes_host,
                   info, nullptr, ws, stream);
}

int rgbd_edsam_decompose_masks(const float* depth3, long long batch_stride, int depth_channels, int B, int H, int W,
                               const float* ratio, int n_scales, const int* out_h_host, const int* out_w_host,
                               uint8_t* const* codes_host, rgbd_decomp_info* info, uint32_t* code_masks, void* ws,
                               void* stream) {
  RGBD_REQUIRE(code_masks, RGBD_E_ARG);
  return decompose(depth3, batch_stride, depth_channels, B, H, W, ratio, n_scales, out_h_host, out_w_host, codes_host,
                   info, code_masks, ws, stream);
}

int rgbd_edsam_modes(const float* depth3, long long batch_stride, int depth_channels, int B, int H, int W,
                     rgbd_decomp_info* info, uint32_t* code_masks, int n_masks, void* ws, void* stream) {
  RGBD_REQUIRE(depth3 && info && ws, RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && H > 0 && W > 0 && n_masks >= 0 && n_masks <= 8, RGBD_E_ARG);
  RGBD_REQUIRE(depth_channels == 1 || depth_channels == 3, RGBD_E_SHAPE);
  TimerScope ts("decompose_modes", (hipStream_t)stream);
  float* grey = (float*)((char*)ws + ws_head(B));
  return modes_impl(depth3, batch_stride, depth_channels, B, H, W, info, ws, grey, code_masks, n_masks,
                    (hipStream_t)stream);
}

int rgbd_edsam_codes(const void* ws, int B, int H, int W, const float* ratio, int n_scales, const int* out_h_host,
                     const int* out_w_host, uint8_t* const* codes_host, rgbd_decomp_info* info,
                     uint32_t* code_masks, void* stream) {
  RGBD_REQUIRE(ws && ratio && info, RGBD_E_ARG);
  const int rc = check_scales(B, H, W, n_scales, out_h_host, out_w_host, codes_host);
  if (rc != RGBD_OK) return rc;
  const float* grey = (const float*)((const char*)ws + ws_head(B));
  return codes_impl(grey, (long long)H * W, 1, B, H, W, ratio, n_scales, out_h_host, out_w_host, codes_host, info,
                    code_masks, (hipStream_t)stream);
}

}  // extern "C"
