// K4: EnhancedDepthImageRatioPredictor (mask2former/utils/custom_model.py:1363-1487) on gfx950.
//
// 216 GFLOP/img at 640x480 — the FLOP-dominant row of the hot path (SURVEY Finding 1).
// Stages (one float32 depth image [3,H,W] in, one ratio out):
//   chain  : per pixel, fully in registers, three chained MFMA GEMMs (k_rp_chain):
//            stem   = the three 'same' convs 3x3 / 5x5 / 7x7 (3->64 each, :1378-1394) merged into
//                     ONE 7x7 conv 3->192 (3x3 and 5x5 kernels embedded at the centre, zero
//                     elsewhere; torch.cat order of :1463 preserved), implicit GEMM K=147->160
//            fusion = 1x1 192->128 (:1397-1401), attention 1x1 128->64 ->ReLU-> 64->128 ->sigmoid
//                     and the gate (:1404-1470).  Each GEMM's accumulator (channel in the
//                     registers, pixel on the lane) is directly the next GEMM's B operand; the
//                     packed weights use the matching k permutation, so nothing touches LDS.
//   conv5  : 3x3 128->256 (:1413), 84 % of the FLOPs, LDS-tiled implicit GEMM (bf16:
//            k_rp_conv5_v4, 16x32-pixel tiles x 128-channel halves over 32-channel quarters, the
//            halo of a quarter staged once for all 9 taps; float32: k_rp_conv3x3): output y +
//            per-workgroup BN partial sums (train), or BN + ReLU + pool in the epilogue (eval)
//   pool   : BN + ReLU + AdaptiveAvgPool(4) streamed over y (k_rp_bn_relu_pool*)
//   tail   : 3x3 256->512 on 4x4 + BN + ReLU + GAP (k_rp_tail_conv), MLP + dropout + sigmoid
//            (k_rp_tail_mlp), ratio = 0.01 + 0.49 sigmoid(raw) (:1485).
// BatchNorm: eval mode uses running stats (folded into per-channel scale/shift); train mode
// uses batch statistics (three recompute passes of the chain for the stem / fusion BNs,
// deterministic fixed-order reductions in double) and updates running stats like torch
// (momentum, unbiased variance).  Dropout uses a counter-hash RNG (train mode only).
#include <cstdlib>
#include <type_traits>

#include "mfma.hpp"
#include "timing.hpp"

using namespace rgbd;

namespace {

constexpr int STEM_K = 160, STEM_C = 192, FUS_C = 128, ATT_C = 64, C5 = 256, C6 = 512;
// bf16 chain v2 stem: k = (c*7 + dy)*8 + dx over the 7x7 window, dx = 7 a zero pad (21 groups of 8)
constexpr int STEM_K2 = 168;
constexpr int NBN = 6;  // BN layers: scale1, scale2, scale3, fusion, fe.1, fe.5
constexpr float BN_EPS = 1e-5f;

struct Layout {  // byte offsets into the packed blob
  size_t w1, b1, w2, b2, w3, b3, w4, b4, w5, b5, w6, b6, w7, b7, w8, b8, w9, b9, w10, b10;
  size_t zero;       // 256 zero bytes
  size_t w5q;        // bf16: conv5 weights in k_rp_conv5_v4's step order
  size_t w1s;        // bf16: stem weights in the chain v2 K order
  size_t w1f, w2f;   // bf16 blobs: f32 stem (w1s order) and fusion (chain order) weights, the BN-fold sources
  size_t total;
};

inline Layout make_layout(int es) {
  Layout L;
  size_t o = 0;
  auto seg = [&](size_t bytes) {
    size_t r = o;
    o += align256(bytes);
    return r;
  };
  L.w1 = seg((size_t)STEM_C * STEM_K * es);
  L.b1 = seg(STEM_C * 4);
  L.w2 = seg((size_t)FUS_C * STEM_C * es);
  L.b2 = seg(FUS_C * 4);
  L.w3 = seg((size_t)ATT_C * FUS_C * es);
  L.b3 = seg(ATT_C * 4);
  L.w4 = seg((size_t)FUS_C * ATT_C * es);
  L.b4 = seg(FUS_C * 4);
  L.w5 = seg((size_t)C5 * 9 * FUS_C * es);
  L.b5 = seg(C5 * 4);
  L.w6 = seg((size_t)C6 * C5 * 9 * 4);
  L.b6 = seg(C6 * 4);
  L.w7 = seg(128 * 512 * 4);
  L.b7 = seg(128 * 4);
  L.w8 = seg(64 * 128 * 4);
  L.b8 = seg(64 * 4);
  L.w9 = seg(32 * 64 * 4);
  L.b9 = seg(32 * 4);
  L.w10 = seg(32 * 4);
  L.b10 = seg(4);
  L.zero = seg(256);
  L.w1s = seg(es == 2 ? (size_t)STEM_C * STEM_K2 * 2 : 0);
  L.w1f = seg(es == 2 ? (size_t)STEM_C * STEM_K2 * 4 : 0);
  L.w2f = seg(es == 2 ? (size_t)FUS_C * STEM_C * 4 : 0);
  L.w5q = seg(es == 2 ? (size_t)C5 * 9 * FUS_C * 2 : 0);
  L.total = o;
  return L;
}

// chained-operand permutation: packed position (g, e) of a 32-wide k step <-> channel
__host__ __device__ __forceinline__ int chain_perm(int g, int e) { return e < 4 ? 4 * g + e : 16 + 4 * g + (e - 4); }

struct WPtrs {  // reference-layout float32 weights (device), order of RGBD_RATIO_NW
  const float* p[RGBD_RATIO_NW];
};
struct BnPtrs {  // per BN layer: weight, bias, running_mean, running_var
  float* p[NBN * 4];
};

// ------------------------------------------------------------------ packing
template <typename T>
__global__ void k_rp_pack(WPtrs w, char* blob, Layout L) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
  T* w1 = (T*)(blob + L.w1);
  float* b1 = (float*)(blob + L.b1);
  for (int e = tid; e < STEM_C * STEM_K; e += nth) {  // stem: k = tap*3 + c over a 7x7 window
    const int o = e / STEM_K, k = e % STEM_K;
    float v = 0.f;
    if (k < 147) {
      const int tap = k / 3, c = k % 3, ky = tap / 7, kx = tap % 7;
      const int br = o / 64, oo = o % 64, ks = 3 + 2 * br, off = 3 - ks / 2;  // 3x3 / 5x5 / 7x7
      const int y = ky - off, x = kx - off;
      if (y >= 0 && y < ks && x >= 0 && x < ks) v = w.p[2 * br][((oo * 3 + c) * ks + y) * ks + x];
    }
    w1[e] = Num<T>::from_f(v);
  }
  for (int e = tid; e < STEM_C; e += nth) b1[e] = w.p[2 * (e / 64) + 1][e % 64];
  // chained 1x1 layers: packed[o][32s + 8g + e] = W[o][32s + perm(g, e)]
  auto pack_chain = [&](const float* src, T* dst, int O, int K) {
    for (int e = tid; e < O * K; e += nth) {
      const int o = e / K, kk = e % K, s = kk / 32, g = (kk % 32) / 8, ee = kk % 8;
      dst[e] = Num<T>::from_f(src[o * K + 32 * s + chain_perm(g, ee)]);
    }
  };
  pack_chain(w.p[6], (T*)(blob + L.w2), FUS_C, STEM_C);
  pack_chain(w.p[8], (T*)(blob + L.w3), ATT_C, FUS_C);
  pack_chain(w.p[10], (T*)(blob + L.w4), FUS_C, ATT_C);
  for (int e = tid; e < FUS_C; e += nth) ((float*)(blob + L.b2))[e] = w.p[7][e];
  for (int e = tid; e < ATT_C; e += nth) ((float*)(blob + L.b3))[e] = w.p[9][e];
  for (int e = tid; e < FUS_C; e += nth) ((float*)(blob + L.b4))[e] = w.p[11][e];
  // conv5 [256][9][128] (k = tap*128 + c) from [256][128][3][3]
  T* w5 = (T*)(blob + L.w5);
  for (int e = tid; e < C5 * 9 * FUS_C; e += nth) {
    const int o = e / (9 * FUS_C), tap = (e / FUS_C) % 9, c = e % FUS_C;
    w5[e] = Num<T>::from_f(w.p[12][(o * FUS_C + c) * 9 + tap]);
  }
  for (int e = tid; e < C5; e += nth) ((float*)(blob + L.b5))[e] = w.p[13][e];
  if constexpr (sizeof(T) == 2) {
    bf16_t* w1s = (bf16_t*)(blob + L.w1s);
    for (int e = tid; e < STEM_C * STEM_K2; e += nth) {  // stem for chain v2: k = (c*7 + ky)*8 + kx
      const int o = e / STEM_K2, k = e % STEM_K2, grp = k / 8, kx = k % 8, c = grp / 7, ky = grp % 7;
      float v = 0.f;
      if (kx < 7) {
        const int br = o / 64, oo = o % 64, ks = 3 + 2 * br, off = 3 - ks / 2;  // 3x3 / 5x5 / 7x7
        const int y = ky - off, x = kx - off;
        if (y >= 0 && y < ks && x >= 0 && x < ks) v = w.p[2 * br][((oo * 3 + c) * ks + y) * ks + x];
      }
      w1s[e] = f32_to_bf16(v);
      ((float*)(blob + L.w1f))[e] = v;
    }
    for (int e = tid; e < FUS_C * STEM_C; e += nth) {  // f32 fusion weights in the chain order
      const int o = e / STEM_C, kk = e % STEM_C, s = kk / 32, g = (kk % 32) / 8, ee = kk % 8;
      ((float*)(blob + L.w2f))[e] = w.p[6][o * STEM_C + 32 * s + chain_perm(g, ee)];
    }
    // k_rp_conv5_v4: [half][step = quarter*3 + ky][kx][n][32 ch] (64-byte rows, chunk slot s <-
    // chunk s ^ ((n >> 1) & 2)): one step of one channel half is one linear 24 KiB copy
    bf16_t* w5q = (bf16_t*)(blob + L.w5q);
    for (int e = tid; e < C5 * 9 * FUS_C; e += nth) {
      const int k8 = e % 8, sl = (e / 8) % 4, n = (e / 32) % 128, kx = (e / 4096) % 3, st = (e / 12288) % 12,
                nh = e / 147456;
      const int qt = st / 3, ky = st % 3, c = 32 * qt + 8 * (sl ^ ((n >> 1) & 2)) + k8;
      w5q[e] = f32_to_bf16(w.p[12][((nh * 128 + n) * FUS_C + c) * 9 + ky * 3 + kx]);
    }
  }
  for (int e = tid; e < 64; e += nth) ((float*)(blob + L.zero))[e] = 0.f;
  // tail + MLP stay float32 in reference layout
  auto copy = [&](const float* src, size_t off, int n) {
    for (int e = tid; e < n; e += nth) ((float*)(blob + off))[e] = src[e];
  };
  copy(w.p[14], L.w6, C6 * C5 * 9);
  copy(w.p[15], L.b6, C6);
  copy(w.p[16], L.w7, 128 * 512);
  copy(w.p[17], L.b7, 128);
  copy(w.p[18], L.w8, 64 * 128);
  copy(w.p[19], L.b8, 64);
  copy(w.p[20], L.w9, 32 * 64);
  copy(w.p[21], L.b9, 32);
  copy(w.p[22], L.w10, 32);
  copy(w.p[23], L.b10, 1);
}

// ------------------------------------------------------------------ BN affine
// scale/shift per channel: eval from running stats; train from a stats slab [nslab][C][2]
// (sum, sum of squares), reduced in fixed order in double; running stats updated like torch.
// one 256-thread block per channel; thread i sums slab rows i, i+256, ... in double, then a
// fixed-shape tree reduction: deterministic for a given nslab.
// BatchNorm from the batch sums (s, q) = (sum, sum of squares) over `count` values (train) or the
// running stats (eval): per-channel affine, running stats updated like torch (unbiased variance)
struct BnVals {  // one channel's gamma, beta and running statistics, loaded ahead of its sums
  float g, b, rm, rv;
};
__device__ __forceinline__ BnVals bn_vals(const float* gamma, const float* beta, const float* run_mean,
                                          const float* run_var, int c) {
  return BnVals{gamma[c], beta[c], run_mean[c], run_var[c]};
}
__device__ __forceinline__ float2 bn_finish_v(double s, double q, double count, int training, float momentum,
                                              const BnVals& p, float* run_mean, float* run_var, int c,
                                              float2* __restrict__ affine) {
  float mean, var;
  if (training) {
    const double m = s / count;
    double v = q / count - m * m;
    if (v < 0.0) v = 0.0;
    mean = (float)m;
    var = (float)v;
    const double unb = count > 1.0 ? v * count / (count - 1.0) : v;
    run_mean[c] = (1.f - momentum) * p.rm + momentum * mean;
    run_var[c] = (1.f - momentum) * p.rv + momentum * (float)unb;
  } else {
    mean = p.rm;
    var = p.rv;
  }
  const float sc = p.g / sqrtf(var + BN_EPS);
  const float2 af = make_float2(sc, p.b - mean * sc);
  affine[c] = af;
  return af;
}
__device__ __forceinline__ float2 bn_finish(double s, double q, double count, int training, float momentum,
                                            const float* gamma, const float* beta, float* run_mean, float* run_var,
                                            int c, float2* __restrict__ affine) {
  return bn_finish_v(s, q, count, training, momentum, bn_vals(gamma, beta, run_mean, run_var, c), run_mean, run_var,
                     c, affine);
}
__device__ __forceinline__ double wave_sum_dbl(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// the channel's parameters load with the slab rows (thread 0), the sums reduce per wave by
// shuffles, then the four wave sums in order: one barrier instead of the eight of a tree
// slab layouts: row-major [nslab][row][2] (cm = 0), or channel-major [channel][nslab][2] (cm = 1:
// the bf16 chain's phase 1 and conv5 v4 write it, so a block's reads are contiguous; the rows are
// summed in the same order either way)
__device__ __forceinline__ void bn_affine_body(const float* __restrict__ slab, int nslab, int row, int c_off, int c,
                                               double count, int training, float momentum, const float* gamma,
                                               const float* beta, float* run_mean, float* run_var,
                                               float2* __restrict__ affine, int cm = 0) {
  __shared__ double red[2][4];
  BnVals pv{};
  if (threadIdx.x == 0) pv = bn_vals(gamma, beta, run_mean, run_var, c);
  double s = 0.0, q = 0.0;
  if (training) {
    // eight slab rows per thread in flight at once, summed in the same (row) order
    int i = threadIdx.x;
    for (; i + 256 * 7 < nslab; i += 256 * 8) {
      float2 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = *reinterpret_cast<const float2*>(
            slab + (cm ? (long long)(c_off + c) * nslab + i + 256 * u : (long long)(i + 256 * u) * row + c_off + c) * 2);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s += (double)v[u].x;
        q += (double)v[u].y;
      }
    }
    for (; i < nslab; i += 256) {
      const long long e = cm ? (long long)(c_off + c) * nslab + i : (long long)i * row + c_off + c;
      s += (double)slab[e * 2 + 0];
      q += (double)slab[e * 2 + 1];
    }
  }
  s = wave_sum_dbl(s);
  q = wave_sum_dbl(q);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s;
    red[1][threadIdx.x >> 6] = q;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  bn_finish_v(((red[0][0] + red[0][1]) + red[0][2]) + red[0][3], ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3],
              count, training, momentum, pv, run_mean, run_var, c, affine);
}
__global__ __launch_bounds__(256) void k_bn_affine(const float* __restrict__ slab, int nslab, int row, int c_off,
                                                   int C, double count, int training, float momentum,
                                                   const float* gamma, const float* beta, float* run_mean,
                                                   float* run_var, float2* __restrict__ affine, int cm = 0) {
  if ((int)blockIdx.x >= C) return;
  bn_affine_body(slab, nslab, row, c_off, blockIdx.x, count, training, momentum, gamma, beta, run_mean, run_var, affine,
                 cm);
}
// the three stem BNs (scale1/2/3, 64 channels each, concatenated :1463) in one launch
__global__ __launch_bounds__(256) void k_bn_affine_stem(const float* __restrict__ slab, int nslab, double count,
                                                        int training, float momentum, BnPtrs bn,
                                                        float2* __restrict__ affine) {
  const int l = blockIdx.x / 64, c = blockIdx.x % 64;
  bn_affine_body(slab, nslab, STEM_C, 64 * l, c, count, training, momentum, bn.p[4 * l], bn.p[4 * l + 1],
                 bn.p[4 * l + 2], bn.p[4 * l + 3], affine + 64 * l);
}

// ------------------------------------------------------------------ stem BN statistics (bf16, train)
// The three stem BatchNorms (custom_model.py:1378-1394, 1463) need, per stem channel o, the batch
// sums  sum_p y_o(p)  and  sum_p y_o(p)^2  of  y_o(p) = b_o + sum_k W_ok x_k(p),  x(p) the 7x7x3
// window of the (bf16-rounded, zero-padded) depth planes at pixel p.  Both are moments of the
// windows:  sum_p y = N b + W S1,  sum_p y^2 = N b^2 + 2 b W S1 + W S2 W^T  with
// S1_k = sum_p x_k(p) and the Gram matrix S2_kl = sum_p x_k(p) x_l(p) (147 x 147).  S2 is a lag
// sum: for k = (c1, a), l = (c2, a + L) it equals the full-image correlation
//   F(c1, c2, L) = sum_{u1, v1} X_c1(u1, v1) X_c2(u1 + Ly, v1 + Lx)       (L in [-6, 6]^2)
// minus the anchors (u1, v1) that window offset a moves outside the image (at most 3 border rows
// and 3 border columns), so the whole Gram matrix costs 1 521 correlations instead of a stem
// convolution: 9 MFMAs per 32 pixels (k_stem_lag: D[(c1,Ly)][(c2,Lx)] += X_c1(u - Ly, v)
// X_c2(u, v + Lx) over rows u and 32-pixel blocks v, bf16 products exact, f32 accumulation per
// wave, double across waves / workgroups), the border rows / columns by its trailing workgroups, and
// k_stem_s2 / k_stem_bn assemble S2, S1 and the BN affines in double.  This replaces the former
// statistics pass over the stem (126 MFMAs per 32 pixels, 181 us per bench step).
constexpr int SL_R = 32, SL_CW = 256, SL_PADL = 8;          // B rows per band, columns per chunk
constexpr int SL_ROWS = SL_R + 12, SL_LD = SL_CW + 2 * SL_PADL;
constexpr int SL_NL = 39, SL_NF = SL_NL * SL_NL;             // (channel, lag) per side; correlations
constexpr int SL_REC = SL_NF + 3;                            // + the three plane sums
constexpr size_t SL_SMEM = (size_t)3 * SL_ROWS * SL_LD * 2;
constexpr int SL_GRP = 3 * SL_ROWS * (SL_LD / 4), SL_GPT = (SL_GRP + 511) / 512;  // 4-pixel groups staged
static_assert(SL_GPT % 6 == 0, "k_stem_lag staging rounds");
static_assert(SL_SMEM >= 8 * SL_NF * sizeof(float) + 8 + 24 * sizeof(double), "k_stem_lag: LDS reused for the wave reduction");
constexpr int SF_CH = 64;                                    // stem_frame_body: pixels per chunk
constexpr int SF_T = 351, SF_REC = SF_T * 13 + 9;            // sums per (kind, image, chunk)
constexpr int SF_THR = 512;  // >= SF_T + 9 + 27: the sum threads, the plain sums, the plain corner values
constexpr int SF_AL = SF_CH + 12, SF_N = 3 * 15 * SF_AL, SF_PT = (SF_N + SF_THR - 1) / SF_THR;
static_assert(SF_THR >= SF_T + 9 + 27 && SF_THR == 512, "stem_frame_body thread roles (k_stem_lag workgroups)");
static_assert(SL_SMEM >= sizeof(float) * 3 * 15 * SF_AL, "stem_frame_body strip in k_stem_lag LDS");
constexpr int SC_REC = SF_T * 39 + 27;                       // corner cells per (row kind, side, image)

struct StemGeom {
  int nband, ncol, nwg, nfr_row, nfr_col, mx;  // lag workgroups; frame chunks per row / col kind
};
inline StemGeom stem_geom(int B, int H, int W) {
  StemGeom g;
  g.nband = ceil_div(H, SL_R);
  g.ncol = ceil_div(W, SL_CW);
  g.nwg = B * g.nband * g.ncol;
  g.nfr_row = ceil_div(W, SF_CH);
  g.nfr_col = ceil_div(H, SF_CH);
  g.mx = std::max(g.nfr_row, g.nfr_col);
  return g;
}
inline bool stem_moments_ok(int H, int W) { return H >= 8 && W >= 8; }
// The row-kind chunk that writes the right corner cells: the one holding anchor column W - 3.
// Its strip (columns a0 - 6 .. a0 + SF_CH + 5) then covers every in-image column the three
// right anchors' lag windows reach (W - 9 .. W - 1); the last chunk does not when it holds
// fewer than three columns (W % 64 in {1, 2}).
__host__ __device__ __forceinline__ int stem_right_chunk(int W) { return (W - 3) / SF_CH; }

// bf16-rounded depth value (c, y, x) of image b, 0 outside: the load always reads an in-range
// element (clamped) and the value is selected after it, so loads issued together stay in flight
__device__ __forceinline__ float stem_ld(const float* __restrict__ depth3, long long bstride, long long HW, int b, int c,
                                         int H, int W, int y, int x) {
  return depth3[b * bstride + c * HW + (long long)min(max(y, 0), H - 1) * W + min(max(x, 0), W - 1)];
}
__device__ __forceinline__ float stem_sel(float v, int H, int W, int y, int x) {
  return (y >= 0 && y < H && x >= 0 && x < W) ? bf16_to_f32(f32_to_bf16(v)) : 0.f;
}

// Border rows / columns of every image: for the anchors of the three top (bottom) rows, per
// (c1, c2, Ly) and anchor row j the 13 row sums over Lx of X_c1(u1, v) X_c2(u1 + Ly, v + Lx)
// over this chunk's 64 columns; the column kinds likewise with the roles of the axes swapped; plus
// the plain sums of X_c over the anchor rows / columns.  Workgroup = (chunk, kind, image), kind 0
// top rows, 1 bottom rows, 2 left columns, 3 right columns: out [kind][image][chunk][SF_REC] f32
// (a kind's chunks past its own count write zeros).  The row kinds' first / last chunk also write
// the corner cells of the three left / right columns: cells [row kind][side][image][SC_REC] =
// the products [t][Lx][column] and the plain values [c][row][column].
// (run by the trailing workgroups of k_stem_lag: wid = (image * 4 + kind) * mx + chunk)
__device__ __forceinline__ void stem_frame_body(const float* __restrict__ depth3, long long bstride, int B, int H, int W,
                                                int nfr_row, int nfr_col, float* __restrict__ out,
                                                float* __restrict__ cells, int wid, char* smem) {
  float(*S)[15][SF_AL] = reinterpret_cast<float(*)[15][SF_AL]>(smem);  // strip: 15 lines across, 64 + 12 along
  const int mx0 = max(nfr_row, nfr_col);
  const int chunk = wid % mx0, kind = (wid / mx0) % 4, b = wid / (4 * mx0);
  const bool rows = kind < 2;
  const int nch = rows ? nfr_row : nfr_col, mx = max(nfr_row, nfr_col);
  float* o = out + (((long long)kind * B + b) * mx + chunk) * SF_REC;
  if (chunk >= nch) {
    for (int i = threadIdx.x; i < SF_REC; i += SF_THR) o[i] = 0.f;
    return;
  }
  const long long HW = (long long)H * W;
  const int a0 = chunk * SF_CH;                                      // first anchor along the strip
  const int line0 = kind == 0 ? 0 : (kind == 1 ? H - 3 : (kind == 2 ? 0 : W - 3));  // first anchor line
  float pre[SF_PT];
#pragma unroll
  for (int k = 0; k < SF_PT; ++k) {
    const int i = min((int)threadIdx.x + SF_THR * k, SF_N - 1);
    const int c = i / (15 * SF_AL), li = (i / SF_AL) % 15, al = i % SF_AL;
    const int ln = line0 - 6 + li, at = a0 - 6 + al;                // across, along
    pre[k] = rows ? stem_ld(depth3, bstride, HW, b, c, H, W, ln, at) : stem_ld(depth3, bstride, HW, b, c, H, W, at, ln);
  }
#pragma unroll
  for (int k = 0; k < SF_PT; ++k) {
    const int i = threadIdx.x + SF_THR * k;
    if (i < SF_N) {
      const int c = i / (15 * SF_AL), li = (i / SF_AL) % 15, al = i % SF_AL;
      const int ln = line0 - 6 + li, at = a0 - 6 + al;
      S[c][li][al] = rows ? stem_sel(pre[k], H, W, ln, at) : stem_sel(pre[k], H, W, at, ln);
    }
  }
  __syncthreads();
  const int along_n = rows ? W : H;
  const int nal = min(SF_CH, along_n - a0);
  const int t = threadIdx.x;
  if (t < SF_T) {  // t = ((c1 * 3 + c2) * 13 + s1) * 3 + j: s1 the across lag, 13 along lags
    const int j = t % 3, s1 = (t / 3) % 13, c2 = (t / 39) % 3, c1 = t / 117;
    float acc[13];
#pragma unroll
    for (int q = 0; q < 13; ++q) acc[q] = 0.f;
    float win[13];
#pragma unroll
    for (int q = 0; q < 13; ++q) win[q] = S[c2][j + s1][q];  // along positions a - 6 .. a + 6 of a = 0
    for (int a = 0; a < nal; ++a) {
      const float x1 = S[c1][6 + j][6 + a];
#pragma unroll
      for (int q = 0; q < 13; ++q) acc[q] = __builtin_fmaf(x1, win[q], acc[q]);
#pragma unroll
      for (int q = 0; q < 12; ++q) win[q] = win[q + 1];
      win[12] = S[c2][j + s1][min(a + 13, SF_AL - 1)];
    }
#pragma unroll
    for (int q = 0; q < 13; ++q) o[t * 13 + q] = acc[q];
    if (rows) {  // corner cells: the three left (first chunk) / right anchor columns
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        if (chunk != (side == 0 ? 0 : stem_right_chunk(W))) continue;
        float* cl = cells + (((long long)kind * 2 + side) * B + b) * SC_REC;
#pragma unroll
        for (int ci = 0; ci < 3; ++ci) {
          const int a = side == 0 ? ci : W - 3 + ci - a0;
          const float x1 = S[c1][6 + j][6 + a];
          // strip index a + q = column a0 + a + q - 6; past the strip's end the column is >= W (0)
#pragma unroll
          for (int q = 0; q < 13; ++q) cl[(t * 13 + q) * 3 + ci] = a + q < SF_AL ? x1 * S[c2][j + s1][a + q] : 0.f;
        }
      }
    }
  } else if (t < SF_T + 9) {  // plain sums of X_c over anchor line j
    const int c = (t - SF_T) / 3, j = (t - SF_T) % 3;
    float s = 0.f;
    for (int a = 0; a < nal; ++a) s += S[c][6 + j][6 + a];
    o[SF_T * 13 + c * 3 + j] = s;
  } else if (rows && t < SF_T + 9 + 27) {  // plain corner values [c][row][column]
    const int e = t - SF_T - 9, c = e / 9, j = (e / 3) % 3, ci = e % 3;
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      if (chunk != (side == 0 ? 0 : stem_right_chunk(W))) continue;
      const int a = side == 0 ? ci : W - 3 + ci - a0;
      cells[(((long long)kind * 2 + side) * B + b) * SC_REC + SF_T * 39 + e] = S[c][6 + j][6 + a];
    }
  }
}

// Diagnostics (rgbd_debug_stem_lag_stamps, diagnostic build only): every workgroup's waves record
// s_memtime at: kernel entry, window staged (after the barrier), lag loop done, waves joined,
// correlations written, plane sums written: stamps[(wg * 8 + wave) * 6 + point].
__device__ unsigned long long* g_sl_stamps = nullptr;
[[maybe_unused]] static bool sl_stamps_on = false;
[[maybe_unused]] __device__ __forceinline__ void sl_stamp(long long idx) {
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) g_sl_stamps[idx] = t;
  __builtin_amdgcn_sched_barrier(0);
}

// grid: the nwg lag workgroups, then 4 * B * mx border workgroups (stem_frame_body), which fill
// the CU slots the lag workgroups leave free instead of following them in a second launch
template <bool STAMPS = false>
__global__ __launch_bounds__(512) void k_stem_lag(const float* __restrict__ depth3, long long bstride, int B, int H,
                                                  int W, int nband, int ncol, double* __restrict__ part, int nfr_row,
                                                  int nfr_col, float* __restrict__ fch, float* __restrict__ cells) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if ((int)blockIdx.x >= B * nband * ncol) {
    stem_frame_body(depth3, bstride, B, H, W, nfr_row, nfr_col, fch, cells, (int)blockIdx.x - B * nband * ncol, smem);
    return;
  }
  const long long sbase = ((long long)blockIdx.x * 8 + (threadIdx.x >> 6)) * 6;
  if constexpr (STAMPS) sl_stamp(sbase + 0);
  bf16_t* X = (bf16_t*)smem;  // [3][SL_ROWS][SL_LD]: rows u0-6 .., columns cv0-8 ..
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int wg = blockIdx.x, b = wg / (nband * ncol), rem = wg % (nband * ncol);
  const int u0 = (rem / ncol) * SL_R, cv0 = (rem % ncol) * SL_CW;
  const long long HW = (long long)H * W;
  float tsum[3] = {0.f, 0.f, 0.f};
  // the 4-pixel groups in rounds of SL_RND: a round's loads are issued together, then converted
  // (16-byte loads where rows are aligned: the groups then never straddle the image's right edge)
  const bool vec = (W & 3) == 0 && (bstride & 3) == 0 && ((uintptr_t)depth3 & 15) == 0;
  auto put = [&](int i, float4 q) {
    const int c = i / (SL_ROWS * (SL_LD / 4)), rr = (i / (SL_LD / 4)) % SL_ROWS, cc = 4 * (i % (SL_LD / 4));
    const int yy = u0 - 6 + rr, xx = cv0 - SL_PADL + cc;
    const float v0 = stem_sel(q.x, H, W, yy, xx), v1 = stem_sel(q.y, H, W, yy, xx + 1);
    const float v2 = stem_sel(q.z, H, W, yy, xx + 2), v3 = stem_sel(q.w, H, W, yy, xx + 3);
    *reinterpret_cast<uint2*>(X + (c * SL_ROWS + rr) * SL_LD + cc) = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
    // the plane sums over this workgroup's own pixels (rows [u0, u0+R), columns [cv0, cv0+CW))
    if (rr >= 6 && rr < 6 + SL_R && cc >= SL_PADL && cc < SL_PADL + SL_CW) tsum[c] += (v0 + v1) + (v2 + v3);
  };
  constexpr int SL_RND = 6;
  for (int k0 = 0; k0 < SL_GPT; k0 += SL_RND) {
    float4 q[SL_RND];
    if (vec) {
#pragma unroll
      for (int k = 0; k < SL_RND; ++k) {
        const int i = min(tid + 512 * (k0 + k), SL_GRP - 1);
        const int c = i / (SL_ROWS * (SL_LD / 4)), rr = (i / (SL_LD / 4)) % SL_ROWS, cc = 4 * (i % (SL_LD / 4));
        const int yy = u0 - 6 + rr, xx = cv0 - SL_PADL + cc;
        q[k] = *reinterpret_cast<const float4*>(depth3 + b * bstride + c * HW + (long long)min(max(yy, 0), H - 1) * W +
                                                min(max(xx, 0), W - 4));
      }
    } else {
#pragma unroll
      for (int k = 0; k < SL_RND; ++k) {
        const int i = min(tid + 512 * (k0 + k), SL_GRP - 1);
        const int c = i / (SL_ROWS * (SL_LD / 4)), rr = (i / (SL_LD / 4)) % SL_ROWS, cc = 4 * (i % (SL_LD / 4));
        const int yy = u0 - 6 + rr, xx = cv0 - SL_PADL + cc;
        q[k] = make_float4(stem_ld(depth3, bstride, HW, b, c, H, W, yy, xx),
                           stem_ld(depth3, bstride, HW, b, c, H, W, yy, xx + 1),
                           stem_ld(depth3, bstride, HW, b, c, H, W, yy, xx + 2),
                           stem_ld(depth3, bstride, HW, b, c, H, W, yy, xx + 3));
      }
    }
#pragma unroll
    for (int k = 0; k < SL_RND; ++k) {
      const int i = tid + 512 * (k0 + k);
      if (i < SL_GRP) put(i, q[k]);
    }
  }
  __syncthreads();
  if constexpr (STAMPS) sl_stamp(sbase + 1);
  // per-lane fragment bases: A rows m = (c1, Ly), B columns n = (c2, Lx); m, n >= 39 are zero
  int abase[3], bbase[3];
  bool aval[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int m = 16 * i + r;
    aval[i] = m < SL_NL;
    const int c1 = aval[i] ? m / 13 : 0, ly = aval[i] ? m % 13 - 6 : 0;
    abase[i] = (c1 * SL_ROWS + 6 - ly) * SL_LD + SL_PADL + 8 * g;     // + ur * SL_LD + (v0 - cv0)
    bbase[i] = (c1 * SL_ROWS + 6) * SL_LD + SL_PADL + 8 * g + ly;     // (c2, Lx) decode as (c1, ly)
  }
  f32x4 acc[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nrow = min(SL_R, H - u0), nvb = (min(SL_CW, W - cv0) + 31) / 32;
  const uint32_t* Xw = reinterpret_cast<const uint32_t*>(X);
  for (int it = wave; it < nrow * nvb; it += 8) {
    const int ur = it / nvb, off = ur * SL_LD + 32 * (it % nvb);
    Frag<bf16_t> fa[3], fb[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      fa[i].v = *reinterpret_cast<const uint4*>(X + abase[i] + off);
      if (!aval[i]) fa[i].zero();
      const int e = bbase[i] + off, w0 = e >> 1;
      const uint32_t sh = (e & 1) * 2;
      const uint32_t x0 = Xw[w0], x1 = Xw[w0 + 1], x2 = Xw[w0 + 2], x3 = Xw[w0 + 3], x4 = Xw[w0 + 4];
      fb[i].v = make_uint4(__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                           __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh));
      if (!aval[i]) fb[i].zero();
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) mma(acc[i][j], fa[i], fb[j]);
  }
  if constexpr (STAMPS) sl_stamp(sbase + 2);
  // the 8 waves' tiles summed in double, in wave order: every wave parks its f32 tile in LDS
  // (8 x 1 521 floats), then each correlation is summed by one thread
  __syncthreads();
  if constexpr (STAMPS) sl_stamp(sbase + 3);
  float* redf = (float*)smem;  // [8 wave][SL_NF]
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = 16 * i + 4 * g + e, n = 16 * j + r;
        if (m < SL_NL && n < SL_NL) redf[wave * SL_NF + m * SL_NL + n] = acc[i][j][e];
      }
  // plane sums: per wave in double (lane order fixed by the butterfly), parked after the tiles
  double* wsum = (double*)(smem + 8 * SL_NF * sizeof(float) + 8);  // [8 wave][3], 8-byte aligned
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double v = (double)tsum[c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) wsum[wave * 3 + c] = v;
  }
  __syncthreads();
  double* out = part + (long long)wg * SL_REC;
  for (int i = tid; i < SL_NF; i += 512) {
    double t = (double)redf[i];
#pragma unroll
    for (int w = 1; w < 8; ++w) t += (double)redf[w * SL_NF + i];
    out[i] = t;
  }
  if (tid < 3) {
    double t = wsum[tid];
#pragma unroll
    for (int w = 1; w < 8; ++w) t += wsum[w * 3 + tid];
    out[SL_NF + tid] = t;
  }
  if constexpr (STAMPS) sl_stamp(sbase + 4);
  if constexpr (STAMPS) sl_stamp(sbase + 5);
}

// dst[s][e] = sum_k src[s * seg_stride + k * stride + e] (k < n, fixed order: 16 groups of every
// 16th k, then the groups in order): workgroup = 16 consecutive elements x 16 groups.
template <typename T>
__device__ __forceinline__ void stem_sum_body(const T* __restrict__ src, int n, long long stride, long long seg_stride,
                                              int seg_len, double* __restrict__ dst, int bx, int s,
                                              double (*red)[17]) {
  const int el = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int e = bx * 16 + el;
  double acc = 0.0;
  if (e < seg_len) {
    const T* p = src + s * seg_stride + e;
    int k = grp;
    for (; k + 112 < n; k += 128) {  // eight loads in flight, added in k order
      double a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = (double)p[(k + 16 * u) * stride];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += a[u];
    }
    for (; k < n; k += 16) acc += (double)p[k * stride];
  }
  red[grp][el] = acc;
  __syncthreads();
  if (grp == 0 && e < seg_len) {
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][el];
    dst[(long long)s * seg_len + e] = t;
  }
}

// The three reductions of the stem moments in one launch (1-D grid): the lag partials -> F
// (double), the border chunks -> fr [kind] and the corner cells -> ce [row kind][side] (float).
struct StemSums {
  const double* part;
  const float *fch, *cells;
  double *F, *fr, *ce;
  int nwg, nfch, B;
};
constexpr int SS_B0 = (SL_REC + 15) / 16, SS_B1 = 4 * ((SF_REC + 15) / 16), SS_B2 = 4 * ((SC_REC + 15) / 16);
__global__ __launch_bounds__(256) void k_stem_sums(const StemSums a) {
  __shared__ double red[16][17];
  int bx = blockIdx.x;
  if (bx < SS_B0) {
    stem_sum_body<double>(a.part, a.nwg, SL_REC, 0, SL_REC, a.F, bx, 0, red);
    return;
  }
  bx -= SS_B0;
  if (bx < SS_B1) {
    const int per = SS_B1 / 4;
    stem_sum_body<float>(a.fch, a.nfch, SF_REC, (long long)a.nfch * SF_REC, SF_REC, a.fr, bx % per, bx / per, red);
    return;
  }
  bx -= SS_B1;
  const int per = SS_B2 / 4;
  stem_sum_body<float>(a.cells, a.B, SC_REC, (long long)a.B * SC_REC, SC_REC, a.ce, bx % per, bx / per, red);
}

// S2 [147][147] and S1 [147] (k = c * 49 + ay * 7 + ax, the window offset a = (ay, ax) of
// channel c) over the batch, double: thread per (k, l), the extra 147 threads S1.  fr [kind][SF_REC]
// and ce [row kind][side][SC_REC] are already summed over the images.
__global__ __launch_bounds__(256) void k_stem_s2(const double* __restrict__ F, const double* __restrict__ fr,
                                                 const double* __restrict__ ce, double* __restrict__ S2,
                                                 double* __restrict__ S1) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= 147 * 147 + 147) return;
  const bool is_s1 = i >= 147 * 147;
  const int k = is_s1 ? i - 147 * 147 : i / 147, l = is_s1 ? k : i % 147;
  const int c1 = k / 49, ay = (k % 49) / 7, ax = k % 7;
  const int c2 = l / 49, by = (l % 49) / 7, bx = l % 7;
  const int ly = by - ay, lx = bx - ax;
  // excluded anchor rows / columns of offset a: top j < ay - 3, or bottom j >= ay (j = 0..2)
  const int rkind = ay > 3 ? 0 : 1, rlo = ay > 3 ? 0 : ay, rhi = ay > 3 ? ay - 3 : (ay < 3 ? 3 : 0);
  const int ckind = ax > 3 ? 2 : 3, clo = ax > 3 ? 0 : ax, chi = ax > 3 ? ax - 3 : (ax < 3 ? 3 : 0);
  const double* rk = fr + (long long)rkind * SF_REC;
  const double* ck = fr + (long long)ckind * SF_REC;
  const double* cc = ce + ((long long)rkind * 2 + (ckind - 2)) * SC_REC;
  const int trow = ((c1 * 3 + c2) * 13 + ly + 6) * 3, tcol = ((c1 * 3 + c2) * 13 + lx + 6) * 3;
  // every load in flight together (j = 0..2 index valid rows whatever the bounds; the loops over
  // the data-dependent bounds waited for each load in turn), applied in the same order as before
  double s = is_s1 ? F[SL_NF + c1] : F[(c1 * 13 + ly + 6) * SL_NL + c2 * 13 + lx + 6];
  double rv[3], cv[3], xv[3][3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    rv[j] = is_s1 ? rk[SF_T * 13 + c1 * 3 + j] : rk[(trow + j) * 13 + lx + 6];
    cv[j] = is_s1 ? ck[SF_T * 13 + c1 * 3 + j] : ck[(tcol + j) * 13 + ly + 6];
#pragma unroll
    for (int jc = 0; jc < 3; ++jc)
      xv[j][jc] = is_s1 ? cc[SF_T * 39 + (c1 * 3 + j) * 3 + jc] : cc[((trow + j) * 13 + lx + 6) * 3 + jc];
  }
#pragma unroll
  for (int j = 0; j < 3; ++j)
    if (j >= rlo && j < rhi) s -= rv[j];
#pragma unroll
  for (int j = 0; j < 3; ++j)
    if (j >= clo && j < chi) s -= cv[j];
#pragma unroll
  for (int jr = 0; jr < 3; ++jr)  // corners: excluded in both, subtracted twice
#pragma unroll
    for (int jc = 0; jc < 3; ++jc)
      if (jr >= rlo && jr < rhi && jc >= clo && jc < chi) s += xv[jr][jc];
  if (is_s1)
    S1[k] = s;
  else
    S2[i] = s;
}

// fold: [W1' 192 x 168 bf16][W2' 128 x 192 bf16][b1' 192 f32][b2' 128 f32] (BN folding below)
constexpr size_t FOLD_W1 = 0, FOLD_W2 = FOLD_W1 + (size_t)STEM_C * STEM_K2 * 2;
constexpr size_t FOLD_B1 = FOLD_W2 + (size_t)FUS_C * STEM_C * 2, FOLD_B2 = FOLD_B1 + STEM_C * 4;
constexpr size_t FOLD_BYTES = FOLD_B2 + FUS_C * 4;

// Per stem channel o (one block each): sum y = N b + w.S1, sum y^2 = N b^2 + 2 b w.S1 + w S2 w^T,
// then the BatchNorm of bn_affine_body (train mode) from the double sums, and the block folds
// its affine into W1' / b1' row o as k_rp_fold (which 1) does.  Blocks STEM_C .. STEM_C + 32 B - 1
// zero conv5 v4's input padding (k_c4_pad_zero's work: grid (8, 4 B) flattened), so neither
// small kernel is a launch of its own on the predictor's critical path.
__device__ void c4_pad_body(bf16_t* __restrict__ att, int H, int W, int bx, int plane, int nbx);
__global__ __launch_bounds__(256) void k_stem_bn(const double* __restrict__ S2, const double* __restrict__ S1,
                                                 const char* __restrict__ blob, Layout L, double count, float momentum,
                                                 BnPtrs bn, float2* __restrict__ affine, char* __restrict__ fold,
                                                 bf16_t* __restrict__ att, int H, int W) {
  if ((int)blockIdx.x >= STEM_C) {  // block-uniform
    const int p = (int)blockIdx.x - STEM_C;
    c4_pad_body(att, H, W, p % 8, p / 8, 8);
    return;
  }
  __shared__ double red[2][256];
  __shared__ double w[147];
  __shared__ float2 s_aff;
  const int o = blockIdx.x, t = threadIdx.x;
  const bf16_t* w1s = (const bf16_t*)(blob + L.w1s);
  // the fold's source row, loaded now (in flight through the reduction)
  const float wf = t < STEM_K2 ? ((const float*)(blob + L.w1f))[(size_t)o * STEM_K2 + t] : 0.f;
  const float bf = ((const float*)(blob + L.b1))[o];
  if (t < 147) w[t] = (double)bf16_to_f32(w1s[o * STEM_K2 + ((t / 49) * 7 + (t % 49) / 7) * 8 + t % 7]);
  __syncthreads();
  double a = 0.0, q = 0.0;
  if (t < 147) {
    a = w[t] * S1[t];
    // S2 symmetric: coalesced rows.  49 rows per batch in flight together, summed in row order
    // (seven loads per round trip made the 147 serial L2 round trips most of the kernel)
    for (int l0 = 0; l0 < 147; l0 += 49) {
      double sv[49];
#pragma unroll
      for (int u = 0; u < 49; ++u) sv[u] = S2[(l0 + u) * 147 + t];
#pragma unroll
      for (int u = 0; u < 49; ++u) q += w[l0 + u] * sv[u];
    }
    q *= w[t];
  }
  red[0][t] = a;
  red[1][t] = q;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) {
      red[0][t] += red[0][t + s];
      red[1][t] += red[1][t + s];
    }
    __syncthreads();
  }
  if (t == 0) {
    const double bias = (double)bf;
    const double sy = count * bias + red[0][0];
    const double sq = count * bias * bias + 2.0 * bias * red[0][0] + red[1][0];
    const int l = o / 64, c = o % 64;
    s_aff = bn_finish(sy, sq, count, 1, momentum, bn.p[4 * l], bn.p[4 * l + 1], bn.p[4 * l + 2], bn.p[4 * l + 3], c,
                      affine + 64 * l);
  }
  __syncthreads();
  // BN1 -> W1', b1' (k_rp_fold's arithmetic)
  const float2 af = s_aff;
  if (t < STEM_K2) ((bf16_t*)(fold + FOLD_W1))[(size_t)o * STEM_K2 + t] = f32_to_bf16(wf * af.x);
  if (t == 0) ((float*)(fold + FOLD_B1))[o] = __builtin_fmaf(bf, af.x, af.y);
}

struct StemWs {
  size_t part, fchunks, cells, F, fr, ce, S2, S1, total;
};
inline StemWs stem_ws(int B, int H, int W) {
  const StemGeom g = stem_geom(B, H, W);
  StemWs s;
  size_t o = 0;
  auto seg = [&](size_t bytes) {
    size_t r = o;
    o += align256(bytes);
    return r;
  };
  s.part = seg((size_t)g.nwg * SL_REC * sizeof(double));
  s.fchunks = seg((size_t)4 * B * g.mx * SF_REC * sizeof(float));
  s.cells = seg((size_t)4 * B * SC_REC * sizeof(float));
  s.F = seg(SL_REC * sizeof(double));
  s.fr = seg((size_t)4 * SF_REC * sizeof(double));
  s.ce = seg((size_t)4 * SC_REC * sizeof(double));
  s.S2 = seg(147 * 147 * sizeof(double));
  s.S1 = seg(147 * sizeof(double));
  s.total = o;
  return s;
}

// the moments of every window and the stem BN affines (aff1) + running stats, train mode
int stem_bn_moments(const float* depth3, long long bstride, int B, int H, int W, const char* blob, const Layout& L,
                    float momentum, const BnPtrs& bn, float2* aff1, char* fold, bf16_t* att, char* ws, hipStream_t s) {
  const StemGeom g = stem_geom(B, H, W);
  const StemWs w = stem_ws(B, H, W);
  double* part = (double*)(ws + w.part);
  float* fch = (float*)(ws + w.fchunks);
  float* cells = (float*)(ws + w.cells);
  double* F = (double*)(ws + w.F);
  double* fr = (double*)(ws + w.fr);
  double* ce = (double*)(ws + w.ce);
  double* S2 = (double*)(ws + w.S2);
  double* S1 = (double*)(ws + w.S1);
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)k_stem_lag<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)SL_SMEM);
  if (attr != hipSuccess) return (int)attr;
  const int nall = g.nwg + 4 * B * g.mx;
#ifdef RGBD_DIAG
  if (sl_stamps_on) {
    static const hipError_t dattr =
        hipFuncSetAttribute((const void*)k_stem_lag<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)SL_SMEM);
    (void)dattr;
    k_stem_lag<true><<<nall, 512, SL_SMEM, s>>>(depth3, bstride, B, H, W, g.nband, g.ncol, part, g.nfr_row, g.nfr_col,
                                               fch, cells);
  } else
#endif
    k_stem_lag<false><<<nall, 512, SL_SMEM, s>>>(depth3, bstride, B, H, W, g.nband, g.ncol, part, g.nfr_row,
                                                g.nfr_col, fch, cells);
  StemSums ss{part, fch, cells, F, fr, ce, g.nwg, B * g.mx, B};
  k_stem_sums<<<SS_B0 + SS_B1 + SS_B2, 256, 0, s>>>(ss);
  k_stem_s2<<<ceil_div(147 * 147 + 147, 256), 256, 0, s>>>(F, fr, ce, S2, S1);
  k_stem_bn<<<STEM_C + 32 * B, 256, 0, s>>>(S2, S1, blob, L, (double)B * H * W, momentum, bn, aff1, fold, att, H, W);
  return RGBD_OK;
}

// ------------------------------------------------------------------ chain (stem, fusion, attention)
constexpr int CH_TW = 16, CH_TH = 4;                    // tile: 4 rows x 16 cols, one row per wave
constexpr int PATCH_H = CH_TH + 6, PATCH_W = CH_TW + 6;  // 7x7 halo

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
// bf16 path: v_exp_f32 + v_rcp_f32 (~1 ulp each; the result is rounded to bf16).  The bf16 chain
// also writes its BN affines and statistics with explicit fmaf (the file builds with
// -ffp-contract=off for the bit-exact paths, which would split them into v_mul + v_add).
__device__ __forceinline__ float sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}

template <typename T>
__device__ __forceinline__ Frag<T> load_w(const T* base, int row, int K, int s, int g) {
  Frag<T> f;
  f.load(base + (long long)row * K + 32 * s + 8 * g);
  return f;
}

// PHASE 0: stem stats; 1: fusion stats; 2: write gated attention features (NHWC)
template <typename T, int PHASE>
__global__ __launch_bounds__(256) void k_rp_chain(const float* __restrict__ depth3, long long bstride, int B,
                                                  int H, int W, const char* __restrict__ blob, Layout L,
                                                  const float2* __restrict__ aff1, const float2* __restrict__ aff2,
                                                  float* __restrict__ slab, T* __restrict__ att) {
  __shared__ float patch[3][PATCH_H][PATCH_W];
  __shared__ short ktab[STEM_K];  // k -> (c, ky, kx) offset into patch, -1 for the zero pad
  __shared__ float st[4][STEM_C][2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  constexpr int NST = PHASE == 0 ? STEM_C : FUS_C;
  for (int k = threadIdx.x; k < STEM_K; k += 256) {
    short v = -1;
    if (k < 147) {
      const int tap = k / 3, c = k % 3;
      v = (short)((c * PATCH_H + tap / 7) * PATCH_W + tap % 7);
    }
    ktab[k] = v;
  }
  for (int i = threadIdx.x; i < 4 * STEM_C * 2; i += 256) (&st[0][0][0])[i] = 0.f;
  const int tiles_x = (W + CH_TW - 1) / CH_TW, tiles_y = (H + CH_TH - 1) / CH_TH;
  const long long ntiles = (long long)B * tiles_x * tiles_y;
  const long long HW = (long long)H * W;
  for (long long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int b = (int)(tile / ((long long)tiles_x * tiles_y));
    const int trem = (int)(tile % ((long long)tiles_x * tiles_y));
    const int y0 = (trem / tiles_x) * CH_TH, x0 = (trem % tiles_x) * CH_TW;
    __syncthreads();
    for (int i = threadIdx.x; i < 3 * PATCH_H * PATCH_W; i += 256) {
      const int c = i / (PATCH_H * PATCH_W), yy = (i / PATCH_W) % PATCH_H, xx = i % PATCH_W;
      const int y = y0 + yy - 3, x = x0 + xx - 3;
      (&patch[0][0][0])[i] =
          (y >= 0 && y < H && x >= 0 && x < W) ? depth3[b * bstride + c * HW + (long long)y * W + x] : 0.f;
    }
    __syncthreads();
    const int py = y0 + wave, px = x0 + r;
    const bool pvalid = py < H && px < W;
    const char* bl = opaque(blob);  // re-derived per tile: no LICM of the weight loads
    const T* w1 = (const T*)(bl + L.w1);
    const T* w2 = (const T*)(bl + L.w2);
    const T* w3 = (const T*)(bl + L.w3);
    const T* w4 = (const T*)(bl + L.w4);
    const float* b1 = (const float*)(bl + L.b1);
    const float* b2 = (const float*)(bl + L.b2);
    const float* b3 = (const float*)(bl + L.b3);
    const float* b4 = (const float*)(bl + L.b4);
    const float2* af1 = opaque(aff1);
    const float2* af2 = opaque(aff2);
    // ---- stem: D1[192 ch][16 px]
    f32x4 a1[12];
#pragma unroll
    for (int t = 0; t < 12; ++t) a1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      Frag<T> bfr;
      {
        float vv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int off = ktab[32 * s + 8 * g + e];
          vv[e] = off >= 0 ? (&patch[0][0][0])[off + wave * PATCH_W + r] : 0.f;
        }
        bfr.from8(vv);
      }
#pragma unroll
      for (int t = 0; t < 12; ++t) {
        // the 3x3 / 5x5 branches have all-zero weights outside k in [48,99) / [24,123)
        if (t < 4 && (s == 0 || s == 4)) continue;
        if (t >= 4 && t < 8 && s == 4) continue;
        mma(a1[t], load_w(w1, 16 * t + r, STEM_K, s, g), bfr);
        __builtin_amdgcn_sched_barrier(0);  // keep weight loads from being hoisted (VGPR budget)
      }
    }
    // z1 = a1 + b1 ; stats or BN+ReLU -> chained operand
#pragma unroll
    for (int t = 0; t < 12; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) a1[t][j] += b1[16 * t + 4 * g + j];
    if constexpr (PHASE == 0) {
#pragma unroll
      for (int t = 0; t < 12; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = pvalid ? a1[t][j] : 0.f, q = v * v;
          for (int o = 1; o < 16; o <<= 1) {
            v += __shfl_xor(v, o);
            q += __shfl_xor(q, o);
          }
          if (r == 0) {
            st[wave][16 * t + 4 * g + j][0] += v;
            st[wave][16 * t + 4 * g + j][1] += q;
          }
        }
      continue;
    }
    Frag<T> f1[6];
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      float vv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int t = 2 * s + (e >> 2), j = e & 3, ch = 16 * t + 4 * g + j;
        const float2 af = af1[ch];
        vv[e] = fmaxf(a1[t][j] * af.x + af.y, 0.f);
      }
      f1[s].from8(vv);
    }
    // ---- fusion: D2[128][16 px]
    f32x4 a2[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      a2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 6; ++s) mma(a2[t], load_w(w2, 16 * t + r, STEM_C, s, g), f1[s]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; ++j) a2[t][j] += b2[16 * t + 4 * g + j];
    }
    if constexpr (PHASE == 1) {
#pragma unroll
      for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = pvalid ? a2[t][j] : 0.f, q = v * v;
          for (int o = 1; o < 16; o <<= 1) {
            v += __shfl_xor(v, o);
            q += __shfl_xor(q, o);
          }
          if (r == 0) {
            st[wave][16 * t + 4 * g + j][0] += v;
            st[wave][16 * t + 4 * g + j][1] += q;
          }
        }
      continue;
    }
    if constexpr (PHASE == 2) {
#pragma unroll
      for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float2 af = af2[16 * t + 4 * g + j];
          a2[t][j] = fmaxf(a2[t][j] * af.x + af.y, 0.f);  // fused = ReLU(BN(z2))
        }
      Frag<T> f2[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        float vv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) vv[e] = a2[2 * s + (e >> 2)][e & 3];
        f2[s].from8(vv);
      }
      // ---- attention 1: D3[64][16 px], ReLU
      f32x4 a3[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        a3[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) mma(a3[t], load_w(w3, 16 * t + r, FUS_C, s, g), f2[s]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 4; ++j) a3[t][j] = fmaxf(a3[t][j] + b3[16 * t + 4 * g + j], 0.f);
      }
      Frag<T> f3[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float vv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) vv[e] = a3[2 * s + (e >> 2)][e & 3];
        f3[s].from8(vv);
      }
      // ---- attention 2 + sigmoid gate, store NHWC
      T* orow = att + ((long long)b * HW + (long long)py * W + px) * FUS_C;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        f32x4 a4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 2; ++s) mma(a4, load_w(w4, 16 * t + r, ATT_C, s, g), f3[s]);
        __builtin_amdgcn_sched_barrier(0);
        if (pvalid) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int ch = 16 * t + 4 * g + j;
            orow[ch] = Num<T>::from_f(a2[t][j] * sigmoidf_(a4[j] + b4[ch]));
          }
        }
      }
    }
  }
  if constexpr (PHASE < 2) {
    __syncthreads();
    for (int c = threadIdx.x; c < NST; c += 256)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        slab[((long long)blockIdx.x * NST + c) * 2 + q] = ((st[0][c][q] + st[1][c][q]) + st[2][c][q]) + st[3][c][q];
  }
}

// Butterfly reduce-scatter of N per-lane values over the 16 lanes sharing lane>>4: after the
// call, v[i] (i < N/16) of lane r holds the 16-lane sum of original value
// (r&1)N/2 + ((r>>1)&1)N/4 + ((r>>2)&1)N/8 + ((r>>3)&1)N/16 + i.
template <int N>
__device__ __forceinline__ void reduce_scatter16(float (&v)[N], int r) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int n = N >> k, half = n >> 1;
    const bool hi = (r >> k) & 1;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const float a = v[i], b = v[i + half];
      const float keep = hi ? b : a, send = hi ? a : b;
      v[i] = keep + __shfl_xor(send, 1 << k);
    }
  }
}

// ------------------------------------------------------------------ BN folding (bf16 chain)
// Once the statistics of a BN layer are known, fold its affine (sc, sh) into the producing
// layer: W' = bf16(sc * W_f32) row-wise, b' = sc * b + sh, so the chain applies only the ReLU.
// (fold layout: FOLD_W1 .. FOLD_BYTES above)  which = 1 | 2.
__global__ __launch_bounds__(256) void k_rp_fold(const char* __restrict__ blob, Layout L,
                                                 const float2* __restrict__ aff, int which, char* __restrict__ fold) {
  const int c = blockIdx.x;
  const int K = which == 1 ? STEM_K2 : STEM_C;
  const float* w = (const float*)(blob + (which == 1 ? L.w1f : L.w2f)) + (size_t)c * K;
  bf16_t* wo = (bf16_t*)(fold + (which == 1 ? FOLD_W1 : FOLD_W2)) + (size_t)c * K;
  const float2 a = aff[c];
  for (int k = threadIdx.x; k < K; k += 256) wo[k] = f32_to_bf16(w[k] * a.x);
  if (threadIdx.x == 0) {
    const float b = ((const float*)(blob + (which == 1 ? L.b1 : L.b2)))[c];
    ((float*)(fold + (which == 1 ? FOLD_B1 : FOLD_B2)))[c] = __builtin_fmaf(b, a.x, a.y);
  }
}

// tile index -> (image, first row, first column) with 32-bit unsigned divisions (the 64-bit
// ones cost ~150 scalar instructions per decode, twice per tile in the chain kernels)
struct TileDec {
  int b, y0, x0;
};
__device__ __forceinline__ TileDec tile_dec(unsigned t, unsigned per, unsigned tiles_x, int th, int tw) {
  const unsigned b = t / per, rem = t - b * per, ty = rem / tiles_x;
  return TileDec{(int)b, (int)ty * th, (int)(rem - ty * tiles_x) * tw};
}

// ------------------------------------------------------------------ chain v2 (bf16)
// 512 threads = 8 waves; persistent; ALL chain weights (143 KB bf16) live in LDS for the
// workgroup's lifetime; a wave owns 32 pixels (one row of a 8x32 tile, two 16-px MFMA
// columns) so every weight fragment read from LDS feeds two MFMAs.  BN statistics (phases
// 0/1) are reduced across the wave's 32 pixels and kept per lane in registers, then written
// as one slab row per wave: deterministic.
constexpr int C2W_TH = 8, C2W_TW = 32, C2W_PH = C2W_TH + 6, C2W_PW = C2W_TW + 6;
// LDS weight rows padded by 16 bytes: W1's 352-B rows are conflict-free for the ds_read_b128
// lane groups; W2/W3/W4 (400/272/144 B) are 2-way (conflict-free strides or chunk swizzles do
// not fit the LDS budget / cost more in per-lane offsets and spills than they save, measured).
constexpr int C2W_S1 = STEM_K2 + 8, C2W_S2 = STEM_C + 8, C2W_S3 = FUS_C + 8, C2W_S4 = ATT_C + 8;
constexpr int C2W_PWP = 40;  // bf16 patch row: 38 pixels + 2 zero pad (a lane reads 5 words from col & ~1)
constexpr size_t C2W_OFF_W1 = 0;
constexpr size_t C2W_OFF_W2 = C2W_OFF_W1 + (size_t)STEM_C * C2W_S1 * 2;
constexpr size_t C2W_OFF_W3 = C2W_OFF_W2 + (size_t)FUS_C * C2W_S2 * 2;
constexpr size_t C2W_OFF_W4 = C2W_OFF_W3 + (size_t)ATT_C * C2W_S3 * 2;
// Phase 0 (stem statistics) keeps only W1 resident: ~76 KB, two workgroups per CU.
template <int PH> constexpr size_t c2w_off_b() {  // b1 b2 b3 b4 (f32)
  return PH == 0 ? C2W_OFF_W2 : C2W_OFF_W4 + (size_t)FUS_C * C2W_S4 * 2;
}
template <int PH> constexpr size_t c2w_off_aff() {  // aff1, aff2
  return c2w_off_b<PH>() + (size_t)(STEM_C + FUS_C + ATT_C + FUS_C) * 4;
}
template <int PH> constexpr size_t c2w_off_patch() {  // bf16 [3][14][40]
  return c2w_off_aff<PH>() + (size_t)(STEM_C + FUS_C) * 8;
}
template <int PH> constexpr size_t c2w_smem() { return c2w_off_patch<PH>() + (size_t)3 * C2W_PH * C2W_PWP * 2 + 16; }
static_assert(c2w_smem<1>() <= 163840, "chain v2 LDS budget");
// Phase 1 (train: stem + fusion + fusion statistics) needs neither W3 nor W4: their space holds
// eight copies of the depth patch shifted by 0..7 columns, [shift k][3][14][40] with element j of
// copy k = patch column j + k, so the 8 patch values a lane feeds the stem (columns col .. col+7)
// are ONE 16-byte-aligned ds_read_b128 from copy col % 8 (the other phases: 5 dword reads and 4
// byte-aligns per fragment)
constexpr size_t C2W_OFF_P8 = C2W_OFF_W3;
constexpr int C2W_P8 = 8 * 3 * C2W_PH * C2W_PWP;  // bf16 elements
static_assert(C2W_OFF_P8 + (size_t)C2W_P8 * 2 <= c2w_off_b<1>(), "phase-1 shifted patches fit W3 + W4");
static_assert(2 * c2w_smem<0>() <= 163840, "chain v2 phase 0: two workgroups per CU");

// Diagnostics (rgbd_debug_chain_stamps): the STAMPS instantiation records, for workgroup 0's tiles
// 8-11, s_memtime per wave at: tile top, patch staged (after the second barrier), next
// patch's loads issued, stem MFMAs issued (phase 0: statistics done), stem ReLU/pack done, fusion
// MFMAs issued, tile end (statistics + stores): stamps[((phase * 4 + tile) * 8 + wave) * 7 + point].
__device__ unsigned long long* g_c2_stamps = nullptr;
// the stamped instantiations exist only in the diagnostic build (make diag); in the product
// library the stamps branch below launches the production kernel and is never taken
#ifdef RGBD_DIAG
constexpr bool RGBD_DIAG_ON = true;
#else
constexpr bool RGBD_DIAG_ON = false;
#endif
static bool c2_stamps_on = false;
__device__ __forceinline__ void c2_stamp(unsigned long long* st, long long idx) {
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) st[idx] = t;
  __builtin_amdgcn_sched_barrier(0);
}

// conv5 v4's input (bf16): channel-quarter-major, zero-padded planes [B][4][PH][PW][32]: pixel
// (y, x) at plane row y + 1, column x + 1, PH / PW = the 16x32 tile grid + a one-pixel border, so
// every halo read of every tile is in bounds and reads zeros outside the image.
__host__ __device__ __forceinline__ int c4_ph(int H) { return (H + 15) / 16 * 16 + 2; }
__host__ __device__ __forceinline__ int c4_pw(int W) { return (W + 31) / 32 * 32 + 2; }
__host__ __device__ __forceinline__ long long c4_att_idx(int b, int q, int y, int x, int H, int W) {
  return (((long long)b * 4 + q) * c4_ph(H) + y + 1) * c4_pw(W) * 32 + (long long)(x + 1) * 32;
}

template <int PHASE, bool STAMPS = false>
__global__ __launch_bounds__(512, PHASE == 0 ? 4 : 2) void k_rp_chain_v2(const float* __restrict__ depth3, long long bstride, int B,
                                                     int H, int W, const char* __restrict__ blob, Layout L,
                                                     const float2* __restrict__ aff1, const float2* __restrict__ aff2,
                                                     const char* __restrict__ fold, float* __restrict__ slab,
                                                     bf16_t* __restrict__ att) {
  // phases 1/2 take W1 (and in phase 2 W2) with their BN folded in (k_rp_fold): ReLU only
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const bf16_t* sW1 = (const bf16_t*)(smem + C2W_OFF_W1);
  const bf16_t* sW2 = (const bf16_t*)(smem + C2W_OFF_W2);
  const bf16_t* sW3 = (const bf16_t*)(smem + C2W_OFF_W3);
  const bf16_t* sW4 = (const bf16_t*)(smem + C2W_OFF_W4);
  float* sb = (float*)(smem + c2w_off_b<PHASE>());
  float* sb1 = sb;
  float* sb2 = sb1 + STEM_C;
  float* sb3 = sb2 + FUS_C;
  float* sb4 = sb3 + ATT_C;
  bf16_t* patch = (bf16_t*)(smem + c2w_off_patch<PHASE>());
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  // ---- one-time LDS fill: weights, biases, BN affines, im2col table
  {
    auto copy_rows = [&](size_t dst, size_t src, int rows, int k, int stride) {  // 16-byte pieces
      const int per = k / 8;
      for (int i = tid; i < rows * per; i += 512) {
        const int rr = i / per, q = i % per;
        *reinterpret_cast<uint4*>(smem + dst + ((size_t)rr * stride + 8 * q) * 2) =
            *reinterpret_cast<const uint4*>(blob + src + ((size_t)rr * k + 8 * q) * 2);
      }
    };
    auto copy_rows_p = [&](size_t dst, const char* base, int rows, int k, int stride) {
      const int per = k / 8;
      for (int i = tid; i < rows * per; i += 512) {
        const int rr = i / per, q = i % per;
        *reinterpret_cast<uint4*>(smem + dst + ((size_t)rr * stride + 8 * q) * 2) =
            *reinterpret_cast<const uint4*>(base + ((size_t)rr * k + 8 * q) * 2);
      }
    };
    if (PHASE == 0)
      copy_rows(C2W_OFF_W1, L.w1s, STEM_C, STEM_K2, C2W_S1);
    else
      copy_rows_p(C2W_OFF_W1, fold + FOLD_W1, STEM_C, STEM_K2, C2W_S1);
    if (PHASE >= 1) {
      if (PHASE == 2)
        copy_rows_p(C2W_OFF_W2, fold + FOLD_W2, FUS_C, STEM_C, C2W_S2);
      else
        copy_rows(C2W_OFF_W2, L.w2, FUS_C, STEM_C, C2W_S2);
    }
    if (PHASE == 2) {  // phase 1 keeps its shifted patch copies there
      copy_rows(C2W_OFF_W3, L.w3, ATT_C, FUS_C, C2W_S3);
      copy_rows(C2W_OFF_W4, L.w4, FUS_C, ATT_C, C2W_S4);
    }
    for (int i = tid; i < STEM_C; i += 512)
      sb1[i] = PHASE == 0 ? ((const float*)(blob + L.b1))[i] : ((const float*)(fold + FOLD_B1))[i];
    for (int i = tid; i < FUS_C; i += 512)
      sb2[i] = PHASE == 2 ? ((const float*)(fold + FOLD_B2))[i] : ((const float*)(blob + L.b2))[i];
    for (int i = tid; i < ATT_C; i += 512) sb3[i] = ((const float*)(blob + L.b3))[i];
    for (int i = tid; i < FUS_C; i += 512) sb4[i] = ((const float*)(blob + L.b4))[i];
    for (int i = tid; i < 3 * C2W_PH * C2W_PWP; i += 512) patch[i] = 0;  // pad columns stay zero
    for (int i = tid; i < STEM_C * (C2W_S1 - STEM_K2); i += 512)  // W1 row pads: never garbage in an MFMA
      ((bf16_t*)(smem + C2W_OFF_W1))[(i / (C2W_S1 - STEM_K2)) * C2W_S1 + STEM_K2 + i % (C2W_S1 - STEM_K2)] = 0;
  }
  // BN statistics (phases 0/1): the layer whose statistics the phase collects runs with its MFMA
  // operands swapped, so its accumulator is [pixel][channel]: lane (r, g) owns channel 16t + r
  // and the pixels {4g .. 4g+3} of each 16-px half.  Running sums stay per lane across tiles (no
  // cross-lane traffic per tile) and the 4 lane groups are combined once, in fixed order, at
  // the end.
  constexpr int NST = PHASE == 0 ? 12 : 8;  // channel tiles whose stats this phase collects
  float ssum[NST], ssq[NST];
#pragma unroll
  for (int i = 0; i < NST; ++i) ssum[i] = ssq[i] = 0.f;
  const int tiles_x = (W + C2W_TW - 1) / C2W_TW, tiles_y = (H + C2W_TH - 1) / C2W_TH;
  const unsigned per = (unsigned)(tiles_x * tiles_y);
  const int ntiles = B * tiles_x * tiles_y;  // < 2^31 (rgbd_ratio_predict checks the shape)
  const long long HW = (long long)H * W;
  // the next tile's depth patch is prefetched into registers while the current one computes
  constexpr int PATCH_N = 3 * C2W_PH * C2W_PW, PATCH_PER = (PATCH_N + 511) / 512;
  float pre[PATCH_PER];
  // Phases 1-2: the loads go through a buffer descriptor, unconditionally; an element outside the
  // image or the patch gets an offset past the descriptor's end, which the hardware returns as
  // zero.  Behind per-element branches (phase 0's form) the compiler waits for each load right
  // where it is issued, so the "prefetch" stalled every phase-1 tile by a memory round trip
  // (3 600 of 18 700 cycles in the stamps); this way nothing reads pre[] before the next tile's
  // staging.  Phase 0 keeps the branches: at four workgroups per CU its waits are hidden, and
  // the other form spilled it past its 128-register budget.
  const long long dbytes = ((long long)(B - 1) * bstride + 3 * HW) * 4;
  const bool dbuf = PHASE >= 1 && dbytes < (1ll << 31);  // 32-bit byte offsets cover the input
  const __amdgpu_buffer_rsrc_t drs = wt_rsrc(depth3, dbuf ? (int)dbytes : 0);
  auto fetch_patch = [&](int t) {
    const TileDec td = tile_dec((unsigned)t, per, (unsigned)tiles_x, C2W_TH, C2W_TW);
#pragma unroll
    for (int k = 0; k < PATCH_PER; ++k) {
      const int i = tid + 512 * k;
      const int c = i / (C2W_PH * C2W_PW), yy = (i / C2W_PW) % C2W_PH, xx = i % C2W_PW;
      const int yv = td.y0 + yy - 3, xv = td.x0 + xx - 3;
      const bool ok = i < PATCH_N && t < ntiles && yv >= 0 && yv < H && xv >= 0 && xv < W;
      if (dbuf) {
        const uint32_t off = ok ? (uint32_t)((td.b * bstride + c * HW + (long long)yv * W + xv) * 4) : 0x80000000u;
        pre[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(drs, off, 0, 0));
      } else {
        float v = 0.f;
        if (ok) v = depth3[td.b * bstride + c * HW + (long long)yv * W + xv];
        pre[k] = v;
      }
    }
  };
  // per-lane statistics of a transposed accumulator tile (pixel validity only on ragged tiles)
  auto add_stats = [&](float& sm, float& sq, const f32x4 (&a)[2], bool full, int x0, bool row_ok) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = a[u][j];
        if (!full) v = (row_ok && x0 + 16 * u + 4 * g + j < W) ? v : 0.f;
        sm += v;
        sq = __builtin_fmaf(v, v, sq);
      }
  };
  fetch_patch(blockIdx.x);
  int tcount = 0;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++tcount) {
    // tiles 8..11 of workgroup 0 (past the start-up: weights landing, every workgroup's first loads)
    unsigned long long* const sts = (STAMPS && blockIdx.x == 0 && tcount >= 8 && tcount < 12) ? g_c2_stamps : nullptr;
    const long long sidx = ((long long)PHASE * 32 + (long long)(tcount - 8) * 8 + wave) * 7;
    if (STAMPS && sts) c2_stamp(sts, sidx + 0);
    const TileDec td = tile_dec((unsigned)tile, per, (unsigned)tiles_x, C2W_TH, C2W_TW);
    const int b = td.b, y0 = td.y0, x0 = td.x0;
    lds_barrier();  // everyone is done with the previous patch
#pragma unroll
    for (int k = 0; k < PATCH_PER; ++k) {
      const int i = tid + 512 * k;
      if (i < PATCH_N) patch[(i / C2W_PW) * C2W_PWP + i % C2W_PW] = f32_to_bf16(pre[k]);
    }
    lds_barrier();
    if constexpr (PHASE == 1) {  // the eight shifted copies, 16 bytes at a time
      // a lane reads copy (col & 7) at elements (col & ~7) .. +7 <= 31: chunks 0..3 of each row
      bf16_t* p8 = (bf16_t*)(smem + C2W_OFF_P8);
      for (int i = tid; i < 8 * 3 * C2W_PH * 4; i += 512) {
        const int j8 = i & 3, row = (i >> 2) % (3 * C2W_PH), k = i / (3 * C2W_PH * 4);
        const int e = 8 * j8 + k;  // first patch column of this chunk (<= 31: five words in the row)
        const uint32_t* wp = reinterpret_cast<const uint32_t*>(patch + row * C2W_PWP + (e & ~1));
        const uint32_t w0 = wp[0], w1 = wp[1], w2 = wp[2], w3 = wp[3], w4 = wp[4];
        const uint32_t sh = (e & 1) * 2;
        *reinterpret_cast<uint4*>(p8 + (k * 3 * C2W_PH + row) * C2W_PWP + 8 * j8) =
            make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                       __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
      }
      lds_barrier();
    }
    if (STAMPS && sts) c2_stamp(sts, sidx + 1);
    fetch_patch(tile + gridDim.x);
    if (STAMPS && sts) c2_stamp(sts, sidx + 2);
    const int py = y0 + wave;
    const bool row_ok = py < H;
    const bool full = row_ok && x0 + C2W_TW <= W;  // wave-uniform
    bool pv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) pv[u] = row_ok && x0 + 16 * u + r < W;
    // ---- stem B operand: K = (c, dy, dx8) groups; lane (r, g) of step s takes group q = 4s + g,
    // i.e. the 8 bf16 patch values (c, row wave+dy, cols 16u+r .. +7): five aligned words from
    // col & ~1 and a byte-align by 2*(col & 1).
    auto stem_b = [&](int s, Frag<bf16_t> (&bf)[2]) {
      const int q = 4 * s + g;
      if constexpr (PHASE == 1) {  // copy (col & 7) = (r & 7) for both halves u, 16 columns apart
        const int qc = q < 21 ? q : 20;
        const int cq = qc / 7, dy = qc - 7 * cq;
        const bf16_t* p8 = (const bf16_t*)(smem + C2W_OFF_P8) + (((r & 7) * 3 + cq) * C2W_PH + wave + dy) * C2W_PWP +
                           (r & 8);
        bf[0].v = *reinterpret_cast<const uint4*>(p8);
        bf[1].v = *reinterpret_cast<const uint4*>(p8 + 16);
        if (q >= 21) {
          bf[0].zero();
          bf[1].zero();
        }
        return;
      }
      const int cq = q / 7, dy = q - 7 * cq;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (q < 21) {
          const int col = 16 * u + r;
          const uint32_t* wp = reinterpret_cast<const uint32_t*>(patch + (cq * C2W_PH + wave + dy) * C2W_PWP + (col & ~1));
          const uint32_t w0 = wp[0], w1 = wp[1], w2 = wp[2], w3 = wp[3], w4 = wp[4];
          const uint32_t sh = (col & 1) * 2;
          bf[u].v = make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                               __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
        } else {
          bf[u].zero();
        }
      }
    };
    // Zero K blocks of the 3x3 / 5x5 filters embedded in the 7x7 window are skipped (channel
    // groups t < 4 use steps {0,1,2,4}, t < 8 steps 0..4, t >= 8 all six); groups 21..23 of
    // step 5 lie past the 168 packed columns.  Accumulators start at the bias.
    auto stem_w = [&](int t, int s) {
      Frag<bf16_t> af;
      af.v = *reinterpret_cast<const uint4*>(sW1 + (16 * t + r) * C2W_S1 + 32 * s + 8 * g);
      if (s == 5) af.select(g == 0);
      return af;
    };
    auto stem_live = [](int t, int s) { return !((t < 4 && (s == 3 || s == 5)) || (t >= 4 && t < 8 && s == 5)); };
    if constexpr (PHASE == 0) {
      // statistics only: channel group outermost with the operands swapped (accumulator
      // [pixel][channel]), all six B fragments built once, two accumulators live at a time
      Frag<bf16_t> bfr[6][2];
#pragma unroll
      for (int s = 0; s < 6; ++s) stem_b(s, bfr[s]);
#pragma unroll
      for (int t = 0; t < 12; ++t) {
        const float bb = sb1[16 * t + r];
        f32x4 a1[2] = {f32x4{bb, bb, bb, bb}, f32x4{bb, bb, bb, bb}};
#pragma unroll
        for (int s = 0; s < 6; ++s) {
          if (!stem_live(t, s)) continue;
          const Frag<bf16_t> af = stem_w(t, s);
          mma(a1[0], bfr[s][0], af);
          mma(a1[1], bfr[s][1], af);
        }
        add_stats(ssum[t], ssq[t], a1, full, x0, row_ok);
      }
      if (STAMPS && sts) c2_stamp(sts, sidx + 3);
      continue;
    }
    // phases 1, 2: K step outermost (one B fragment pair live), all 12 channel groups accumulate
    f32x4 a1[12][2];
#pragma unroll
    for (int t = 0; t < 12; ++t) {
      const float4 bb = *reinterpret_cast<const float4*>(sb1 + 16 * t + 4 * g);
      a1[t][0] = a1[t][1] = f32x4{bb.x, bb.y, bb.z, bb.w};
    }
    if constexpr (PHASE == 1) {
      // one K step of patch fragments in flight ahead of the MFMAs that use the current one
      // (the scheduling fences keep the compiler from hoisting more steps: register budget)
      Frag<bf16_t> bcur[2], bnxt[2];
      stem_b(0, bcur);
#pragma unroll
      for (int s = 0; s < 6; ++s) {
        if (s < 5) stem_b(s + 1, bnxt);
#pragma unroll
        for (int t = 0; t < 12; ++t) {
          if (!stem_live(t, s)) continue;
          const Frag<bf16_t> af = stem_w(t, s);
          mma(a1[t][0], af, bcur[0]);
          mma(a1[t][1], af, bcur[1]);
        }
        __builtin_amdgcn_sched_barrier(0);
        bcur[0] = bnxt[0];
        bcur[1] = bnxt[1];
      }
    } else {
#pragma unroll
      for (int s = 0; s < 6; ++s) {
        Frag<bf16_t> bfr[2];
        stem_b(s, bfr);
#pragma unroll
        for (int t = 0; t < 12; ++t) {
          if (!stem_live(t, s)) continue;
          const Frag<bf16_t> af = stem_w(t, s);
          mma(a1[t][0], af, bfr[0]);
          mma(a1[t][1], af, bfr[1]);
        }
      }
    }
    if (STAMPS && sts) c2_stamp(sts, sidx + 3);
    Frag<bf16_t> f1[6][2];
#pragma unroll
    for (int s = 0; s < 6; ++s)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float vv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) vv[e] = fmaxf(a1[2 * s + (e >> 2)][u][e & 3], 0.f);  // BN1 folded into W1
        f1[s][u].from8(vv);
      }
    if (STAMPS && sts) c2_stamp(sts, sidx + 4);
    // ---- fusion (phase 1: operands swapped for the statistics)
    f32x4 a2[8][2];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      if constexpr (PHASE == 1) {
        const float bb = sb2[16 * t + r];
        a2[t][0] = a2[t][1] = f32x4{bb, bb, bb, bb};
      } else {
        const float4 bb = *reinterpret_cast<const float4*>(sb2 + 16 * t + 4 * g);
        a2[t][0] = a2[t][1] = f32x4{bb.x, bb.y, bb.z, bb.w};
      }
#pragma unroll
      for (int s = 0; s < 6; ++s) {
        Frag<bf16_t> af;
        af.v = *reinterpret_cast<const uint4*>(sW2 + (16 * t + r) * C2W_S2 + 32 * s + 8 * g);
        if constexpr (PHASE == 1) {
          mma(a2[t][0], f1[s][0], af);
          mma(a2[t][1], f1[s][1], af);
        } else {
          mma(a2[t][0], af, f1[s][0]);
          mma(a2[t][1], af, f1[s][1]);
        }
      }
    }
    if (STAMPS && sts) c2_stamp(sts, sidx + 5);
    if constexpr (PHASE == 1) {
#pragma unroll
      for (int t = 0; t < 8; ++t) add_stats(ssum[t], ssq[t], a2[t], full, x0, row_ok);
      if (att) {  // raw fusion output for k_rp_gate: [tile][wave][t][lane][u][4 px], 1 KiB per store
        bf16_t* ft = att + (((long long)tile * 8 + wave) * 16) * 256;
#pragma unroll
        for (int t = 0; t < 8; ++t)
          *reinterpret_cast<uint4*>(ft + (t * 64 + lane) * 8) =
              make_uint4(pack_bf16x2(a2[t][0][0], a2[t][0][1]), pack_bf16x2(a2[t][0][2], a2[t][0][3]),
                         pack_bf16x2(a2[t][1][0], a2[t][1][1]), pack_bf16x2(a2[t][1][2], a2[t][1][3]));
      }
      if (STAMPS && sts) c2_stamp(sts, sidx + 6);
      continue;
    }
    if constexpr (PHASE == 2) {
#pragma unroll
      for (int t = 0; t < 8; ++t)  // BN2 folded into W2
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a2[t][0][j] = fmaxf(a2[t][0][j], 0.f);
          a2[t][1][j] = fmaxf(a2[t][1][j], 0.f);
        }
      Frag<bf16_t> f2[4][2];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          float vv[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) vv[e] = a2[2 * s + (e >> 2)][u][e & 3];
          f2[s][u].from8(vv);
        }
      f32x4 a3[4][2];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float4 bb = *reinterpret_cast<const float4*>(sb3 + 16 * t + 4 * g);
        a3[t][0] = a3[t][1] = f32x4{bb.x, bb.y, bb.z, bb.w};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          Frag<bf16_t> af;
          af.v = *reinterpret_cast<const uint4*>(sW3 + (16 * t + r) * C2W_S3 + 32 * s + 8 * g);
          mma(a3[t][0], af, f2[s][0]);
          mma(a3[t][1], af, f2[s][1]);
        }
      }
      Frag<bf16_t> f3[2][2];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          float vv[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) vv[e] = fmaxf(a3[2 * s + (e >> 2)][u][e & 3], 0.f);
          f3[s][u].from8(vv);
        }
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const float4 bb = *reinterpret_cast<const float4*>(sb4 + 16 * t + 4 * g);
        f32x4 a4[2] = {f32x4{bb.x, bb.y, bb.z, bb.w}, f32x4{bb.x, bb.y, bb.z, bb.w}};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          Frag<bf16_t> af;
          af.v = *reinterpret_cast<const uint4*>(sW4 + (16 * t + r) * C2W_S4 + 32 * s + 8 * g);
          mma(a4[0], af, f3[s][0]);
          mma(a4[1], af, f3[s][1]);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (!pv[u]) continue;
          float o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = a2[t][u][j] * sigmoid_fast(a4[u][j]);
          // conv5 v4's padded channel-quarter-major planes (c4_att_idx)
          *reinterpret_cast<uint2*>(att + c4_att_idx(b, t >> 1, py, x0 + 16 * u + r, H, W) + 16 * (t & 1) + 4 * g) =
              make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
        }
      }
    }
  }
  if constexpr (PHASE < 2) {
    // lanes r, r+16, r+32, r+48 hold channel 16t + r: combine in fixed order, one slab row per wave
    const long long row = (long long)blockIdx.x * 8 + wave;
    constexpr int NC = PHASE == 0 ? STEM_C : FUS_C;
#pragma unroll
    for (int t = 0; t < NST; ++t) {
      float a = ssum[t], q = ssq[t];
      a += __shfl_xor(a, 16);
      q += __shfl_xor(q, 16);
      a += __shfl_xor(a, 32);
      q += __shfl_xor(q, 32);
      if (g == 0) {
        // phase 1: channel-major (k_bn_affine cm = 1); phase 0: row-major (k_bn_affine_stem)
        const long long e = PHASE == 1 ? (long long)(16 * t + r) * (gridDim.x * 8) + row : row * NC + 16 * t + r;
        slab[e * 2 + 0] = a;
        slab[e * 2 + 1] = q;
      }
    }
  }
}

// ---- train mode, bf16: the chain's last stage from phase 1's stored fusion output.
// Phase 1 has to run the stem + fusion for the BN2 statistics anyway; storing its raw fusion
// output (fragment-native, 256 B/px) lets this kernel skip the stem + fusion recompute that
// phase 2 would do (111 k FLOP/px): per 8x32-px tile a wave owns one pixel row, reads its 8 KB,
// applies BN2 + ReLU, transposes through a wave-private LDS image [32 px][128 ch], and runs the
// attention 1x1s (128->64->128, LDS-resident weights) and the sigmoid gate; HBM-bound
// (512 B/px).  The eval path (no statistics pass) keeps phase 2.
constexpr int GT_S = FUS_C + 8;  // image row: 128 channels + 8 pad (272 B, conflict-free b64 reads)
constexpr size_t GT_OFF_W3 = 0;
constexpr size_t GT_OFF_W4 = GT_OFF_W3 + (size_t)ATT_C * C2W_S3 * 2;
constexpr size_t GT_OFF_B = GT_OFF_W4 + (size_t)FUS_C * C2W_S4 * 2;  // b3[64], b4[128], aff2[128]
constexpr size_t GT_OFF_IMG = GT_OFF_B + (size_t)(ATT_C + FUS_C + 2 * FUS_C) * 4;
constexpr size_t GT_SMEM = GT_OFF_IMG + (size_t)8 * C2W_TW * GT_S * 2;
static_assert(GT_SMEM <= 163840, "gate LDS budget");

__global__ __launch_bounds__(512) void k_rp_gate(const bf16_t* __restrict__ fus, int B, int H, int W,
                                                 const char* __restrict__ blob, Layout L,
                                                 const float2* __restrict__ aff2, bf16_t* __restrict__ att) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const bf16_t* sW3 = (const bf16_t*)(smem + GT_OFF_W3);
  const bf16_t* sW4 = (const bf16_t*)(smem + GT_OFF_W4);
  float* sb3 = (float*)(smem + GT_OFF_B);
  float* sb4 = sb3 + ATT_C;
  float2* saff = (float2*)(sb4 + FUS_C);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  bf16_t* img = (bf16_t*)(smem + GT_OFF_IMG) + (size_t)wave * C2W_TW * GT_S;
  {
    auto copy_rows = [&](size_t dst, size_t src, int rows, int k, int stride) {
      const int per = k / 8;
      for (int i = tid; i < rows * per; i += 512) {
        const int rr = i / per, q = i % per;
        *reinterpret_cast<uint4*>(smem + dst + ((size_t)rr * stride + 8 * q) * 2) =
            *reinterpret_cast<const uint4*>(blob + src + ((size_t)rr * k + 8 * q) * 2);
      }
    };
    copy_rows(GT_OFF_W3, L.w3, ATT_C, FUS_C, C2W_S3);
    copy_rows(GT_OFF_W4, L.w4, FUS_C, ATT_C, C2W_S4);
    for (int i = tid; i < ATT_C; i += 512) sb3[i] = ((const float*)(blob + L.b3))[i];
    for (int i = tid; i < FUS_C; i += 512) {
      sb4[i] = ((const float*)(blob + L.b4))[i];
      saff[i] = aff2[i];
    }
  }
  __syncthreads();
  const int tiles_x = (W + C2W_TW - 1) / C2W_TW, tiles_y = (H + C2W_TH - 1) / C2W_TH;
  const unsigned per = (unsigned)(tiles_x * tiles_y);
  const int ntiles = B * tiles_x * tiles_y;
  // this wave's raw fusion output of a tile ([t][lane][u][4 px]): lane (r, g) has channel 16t + r,
  // pixels 16u + 4g + j;
  // the next tile's 8 KB are loaded while the current one computes
  uint2 nxt[8][2];
  auto fetch = [&](int tl) {
    if (tl >= ntiles) return;
    const int tp = ntiles - 1 - tl;  // physical tile: last-to-first (see conv5 v4's tile order)
    const bf16_t* ft = fus + (((long long)tp * 8 + wave) * 16) * 256;
#pragma unroll
    for (int t = 0; t < 8; ++t) {  // read once: non-temporal, 16 B per lane (1 KiB per wave load)
      const u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(ft + (t * 64 + lane) * 8));
      nxt[t][0] = make_uint2(q[0], q[1]);
      nxt[t][1] = make_uint2(q[2], q[3]);
    }
  };
  // (one tile ahead: two and three tiles ahead measured the same, 0.252-0.258 ms, round 6)
  fetch(blockIdx.x);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const TileDec td = tile_dec((unsigned)(ntiles - 1 - tile), per, (unsigned)tiles_x, C2W_TH, C2W_TW);
    const int b = td.b, y0 = td.y0, x0 = td.x0;
    const int py = y0 + wave;
    uint2 raw[8][2];
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
      for (int u = 0; u < 2; ++u) raw[t][u] = nxt[t][u];
    fetch(tile + gridDim.x);
    if (py >= H) continue;  // wave-uniform; nothing below synchronises across waves
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // previous tile's image reads are done
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int c = 16 * t + r;
      const float2 a = saff[c];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint32_t w01 = raw[t][u].x, w23 = raw[t][u].y;
        const float v[4] = {__uint_as_float(w01 << 16), __uint_as_float(w01 & 0xffff0000u),
                            __uint_as_float(w23 << 16), __uint_as_float(w23 & 0xffff0000u)};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          img[(16 * u + 4 * g + j) * GT_S + c] = f32_to_bf16(fmaxf(__builtin_fmaf(v[j], a.x, a.y), 0.f));  // BN2 + ReLU
      }
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // ---- W3 B operand in the chain's K order: element e of chunk s = channel 32s + 16(e>>2) + 4g + (e&3)
    Frag<bf16_t> f2[4][2];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const bf16_t* row = img + (16 * u + r) * GT_S + 32 * s + 4 * g;
        const uint2 lo = *reinterpret_cast<const uint2*>(row), hi = *reinterpret_cast<const uint2*>(row + 16);
        f2[s][u].v = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
    f32x4 a3[4][2];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float4 bb = *reinterpret_cast<const float4*>(sb3 + 16 * t + 4 * g);
      a3[t][0] = a3[t][1] = f32x4{bb.x, bb.y, bb.z, bb.w};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        Frag<bf16_t> af;
        af.v = *reinterpret_cast<const uint4*>(sW3 + (16 * t + r) * C2W_S3 + 32 * s + 8 * g);
        mma(a3[t][0], af, f2[s][0]);
        mma(a3[t][1], af, f2[s][1]);
      }
    }
    Frag<bf16_t> f3[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float vv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) vv[e] = fmaxf(a3[2 * s + (e >> 2)][u][e & 3], 0.f);
        f3[s][u].from8(vv);
      }
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float4 bb = *reinterpret_cast<const float4*>(sb4 + 16 * t + 4 * g);
      f32x4 a4[2] = {f32x4{bb.x, bb.y, bb.z, bb.w}, f32x4{bb.x, bb.y, bb.z, bb.w}};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        Frag<bf16_t> af;
        af.v = *reinterpret_cast<const uint4*>(sW4 + (16 * t + r) * C2W_S4 + 32 * s + 8 * g);
        mma(a4[0], af, f3[s][0]);
        mma(a4[1], af, f3[s][1]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        // the gated value replaces the activation it came from (same lane, same 8 bytes)
        uint2* cell = reinterpret_cast<uint2*>(img + (16 * u + r) * GT_S + 16 * t + 4 * g);
        const uint2 act = *cell;
        const float av[4] = {__uint_as_float(act.x << 16), __uint_as_float(act.x & 0xffff0000u),
                             __uint_as_float(act.y << 16), __uint_as_float(act.y & 0xffff0000u)};
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = av[j] * sigmoid_fast(a4[u][j]);
        *cell = make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
      }
    }
    // store into conv5 v4's padded channel-quarter-major planes (c4_att_idx) of the wave's 32 pixels
    // from the image: per store instruction one quarter of 16 consecutive pixels (1 KB contiguous)
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int qt = k >> 1, pr = 16 * (k & 1) + (lane >> 2), q = lane & 3;
      if (x0 + pr < W)
        *reinterpret_cast<uint4*>(att + c4_att_idx(b, qt, py, x0 + pr, H, W) + 8 * q) =
            *reinterpret_cast<const uint4*>(img + pr * GT_S + 32 * qt + 8 * q);
    }
  }
}

// ------------------------------------------------------------------ conv5: 3x3 128->256
constexpr int CV_TH = 4, CV_TW = 32;             // 128-pixel tile
constexpr int CV_PH = CV_TH + 2, CV_PW = CV_TW + 2;
constexpr int CV_BN = 128;                       // output channels per workgroup
constexpr int CV_CPAD = 40;                      // 32 channels + 8 pad (80-byte rows)

template <typename T>
__global__ __launch_bounds__(256) void k_rp_conv3x3(const T* __restrict__ x, int B, int H, int W,
                                                    const char* __restrict__ blob, Layout L, T* __restrict__ y,
                                                    float* __restrict__ slab) {
  // x: NHWC [B][H][W][128]; y: NHWC [B][H][W][256]; slab: [grid][256][2] (sum, sumsq of y)
  __shared__ T patch[CV_PH * CV_PW][CV_CPAD];
  __shared__ float st[4][64][2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int wm = wave & 1, wn = wave >> 1;   // wave tile: 64 px (2 tile rows) x 64 ch
  const int n0 = blockIdx.y * CV_BN + wn * 64;
  const T* w5 = (const T*)(blob + L.w5);
  const float* b5 = (const float*)(blob + L.b5);
  const int tiles_x = (W + CV_TW - 1) / CV_TW, tiles_y = (H + CV_TH - 1) / CV_TH;
  const long long ntiles = (long long)B * tiles_x * tiles_y;
  for (int i = threadIdx.x; i < 4 * 64 * 2; i += 256) (&st[0][0][0])[i] = 0.f;
  for (long long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int b = (int)(tile / ((long long)tiles_x * tiles_y));
    const int trem = (int)(tile % ((long long)tiles_x * tiles_y));
    const int y0 = (trem / tiles_x) * CV_TH, x0 = (trem % tiles_x) * CV_TW;
    f32x4 acc[4][4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int nj = 0; nj < 4; ++nj) acc[mi][nj] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < FUS_C; c0 += 32) {
      __syncthreads();
      // stage the 6x34 halo x 32 channels: 204 pixels x 4 chunks of 8 channels
      for (int i = threadIdx.x; i < CV_PH * CV_PW * 4; i += 256) {
        const int pp = i >> 2, q = i & 3;
        const int yy = y0 + pp / CV_PW - 1, xx = x0 + pp % CV_PW - 1;
        Frag<T> f;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W)
          f.load(x + (((long long)b * H + yy) * W + xx) * FUS_C + c0 + 8 * q);
        else
          f.zero();
        *reinterpret_cast<Frag<T>*>(&patch[pp][8 * q]) = f;
      }
      __syncthreads();
#pragma unroll 1
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap % 3;
        Frag<T> bf[4];
#pragma unroll
        for (int nj = 0; nj < 4; ++nj)
          bf[nj].load(w5 + (long long)(n0 + 16 * nj + r) * (9 * FUS_C) + tap * FUS_C + c0 + 8 * g);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          // rows of this 16-px tile: tile row (wm*2 + mi/2), cols (mi%2)*16 + r
          const int ty = wm * 2 + (mi >> 1), tx = (mi & 1) * 16 + r;
          Frag<T> af = *reinterpret_cast<const Frag<T>*>(&patch[(ty + ky) * CV_PW + tx + kx][8 * g]);
#pragma unroll
          for (int nj = 0; nj < 4; ++nj) mma(acc[mi][nj], af, bf[nj]);
        }
      }
    }
    // epilogue: y = acc + b5 (NHWC), BN partial sums
#pragma unroll
    for (int nj = 0; nj < 4; ++nj) {
      const int n = n0 + 16 * nj + r;
      const float bias = b5[n];
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int ty = wm * 2 + (mi >> 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int tx = (mi & 1) * 16 + 4 * g + j;
          const int yy = y0 + ty, xx = x0 + tx;
          const float v = acc[mi][nj][j] + bias;
          if (yy < H && xx < W) {
            const T tv = Num<T>::from_f(v);
            y[(((long long)b * H + yy) * W + xx) * C5 + n] = tv;
            const float vr = Num<T>::to_f(tv);  // statistics of the stored values
            s += vr;
            q += vr * vr;
          }
        }
      }
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      if (g == 0) {
        st[wave][16 * nj + r][0] += s;
        st[wave][16 * nj + r][1] += q;
      }
    }
  }
  __syncthreads();
  // waves (wm=0,1) with the same wn own the same 64 channels
  for (int i = threadIdx.x; i < CV_BN; i += 256) {
    const int wnn = i / 64, c = i % 64;
#pragma unroll
    for (int q = 0; q < 2; ++q)
      slab[((long long)blockIdx.x * C5 + blockIdx.y * CV_BN + i) * 2 + q] =
          st[2 * wnn][c][q] + st[2 * wnn + 1][c][q];
  }
}

// ------------------------------------------------------------------ BN + ReLU + AdaptiveAvgPool(4)
constexpr int POOL_SPLIT = 16;  // row chunks per pool region

template <typename T>
__global__ __launch_bounds__(256) void k_rp_bn_relu_pool(const T* __restrict__ y, int H, int W,
                                                         const float2* __restrict__ aff,
                                                         float* __restrict__ part) {
  // grid: (16 regions * POOL_SPLIT, B); 256 threads = 32 channel octets x 8 pixel lanes;
  // part[b][region][split][256] (fixed-order sums: deterministic)
  __shared__ float red[8][C5];
  const int b = blockIdx.y, reg = blockIdx.x / POOL_SPLIT, sp = blockIdx.x % POOL_SPLIT;
  const int i = reg / 4, j = reg % 4;
  const int oct = threadIdx.x & 31, pl = threadIdx.x >> 5;
  const int ya = (i * H) / 4, yb = ((i + 1) * H + 3) / 4, xa = (j * W) / 4, xb = ((j + 1) * W + 3) / 4;
  const int rows = yb - ya, cols = xb - xa;
  const int r0 = ya + (rows * sp) / POOL_SPLIT, r1 = ya + (rows * (sp + 1)) / POOL_SPLIT;
  float2 af[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) af[e] = aff[8 * oct + e];
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int npx = (r1 - r0) * cols;
  for (int q = pl; q < npx; q += 8) {
    const int yy = r0 + q / cols, xx = xa + q % cols;
    Frag<T> f;
    f.load(y + (((long long)b * H + yy) * W + xx) * C5 + 8 * oct);
    float v[8];
    f.to8(v);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += fmaxf(v[e] * af[e].x + af[e].y, 0.f);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[pl][8 * oct + e] = acc[e];
  __syncthreads();
  const int c = threadIdx.x;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += red[k][c];
  part[(((long long)b * 16 + reg) * POOL_SPLIT + sp) * C5 + c] = s;
}

// one LDS-DMA wave instruction: 64 lanes x 16 B from per-lane sources to lds_base + 16 * lane
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_base) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_base)
               : "memory");
}

// ---- conv5 v4 (bf16): a work item is a 16x32-pixel tile x one 128-channel half of the output
// (512 px x 128 ch; the two halves of a tile run at the same time on two workgroups of one XCD,
// so the second one's input copies hit the L2 the first one filled).  8 waves, wave w = tile
// rows 2w, 2w+1 (64 px) x all 128 channels = 4x8 MFMA 16x16x32 tiles (the v3 wave tile).  K is
// walked in 12 steps of (input-channel quarter qt, kernel row ky), each step the 3 taps kx of
// that row over the quarter's 32 channels (K 96: 96 MFMAs per wave between two barriers).
// Against v3's 256 px x 256 ch items this halves the weight copies per FLOP (the weights of a
// step serve 512 pixels) at a slightly larger input share: 445 KB of LDS-DMA per item instead of
// 2 x 332 KB for the same FLOPs (-33 %), ~4.6 one-KiB pieces per wave and step instead of 9
// per loader wave.
// LDS: two input slots (quarter qt in slot qt & 1: the whole 18x34 halo x 32 channels, 64-byte
// rows, 16-byte chunk c at slot c ^ ((row >> 1) & 2): ds_read_b128 conflict-free for 16
// consecutive rows from any start row), two weight buffers of one step ([kx][n][32 ch], the same
// swizzle, pre-applied in the blob so a step is one linear 24 KiB copy).
// Pipeline: in step st waves 0-3 issue the weights of step st+1 (the next item's step 0 after
// the last: a workgroup always owns the same channel half) before their MFMAs; waves 4-7 issue
// a third of the next quarter's input (the next item's quarter 0 during quarter 3) after their
// first 32 MFMAs; every wave waits for its own copies, then the step's one barrier.
// MODE 0 (train): y stored fragment-native per item [item = 2 tile + half][wave][mi][np][lane][8]
//   (1 KiB contiguous per store instruction) and the BN statistics of the float32 conv outputs
//   kept in registers across items -> slab[256][workgroup][2] (the other half's entries zero).
// MODE 1 (eval, H % 4 == 0, W % 64 == 0, H >= 64, W >= 128: every 16-px fragment row lies in one
//   AdaptiveAvgPool(4) bin): BN (running statistics, `aff`) + ReLU of the bf16-rounded outputs
//   summed per pool bin in the epilogue -> out[item][4 bin slots][128]; no y.
// MODE 2 (eval, other shapes): y only.
// Tile order: every kernel of the chain -> gate -> conv5 -> pool sequence reads first what the
// previous one wrote last (still in the Infinity Cache): the chain writes its tiles first to last,
// the gate walks them last to first, conv5 first to last, the pool the images last to first
// (round 5: profiles/r05_v2/ab_w.txt, ab_zk.txt).
constexpr int C4_TH = 16, C4_TW = 32, C4_PW = C4_TW + 2;
constexpr int C4_NPIX = (C4_TH + 2) * C4_PW;  // 612 halo pixels
constexpr int C4_APIECES = 39;                // 624 rows of 64 B, 16 rows per 1 KiB piece
constexpr int C4_A_BYTES = C4_APIECES * 1024;
constexpr int C4_STEPS = 12;
constexpr int C4_B_BYTES = 3 * 128 * 64;  // one step: [kx][n][32 ch]
constexpr int C4_B_OFF = 2 * C4_A_BYTES;
constexpr int C4_RED_OFF = C4_B_OFF + 2 * C4_B_BYTES;
constexpr int C4_RED_BYTES = 8 * 4 * 128 * 4;  // MODE 1: per (wave, mi) bin sums of 128 channels
constexpr int C4_PAR_OFF = C4_RED_OFF + C4_RED_BYTES;
constexpr size_t C4_SMEM = C4_PAR_OFF + 128 * 4 + 128 * 8 + 32 * 4;  // bias, BN affine, bin slots
static_assert(C4_SMEM <= 163840, "conv5 v4 LDS budget");
static_assert(C4_APIECES * 16 >= C4_NPIX && C4_APIECES % 3 == 0, "conv5 v4 input pieces");
constexpr int C4_AK = (C4_APIECES + 3) / 4;  // input pieces per copying wave and quarter
static_assert(2 * C4_A_BYTES >= 8 * 128 * 2 * 4, "conv5 v4 statistics scratch");

__device__ __forceinline__ uint32_t c4_off(int row, int chunk) { return row * 64 + 16 * (chunk ^ ((row >> 1) & 2)); }

struct C4Tile {
  int b, y0, x0;
};
__device__ __forceinline__ C4Tile c4_tile(long long t, int tiles_x, int tiles_y) {
  C4Tile o;
  const long long per = (long long)tiles_x * tiles_y;
  o.b = (int)(t / per);
  const int rem = (int)(t % per);
  o.y0 = (rem / tiles_x) * C4_TH;
  o.x0 = (rem % tiles_x) * C4_TW;
  return o;
}

// C4_NODMA (experiment builds only, -DC4_NODMA=bits; results wrong, timing only): bit 0 drops the
// in-loop weight copies, bit 1 the in-loop input copies, bit 2 the step barrier, bit 3 the
// fragment reads (constant operands)
#ifndef C4_NODMA
#define C4_NODMA 0
#endif


// Stamps (the diagnostic build, RGBD_DIAG: rgbd_debug_conv5_stamps): workgroup 0 records, per step
// and wave of its first two items, s_memtime at the step top, after the weight-copy issue, after
// the first kx group (+ the input-copy issue), after the last MFMAs, after the closing wait +
// barrier: stamps[((item * 12 + step) * 8 + wave) * 5 + k].  The product build has no stamp code.
#if defined(RGBD_DIAG) && !defined(C4_STAMPS)
#define C4_STAMPS
#endif
#ifdef C4_STAMPS
__device__ unsigned long long* g_c4_stamps = nullptr;
__device__ __forceinline__ void c4_stamp(unsigned long long* st, long long idx) {
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) st[idx] = t;
  __builtin_amdgcn_sched_barrier(0);
}
#define C4_STAMP(k) \
  if (sts) c4_stamp(sts, (((long long)tcount * C4_STEPS + st) * 8 + wave) * 5 + (k))
#else
#define C4_STAMP(k)
#endif
template <int MODE>
__global__ __launch_bounds__(512) void k_rp_conv5_v4(const bf16_t* __restrict__ x, int B, int H, int W,
                                                     const char* __restrict__ blob, Layout L,
                                                     const float2* __restrict__ aff, bf16_t* __restrict__ y,
                                                     float* __restrict__ out, int xcd_pairs) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, g = lane >> 4;
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  // workgroups b and b + 8 (one XCD under round-robin placement: speed only) share the tiles
  int pair, nh;
  if (xcd_pairs) {
    nh = (blockIdx.x >> 3) & 1;
    pair = (blockIdx.x & 7) | ((blockIdx.x >> 4) << 3);
  } else {
    nh = blockIdx.x & 1;
    pair = blockIdx.x >> 1;
  }
  const int npairs = gridDim.x >> 1;
  const char* w5q = blob + L.w5q + (size_t)nh * C4_STEPS * C4_B_BYTES;
  float* sbias = (float*)(smem + C4_PAR_OFF);
  float2* saff = (float2*)(smem + C4_PAR_OFF + 512);
  int* sslot = (int*)(smem + C4_PAR_OFF + 512 + 1024);
  for (int i = tid; i < 128; i += 512) {
    sbias[i] = ((const float*)(blob + L.b5))[nh * 128 + i];
    if constexpr (MODE == 1) saff[i] = aff[nh * 128 + i];
  }
  const int tiles_x = (W + C4_TW - 1) / C4_TW, tiles_y = (H + C4_TH - 1) / C4_TH;
  const long long ntiles = (long long)B * tiles_x * tiles_y;

  // input piece j (rows 16j .. 16j+15 of the halo image) of quarter qt of tile t into slot sl:
  // the copying waves (4-7) own pieces j = w4 + 4k (k < 10); a lane's source offset from the
  // tile's padded origin depends on the piece and the plane width only, so it is computed once
  const int PW = c4_pw(W);
  const long long plane = (long long)c4_ph(H) * PW * 32;  // elements
  uint32_t aoff[C4_AK];
#pragma unroll
  for (int k = 0; k < C4_AK; ++k) {
    const int row = 16 * ((wave & 3) + 4 * k) + (lane >> 2), q = lane & 3;
    const int hy = row / C4_PW, hx = row - hy * C4_PW;
    aoff[k] = row < C4_NPIX ? (uint32_t)((hy * PW + hx) * 64 + 16 * (q ^ ((row >> 1) & 2))) : 0u;
  }
  auto issue_a = [&](const C4Tile& t, int qt, int sl, int k) {
    const char* base = (const char*)(x + ((long long)t.b * 4 + qt) * plane + ((long long)t.y0 * PW + t.x0) * 32);
    glds16(base + aoff[k], lds0 + sl * C4_A_BYTES + ((wave & 3) + 4 * k) * 1024);
  };
  // weight pieces k0..k1-1 (of 24) of step st into buffer st & 1
  auto issue_b = [&](int st, int k0, int k1) {
    const char* src = w5q + (size_t)st * C4_B_BYTES + 16 * lane;
    const uint32_t dst = lds0 + C4_B_OFF + (st & 1) * C4_B_BYTES;
    for (int k = k0; k < k1; ++k) glds16(src + 1024 * k, dst + 1024 * k);
  };
  const bool loader = wave < 4;

  f32x2 ssum[8], ssq[8];
#pragma unroll
  for (int nj = 0; nj < 8; ++nj) ssum[nj] = ssq[nj] = f32x2{0.f, 0.f};
  const int rh = H >> 2, rw = W >> 2;  // MODE 1: pool bin size

#ifndef C4_NOPRIO
  // the copying waves' partners compute first (static priority; loaders at equal priority
  // measured +20 %, loaders at priority +12 %)
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#endif
  long long tile = pair;
  if (tile < ntiles) {  // prologue: quarter 0 (waves 4-7) + the weights of step 0
    const C4Tile t = c4_tile(tile, tiles_x, tiles_y);
    if (!loader) {
#pragma unroll
      for (int k = 0; k < C4_AK; ++k)
        if ((wave & 3) + 4 * k < C4_APIECES) issue_a(t, 0, 0, k);
    }
    issue_b(0, 3 * wave, 3 * wave + 3);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

#ifdef C4_STAMPS
  int tcount = 0;
#endif
  for (; tile < ntiles; tile += npairs) {
#ifdef C4_STAMPS
    unsigned long long* const sts = (blockIdx.x == 0 && tcount < 2) ? g_c4_stamps : nullptr;
#endif
    const C4Tile t = c4_tile(tile, tiles_x, tiles_y);
    const long long ntile = tile + npairs;
    const bool has_next = ntile < ntiles;
    const C4Tile tn = c4_tile(has_next ? ntile : tile, tiles_x, tiles_y);
    f32x4 acc[4][8];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int nj = 0; nj < 8; ++nj) acc[mi][nj] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
    for (int st = 0; st < C4_STEPS; ++st) {
      const int qt = st / 3, ky = st - 3 * qt;
      C4_STAMP(0);
      if (!(C4_NODMA & 1) && loader && (st + 1 < C4_STEPS || has_next))
        issue_b(st + 1 < C4_STEPS ? st + 1 : 0, 6 * wave, 6 * wave + 6);
      C4_STAMP(1);
      const int qn = qt + 1;  // the quarter copied during this one (4: the next item's quarter 0)
      const bool a_go = !(C4_NODMA & 2) && !loader && (qn < 4 || has_next);
      const char* sa = smem + (qt & 1) * C4_A_BYTES;
      const char* sb = smem + C4_B_OFF + (st & 1) * C4_B_BYTES;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        Frag<bf16_t> fa[4], fb[8];
        if constexpr (!(C4_NODMA & 8)) {
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) {
            const int p = (2 * wave + (mi >> 1) + ky) * C4_PW + (mi & 1) * 16 + r + kx;
            fa[mi].v = *reinterpret_cast<const uint4*>(sa + c4_off(p, g));
          }
#pragma unroll
          for (int nj = 0; nj < 8; ++nj) fb[nj].v = *reinterpret_cast<const uint4*>(sb + c4_off(kx * 128 + 16 * nj + r, g));
        } else {
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) fa[mi].v = make_uint4(lane, kx, st, mi);
#pragma unroll
          for (int nj = 0; nj < 8; ++nj) fb[nj].v = make_uint4(nj, lane, kx, st);
        }
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int nj = 0; nj < 8; ++nj) mma(acc[mi][nj], fa[mi], fb[nj]);
        if (kx == 0 && a_go) {  // this step's 13 pieces [13 ky, 13 ky + 13) of the next quarter
#pragma unroll
          for (int k = 0; k < C4_AK; ++k) {
            const int j = (wave & 3) + 4 * k;
            if (j >= 13 * ky && j < 13 * ky + 13 && j < C4_APIECES) issue_a(qn < 4 ? t : tn, qn & 3, qn & 1, k);
          }
        }
        if (kx == 0) C4_STAMP(2);
      }
      C4_STAMP(3);
      if constexpr (C4_NODMA & 4)
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      C4_STAMP(4);
    }
#ifdef C4_STAMPS
    ++tcount;
#endif

    // ---- epilogue
    const long long item = 2 * tile + nh;
    if constexpr (MODE != 1) {
      bf16_t* yt = y + ((item * 8 + wave) * 16) * 512;  // [mi][np][lane][8]
      const bool interior = t.y0 + C4_TH <= H && t.x0 + C4_TW <= W;
#pragma unroll
      for (int np = 0; np < 4; ++np) {
        const float b0 = sbias[32 * np + r], b1 = sbias[32 * np + 16 + r];
        if (interior) {
          const f32x2 bb0 = {b0, b0}, bb1 = {b1, b1};
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) {
            const f32x4 v = acc[mi][2 * np], w = acc[mi][2 * np + 1];
            const f32x2 a0 = f32x2{v[0], v[1]} + bb0, a1 = f32x2{v[2], v[3]} + bb0;
            const f32x2 c0 = f32x2{w[0], w[1]} + bb1, c1 = f32x2{w[2], w[3]} + bb1;
            const u32x4 pk = {pack_bf16x2(a0.x, a0.y), pack_bf16x2(a1.x, a1.y), pack_bf16x2(c0.x, c0.y),
                              pack_bf16x2(c1.x, c1.y)};
            __builtin_nontemporal_store(pk, reinterpret_cast<u32x4*>(yt + ((mi * 4 + np) * 64 + lane) * 8));
            if constexpr (MODE == 0) {
              ssum[2 * np] += a0 + a1;
              ssq[2 * np] = __builtin_elementwise_fma(a0, a0, __builtin_elementwise_fma(a1, a1, ssq[2 * np]));
              ssum[2 * np + 1] += c0 + c1;
              ssq[2 * np + 1] = __builtin_elementwise_fma(c0, c0, __builtin_elementwise_fma(c1, c1, ssq[2 * np + 1]));
            }
          }
        } else {
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) {
            const bool row_ok = t.y0 + 2 * wave + (mi >> 1) < H;
            const int xb = t.x0 + (mi & 1) * 16 + 4 * g;
            uint32_t hv[8];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int nj = 2 * np + h;
              const float bias = h ? b1 : b0;
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const float av = acc[mi][nj][j] + bias;
                hv[4 * h + j] = (uint32_t)f32_to_bf16(av);
                if (MODE == 0 && row_ok && xb + j < W) {
                  ssum[nj].x += av;
                  ssq[nj].x = __builtin_fmaf(av, av, ssq[nj].x);
                }
              }
            }
            *reinterpret_cast<uint4*>(yt + ((mi * 4 + np) * 64 + lane) * 8) =
                make_uint4(hv[0] | (hv[1] << 16), hv[2] | (hv[3] << 16), hv[4] | (hv[5] << 16), hv[6] | (hv[7] << 16));
          }
        }
      }
    } else {
      // BN + ReLU of the bf16-rounded outputs (what the pool kernels read back from y), summed
      // per 16-px fragment row, then per pool bin in a fixed (wave, mi) order
      float* red = (float*)(smem + C4_RED_OFF);  // [wave][mi][128]
      if (tid < 32) {  // bin slot of fragment (wave, mi) = tid: (row bin - first) * 2 + (col bin - first), -1 off image
        const int row = t.y0 + 2 * (tid >> 2) + ((tid & 3) >> 1), col = t.x0 + 16 * (tid & 1);
        sslot[tid] = row < H ? (row / rh - t.y0 / rh) * 2 + (col / rw - t.x0 / rw) : -1;
      }
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < 8; ++nj) {
          const float bias = sbias[16 * nj + r];
          const float2 a = saff[16 * nj + r];
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float vb = bf16_to_f32(f32_to_bf16(acc[mi][nj][j] + bias));
            s += fmaxf(vb * a.x + a.y, 0.f);
          }
          s += __shfl_xor(s, 16);
          s += __shfl_xor(s, 32);
          if (g == 0) red[(wave * 4 + mi) * 128 + 16 * nj + r] = s;
        }
      __syncthreads();
      {
        const int slot = tid >> 7, c = tid & 127;
        float s = 0.f;
        for (int f = 0; f < 32; ++f)
          if (sslot[f] == slot) s += red[f * 128 + c];
        out[(item * 4 + slot) * 128 + c] = s;
      }
      // red / sslot are rewritten only after the next item's 12 step barriers
    }
  }
  if constexpr (MODE == 0) {
    // statistics: lanes of equal r, then the 8 waves in fixed order (the A slots are free: no
    // copy is in flight after the last item)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float* red = (float*)smem;  // [8 wave][128 n][2]
#pragma unroll
    for (int nj = 0; nj < 8; ++nj) {
      float a = ssum[nj].x + ssum[nj].y, q = ssq[nj].x + ssq[nj].y;
      a += __shfl_xor(a, 16);
      a += __shfl_xor(a, 32);
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      if (g == 0) {
        red[(wave * 128 + 16 * nj + r) * 2] = a;
        red[(wave * 128 + 16 * nj + r) * 2 + 1] = q;
      }
    }
    __syncthreads();
    for (int i = tid; i < C5 * 2; i += 512) {  // channel-major [256][gridDim.x][2] (k_bn_affine cm = 1)
      const int c = i >> 1, k = i & 1;
      float v = 0.f;
      if ((c >> 7) == nh)
        for (int w = 0; w < 8; ++w) v += red[(w * 128 + (c & 127)) * 2 + k];
      out[((long long)c * gridDim.x + blockIdx.x) * 2 + k] = v;
    }
  }
}

// BN + ReLU + AdaptiveAvgPool(4) partial sums over v4's y, 8-row half tiles: when every half tile
// lies inside one pool bin and no bins overlap (H % 32 == 0, W % 128 == 0).  A half tile of one
// channel half is 64 KiB contiguous (waves 4h .. 4h+3 of the item); thread t reads 16-byte chunk
// t + 256k (k = wave x mi), so it keeps channels (np, r) of both h of its lane's chunk -> with
// both channel halves 4 sums; the 4 pixel-quad lanes fold by shuffles at the end.  Split sp of
// bin reg takes the bin's half tiles sp, sp + POOL_SPLIT, ... (raster order).
__global__ __launch_bounds__(256) void k_rp_bn_relu_pool_v4_tiles(const bf16_t* __restrict__ y, int H, int W,
                                                                  const float2* __restrict__ aff,
                                                                  float* __restrict__ part) {
  __shared__ float red[C5];
  const int b = (int)gridDim.y - 1 - (int)blockIdx.y;  // images last-to-first (see conv5 v4's tile order)
  const int reg = blockIdx.x / POOL_SPLIT, sp = blockIdx.x % POOL_SPLIT;
  const int i = reg / 4, j = reg % 4;
  const int tiles_x = W / C4_TW, tiles_y = H / C4_TH;
  const int rhy = H / 32, rtx = W / 128;  // bin size in half tiles (8 rows) and tiles (32 cols)
  const int t = threadIdx.x, lane = t & 63, np = t >> 6, r = lane & 15;
  float2 af[2][2];
#pragma unroll
  for (int nh = 0; nh < 2; ++nh)
#pragma unroll
    for (int h = 0; h < 2; ++h) af[nh][h] = aff[nh * 128 + 32 * np + 16 * h + r];
  float acc[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
  for (int q = sp; q < rhy * rtx; q += POOL_SPLIT) {
    const int hy = i * rhy + q / rtx, tx = j * rtx + q % rtx;  // global half-tile row, tile column
    const long long tile = ((long long)b * tiles_y + (hy >> 1)) * tiles_x + tx;
#pragma unroll
    for (int nh = 0; nh < 2; ++nh) {
      const uint4* src = reinterpret_cast<const uint4*>(y + ((2 * tile + nh) * 8 + 4 * (hy & 1)) * 16 * 512) + t;
      uint4 v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const u32x4 xv = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + 256 * u));
        v[u] = make_uint4(xv.x, xv.y, xv.z, xv.w);
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const float lo = __uint_as_float(w[2 * h + e] << 16), hi = __uint_as_float(w[2 * h + e] & 0xffff0000u);
            acc[nh][h] += fmaxf(lo * af[nh][h].x + af[nh][h].y, 0.f);
            acc[nh][h] += fmaxf(hi * af[nh][h].x + af[nh][h].y, 0.f);
          }
      }
    }
  }
#pragma unroll
  for (int nh = 0; nh < 2; ++nh)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float v = acc[nh][h];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (lane < 16) red[nh * 128 + 32 * np + 16 * h + r] = v;
    }
  __syncthreads();
  part[(((long long)b * 16 + reg) * POOL_SPLIT + sp) * C5 + t] = red[t];
}

// The same over v4's y for any shape (bins may overlap, tiles may be ragged): as
// k_rp_bn_relu_pool_frag with v4's item addressing.
__global__ __launch_bounds__(256) void k_rp_bn_relu_pool_v4_frag(const bf16_t* __restrict__ y, int H, int W,
                                                                 const float2* __restrict__ aff,
                                                                 float* __restrict__ part) {
  __shared__ float red[2][C5];
  const int b = blockIdx.y, reg = blockIdx.x / POOL_SPLIT, sp = blockIdx.x % POOL_SPLIT;
  const int i = reg / 4, j = reg % 4;
  const int cp = threadIdx.x & 127, ql = threadIdx.x >> 7;
  const int nh = cp >> 6, np = (cp >> 4) & 3, r = cp & 15, n0 = nh * 128 + 32 * np + r, n1 = n0 + 16;
  const int ya = (i * H) / 4, yb = ((i + 1) * H + 3) / 4, xa = (j * W) / 4, xb = ((j + 1) * W + 3) / 4;
  const int rows = yb - ya;
  const int r0 = ya + (rows * sp) / POOL_SPLIT, r1 = ya + (rows * (sp + 1)) / POOL_SPLIT;
  const int qa = xa >> 2, nq = ((xb + 3) >> 2) - qa;
  const int tiles_x = (W + C4_TW - 1) / C4_TW, tiles_y = (H + C4_TH - 1) / C4_TH;
  const float2 a0 = aff[n0], a1 = aff[n1];
  float s0 = 0.f, s1 = 0.f;
  constexpr int PU = 8;
  int yy = r0, k = ql;
  while (k >= nq) {
    k -= nq;
    ++yy;
  }
  while (yy < r1) {
    uint4 v[PU];
    int xqs[PU];
    bool ok[PU];
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      ok[u] = yy < r1;
      const int ry = ok[u] ? yy : r1 - 1, xq = (qa + (ok[u] ? k : 0)) * 4;
      xqs[u] = xq;
      const long long tile = ((long long)b * tiles_y + ry / C4_TH) * tiles_x + xq / C4_TW;
      const int ly = ry % C4_TH, lx = xq % C4_TW;
      const int wave = ly >> 1, mi = (ly & 1) * 2 + (lx >> 4), g = (lx & 15) >> 2;
      v[u] = *reinterpret_cast<const uint4*>(y + (((((2 * tile + nh) * 8 + wave) * 4 + mi) * 4 + np) * 64 + g * 16 + r) * 8);
      k += 2;
      while (k >= nq) {
        k -= nq;
        ++yy;
      }
    }
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const uint32_t w0[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int xx = xqs[u] + e;
        if (ok[u] && xx >= xa && xx < xb) {
          const float c0 = bf16_to_f32((bf16_t)(e & 1 ? w0[e >> 1] >> 16 : w0[e >> 1] & 0xffff));
          const float c1 = bf16_to_f32((bf16_t)(e & 1 ? w0[2 + (e >> 1)] >> 16 : w0[2 + (e >> 1)] & 0xffff));
          s0 += fmaxf(c0 * a0.x + a0.y, 0.f);
          s1 += fmaxf(c1 * a1.x + a1.y, 0.f);
        }
      }
    }
  }
  red[ql][n0] = s0;
  red[ql][n1] = s1;
  __syncthreads();
  const int c = threadIdx.x;
  part[(((long long)b * 16 + reg) * POOL_SPLIT + sp) * C5 + c] = red[0][c] + red[1][c];
}

// MODE 1's pool: pooled[b][c][bin] = the sum of the bin's item partials (tiles in raster order)
// / the bin's pixel count.  grid (16 bins, B), thread = channel.
__global__ __launch_bounds__(256) void k_rp_pool_finish_v4(const float* __restrict__ ip, int B, int H, int W,
                                                           float* __restrict__ pooled) {
  const int b = blockIdx.y, reg = blockIdx.x, i = reg / 4, j = reg % 4, c = threadIdx.x;
  const int nh = c >> 7, cc = c & 127;
  const int rh = H >> 2, rw = W >> 2;
  const int tiles_x = W / C4_TW, tiles_y = (H + C4_TH - 1) / C4_TH;
  const int ty0 = (i * rh) / C4_TH, ty1 = ((i + 1) * rh - 1) / C4_TH;
  const int tx0 = (j * rw) / C4_TW, tx1 = ((j + 1) * rw - 1) / C4_TW;
  float s = 0.f;
  for (int ty = ty0; ty <= ty1; ++ty)
    for (int tx = tx0; tx <= tx1; ++tx) {
      const int slot = (i - (ty * C4_TH) / rh) * 2 + (j - (tx * C4_TW) / rw);
      const long long tile = ((long long)b * tiles_y + ty) * tiles_x + tx;
      s += ip[((2 * tile + nh) * 4 + slot) * 128 + cc];
    }
  pooled[((long long)b * C5 + c) * 16 + reg] = s / (float)(rh * rw);
}

// ------------------------------------------------------------------ tail: conv 256->512 on 4x4
__global__ void k_rp_pool_finish(const float* __restrict__ part, int B, int H, int W, float* __restrict__ pooled) {
  // pooled[b][256][16] = mean over the region = sum of the split partials / count
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * C5 * 16) return;
  const int bb = e / (C5 * 16), c = (e / 16) % C5, reg = e % 16;
  const int i = reg / 4, j = reg % 4;
  const int cnt = (((i + 1) * H + 3) / 4 - (i * H) / 4) * (((j + 1) * W + 3) / 4 - (j * W) / 4);
  float s = 0.f;
  for (int sp = 0; sp < POOL_SPLIT; ++sp) s += part[(((long long)bb * 16 + reg) * POOL_SPLIT + sp) * C5 + c];
  pooled[e] = s / (float)cnt;
}

// Tail conv chunks: the 16-channel groups whose partial sums the fused kernel adds in order.
constexpr int TC_C = 16, TC_CHUNKS = C5 / TC_C;

__device__ __forceinline__ float hash_uniform(unsigned long long seed, unsigned long long idx) {
  unsigned long long z = seed + idx * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// Tail conv 256->512 + BN(512) + ReLU + AdaptiveAvgPool2d(1) in one launch (k_rp_tail_conv +
// k_rp_tail_bn, bitwise the same values): workgroup = two output channels over ALL 256 input
// channels, so the BN of its channels needs no other workgroup.  LDS holds 8 images' pooled maps
// unpadded [256 c][8 b][16] (128 KB: out-of-map taps read 0.f, the padded copy's value) and the
// two channels' filters [256 c][3 ky][2 o][4]; 512 threads, thread = (chunk k, image b, row py): 2 o x
// 4 px of the 16-channel chunk k, accumulated in tail_conv's order
// (cl, ky, kx; mul then add); then z = b6 + the 16 chunk partials in chunk order (tail_bn's
// zval) and tail_bn's statistics / running-stat update / ReLU / mean over the 16 positions, one
// wave per channel.  256 workgroups (one per CU), eight waves each (two per SIMD: the LDS reads of
// one wave under the other's arithmetic).
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int TB_SP = C5 * 8 * 16;                  // floats: pooled, 8 images
constexpr int TB_SW = C5 * 3 * 2 * 4;               // floats: filters of 2 channels
constexpr int TB_ZS = 2 * 32 * 16;                  // floats: z of the 2 channels, B <= 32
constexpr size_t TB_SMEM = (size_t)(TB_SP + TB_SW + TB_ZS) * 4;
static_assert(TB_SMEM <= 163840 && TC_CHUNKS * 2 * 8 * 16 <= TB_SP, "tail conv+bn LDS");
__global__ __launch_bounds__(512) void k_rp_tail_convbn(const float* __restrict__ pooled, int B, int training,
                                                        float momentum, const char* __restrict__ blob, Layout L,
                                                        BnPtrs bn, float* __restrict__ feat) {
  extern __shared__ __attribute__((aligned(16))) float tsm[];
  float* sp = tsm;                  // [256 c][8 b][16]; later the chunk partials [16 k][2 o][8 b][16]
  float* sw = tsm + TB_SP;          // [256 c][3 ky][2 o][4]
  float* zs = sw + TB_SW;           // [2 o][B * 16]
  const int tid = threadIdx.x, o0 = blockIdx.x * 2;
  const float* w6 = (const float*)(blob + L.w6);
  {
    float wv[2 * C5 * 9 / 512];
#pragma unroll
    for (int q = 0; q < 2 * C5 * 9 / 512; ++q) wv[q] = w6[(long long)o0 * C5 * 9 + tid + 512 * q];
#pragma unroll
    for (int q = 0; q < 2 * C5 * 9 / 512; ++q) {
      const int i = tid + 512 * q, ol = i / (C5 * 9), r = i % (C5 * 9), c = r / 9, tap = r % 9;
      sw[((c * 3 + tap / 3) * 2 + ol) * 4 + tap % 3] = wv[q];
    }
  }
  const int ck = tid >> 5, bl = (tid >> 2) & 7, py = tid & 3;
  for (int b0 = 0; b0 < B; b0 += 8) {
    __syncthreads();  // previous group's partial sums consumed
    {
      constexpr int NQ = TB_SP / 4 / 512;  // float4 per thread
      float4 pv[NQ];
#pragma unroll
      for (int u = 0; u < NQ; ++u) {
        const int e = tid + 512 * u, q = e & 3, c = (e >> 2) & (C5 - 1), b = b0 + (e >> 10);
        pv[u] = b < B ? *reinterpret_cast<const float4*>(pooled + ((long long)b * C5 + c) * 16 + 4 * q)
                      : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < NQ; ++u) {
        const int e = tid + 512 * u, q = e & 3, c = (e >> 2) & (C5 - 1), b = e >> 10;
        *reinterpret_cast<float4*>(sp + (c * 8 + b) * 16 + 4 * q) = pv[u];
      }
    }
    __syncthreads();
    // pixel pairs in two-wide vectors: packed multiplies and adds (v_pk_mul_f32 / v_pk_add_f32),
    // each lane's arithmetic the scalar mul-then-add of tail_conv
    f32x2 acc[2][2];
#pragma unroll
    for (int ol = 0; ol < 2; ++ol)
#pragma unroll
      for (int x = 0; x < 2; ++x) acc[ol][x] = f32x2{0.f, 0.f};
#pragma unroll 4
    for (int cl = 0; cl < TC_C; ++cl) {
      const int c = ck * TC_C + cl;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int y = py + ky - 1;
        float r[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (y >= 0 && y < 4) {
          const float4 v = *reinterpret_cast<const float4*>(sp + (c * 8 + bl) * 16 + 4 * y);
          r[1] = v.x; r[2] = v.y; r[3] = v.z; r[4] = v.w;
        }
        const float4 w0 = *reinterpret_cast<const float4*>(sw + ((c * 3 + ky) * 2 + 0) * 4);
        const float4 w1 = *reinterpret_cast<const float4*>(sw + ((c * 3 + ky) * 2 + 1) * 4);
        const float wa[3] = {w0.x, w0.y, w0.z}, wb[3] = {w1.x, w1.y, w1.z};
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
#pragma unroll
          for (int x = 0; x < 2; ++x) {
            const f32x2 rv = f32x2{r[2 * x + kx], r[2 * x + 1 + kx]};
            acc[0][x] += f32x2{wa[kx], wa[kx]} * rv;
            acc[1][x] += f32x2{wb[kx], wb[kx]} * rv;
          }
      }
    }
    __syncthreads();  // every thread's pooled reads done: the region takes the chunk partials
#pragma unroll
    for (int ol = 0; ol < 2; ++ol)
      *reinterpret_cast<float4*>(sp + ((ck * 2 + ol) * 8 + bl) * 16 + 4 * py) =
          make_float4(acc[ol][0].x, acc[ol][0].y, acc[ol][1].x, acc[ol][1].y);
    __syncthreads();
    if (tid < 256) {  // z = b6 + the chunk partials in chunk order: thread = (o, image, position)
      const int ol = tid >> 7, b = (tid >> 4) & 7, pos = tid & 15;
      float z = ((const float*)(blob + L.b6))[o0 + ol];
#pragma unroll
      for (int k = 0; k < TC_CHUNKS; ++k) z += sp[((k * 2 + ol) * 8 + b) * 16 + pos];
      if (b0 + b < B) zs[ol * (B * 16) + (b0 + b) * 16 + pos] = z;
    }
  }
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63;
  if (wave >= 2) return;
  const int c = o0 + wave, n = B * 16;
  const float* zc = zs + wave * n;
  float mean, var;
  if (training) {
    double s = 0.0, q = 0.0;
    for (int bp = lane; bp < n; bp += 64) {
      const double v = zc[bp];
      s += v;
      q += v * v;
    }
    s = wave_sum_dbl(s);
    q = wave_sum_dbl(q);
    const double nn = (double)n, m = s / nn;
    double v = q / nn - m * m;
    if (v < 0.0) v = 0.0;
    mean = (float)m;
    var = (float)v;
    if (lane == 0) {
      float* rm = bn.p[5 * 4 + 2];
      float* rv = bn.p[5 * 4 + 3];
      const double unb = nn > 1.0 ? v * nn / (nn - 1.0) : v;
      rm[c] = (1.f - momentum) * rm[c] + momentum * mean;
      rv[c] = (1.f - momentum) * rv[c] + momentum * (float)unb;
    }
  } else {
    mean = bn.p[5 * 4 + 2][c];
    var = bn.p[5 * 4 + 3][c];
  }
  const float sc = bn.p[5 * 4 + 0][c] / sqrtf(var + BN_EPS), sh = bn.p[5 * 4 + 1][c] - mean * sc;
  for (int base = 0; base < n; base += 64) {  // n is a multiple of 16: 16-lane groups are whole images
    const int bp = base + lane;
    float r = bp < n ? fmaxf(zc[bp] * sc + sh, 0.f) : 0.f;
    r += __shfl_xor(r, 8);
    r += __shfl_xor(r, 4);
    r += __shfl_xor(r, 2);
    r += __shfl_xor(r, 1);
    if (bp < n && (lane & 15) == 0) feat[(long long)(bp >> 4) * C6 + c] = r / 16.f;
  }
}

// Linear 512 -> 128 + ReLU + Dropout(0.3): one workgroup per output o, thread = 2 k's for all
// images, fixed-order block reduction per image.
__global__ __launch_bounds__(256) void k_rp_tail_fc1(const float* __restrict__ feat, int B, int training,
                                                     const char* __restrict__ blob, Layout L,
                                                     unsigned long long seed, const unsigned long long* seed_ctr,
                                                     float* __restrict__ h1) {
  __shared__ float red[4][32];
  if (seed_ctr) seed += *seed_ctr;
  const int o = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const float* w7 = (const float*)(blob + L.w7);
  const float wa = w7[o * 512 + t], wb = w7[o * 512 + t + 256];
  // all images' feature loads in flight before the reductions (B <= 32)
  float fa[32], fb[32];
#pragma unroll
  for (int b = 0; b < 32; ++b)
    if (b < B) {
      fa[b] = feat[(long long)b * C6 + t];
      fb[b] = feat[(long long)b * C6 + t + 256];
    }
#pragma unroll
  for (int b = 0; b < 32; ++b)
    if (b < B) {
      float s = wa * fa[b] + wb * fb[b];
      s = wave_sum(s);
      if (lane == 0) red[wv][b] = s;
    }
  __syncthreads();
  if (t < B) {
    const float* b7 = (const float*)(blob + L.b7);
    float s = b7[o] + (((red[0][t] + red[1][t]) + red[2][t]) + red[3][t]);
    s = fmaxf(s, 0.f);
    const int e = t * 128 + o;
    if (training) s = hash_uniform(seed, e) < 0.3f ? 0.f : s / 0.7f;  // Dropout(0.3)
    h1[t * 128 + o] = s;
  }
}

// Linear 128 -> 64 + ReLU + Dropout(0.2), Linear 64 -> 32 + ReLU, Linear 32 -> 1, sigmoid range
// map; one workgroup, the weights row-major in LDS (padded rows: lanes walk output rows).
__global__ __launch_bounds__(512) void k_rp_tail_head(const float* __restrict__ h1g, int B, int training,
                                                      const char* __restrict__ blob, Layout L,
                                                      unsigned long long seed, unsigned long long* seed_ctr,
                                                      float* __restrict__ ratio) {
  // the weights stay row-major in LDS with one float of row padding: the staging writes and the
  // per-output row reads (lanes = outputs, rows 129 / 65 floats apart) are both conflict-free
  // (the transposed images this replaced took 32-way conflicts on every staging write)
  __shared__ float w8s[64][129], w9s[32][65];
  const unsigned long long ctr = seed_ctr ? *seed_ctr : 0ull;
  seed += ctr;
  __shared__ float h1[32][128], h2[32][64], h3[32][32];
  const float* w8 = (const float*)(blob + L.w8);
  const float* b8 = (const float*)(blob + L.b8);
  const float* w9 = (const float*)(blob + L.w9);
  const float* b9 = (const float*)(blob + L.b9);
  const float* w10 = (const float*)(blob + L.w10);
  const float* b10 = (const float*)(blob + L.b10);
  {  // every staging load in flight together, then the LDS writes
    float a8[16], a9[4], ah[8];
#pragma unroll
    for (int q = 0; q < 16; ++q) a8[q] = w8[threadIdx.x + 512 * q];
#pragma unroll
    for (int q = 0; q < 4; ++q) a9[q] = w9[threadIdx.x + 512 * q];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (threadIdx.x + 512 * q < B * 128) ah[q] = h1g[threadIdx.x + 512 * q];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = threadIdx.x + 512 * q;
      w8s[i / 128][i % 128] = a8[q];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = threadIdx.x + 512 * q;
      w9s[i / 64][i % 64] = a9[q];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = threadIdx.x + 512 * q;
      if (i < B * 128) h1[i / 128][i % 128] = ah[q];
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < B * 64; e += 512) {
    const int bb = e / 64, o = e % 64;
    float s = b8[o];
    for (int k = 0; k < 128; ++k) s += w8s[o][k] * h1[bb][k];
    s = fmaxf(s, 0.f);
    if (training) s = hash_uniform(seed ^ 0x5555ull, e) < 0.2f ? 0.f : s / 0.8f;  // Dropout(0.2)
    h2[bb][o] = s;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < B * 32; e += 512) {
    const int bb = e / 32, o = e % 32;
    float s = b9[o];
    for (int k = 0; k < 64; ++k) s += w9s[o][k] * h2[bb][k];
    h3[bb][o] = fmaxf(s, 0.f);
  }
  __syncthreads();
  // every read of the counter (k_rp_tail_fc1, this kernel's prologue) precedes this store: the
  // next forward (or graph replay) draws fresh dropout masks
  if (training && seed_ctr && threadIdx.x == 0) *seed_ctr = ctr + 1ull;
  if (threadIdx.x < B) {
    const int bb = threadIdx.x;
    float s = b10[0];
    for (int k = 0; k < 32; ++k) s += w10[k] * h3[bb][k];
    ratio[bb] = 0.01f + (0.5f - 0.01f) * (1.f / (1.f + expf(-s)));
  }
}

// zero the padding of conv5 v4's input planes (everything of [PH][PW] outside the image):
// grid (8, B * 4 planes), 16 bytes per thread and iteration
__device__ void c4_pad_body(bf16_t* __restrict__ att, int H, int W, int bx, int plane, int nbx) {
  const int PH = c4_ph(H), PW = c4_pw(W);
  bf16_t* pl = att + (long long)plane * PH * PW * 32;
  const int edge_rows = PH - H, side = PW - W;  // full pad rows (top + bottom), pad pixels per image row
  const long long full = (long long)edge_rows * PW * 4, part = (long long)H * side * 4;  // 16-byte chunks
  for (long long i = bx * 256 + threadIdx.x; i < full + part; i += 256LL * nbx) {
    long long px;
    if (i < full) {
      const long long c = i >> 2;
      const int rr = (int)(c / PW), cc = (int)(c % PW);
      px = (long long)(rr == 0 ? 0 : H + rr) * PW + cc;
    } else {
      const long long c = (i - full) >> 2;
      const int rr = (int)(c / side), k = (int)(c % side);
      px = (long long)(rr + 1) * PW + (k == 0 ? 0 : W + k);
    }
    *reinterpret_cast<uint4*>(pl + px * 32 + 8 * (i & 3)) = make_uint4(0u, 0u, 0u, 0u);
  }
}

__global__ __launch_bounds__(256) void k_c4_pad_zero(bf16_t* __restrict__ att, int H, int W) {
  c4_pad_body(att, H, W, blockIdx.x, blockIdx.y, gridDim.x);
}

struct Ws {  // workspace carve
  size_t aff1, aff2, aff5, slab, att, y, part, pooled, feat, h1, fold, stem, total;
};

inline int chain_grid(int B, int H, int W) {
  const long long nt = (long long)B * ((W + CH_TW - 1) / CH_TW) * ((H + CH_TH - 1) / CH_TH);
  return (int)std::min<long long>(nt, 2048);
}
// one 512-thread workgroup per CU (LDS-resident weights); phase 0 two
inline int chain_grid_v2(int B, int H, int W, int phase = 1) {
  const long long nt = (long long)B * ((W + C2W_TW - 1) / C2W_TW) * ((H + C2W_TH - 1) / C2W_TH);
  return (int)std::min<long long>(nt, phase == 0 ? 512 : 256);
}
inline int conv_grid(int B, int H, int W) {
  const long long nt = (long long)B * ((W + CV_TW - 1) / CV_TW) * ((H + CV_TH - 1) / CV_TH);
  return (int)std::min<long long>(nt, 512);
}
inline int device_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      v = 256;
    return v > 0 ? v : 256;
  }();
  return n;
}
// k_rp_gate: persistent, one 512-thread workgroup per CU over 8x32-pixel tiles
inline int gate_grid(int B, int H, int W) {
  return (int)std::min<long long>((long long)B * ((W + 31) / 32) * ((H + 7) / 8), device_cus());
}

inline long long conv4_tiles(int B, int H, int W) {
  return (long long)B * ((W + C4_TW - 1) / C4_TW) * ((H + C4_TH - 1) / C4_TH);
}
// persistent, one 147 KB-LDS workgroup per CU, in pairs (the two channel halves of a tile)
inline int conv4_grid(int B, int H, int W) { return 2 * (int)std::min<long long>(conv4_tiles(B, H, W), device_cus() / 2); }
// eval: BN + ReLU + AdaptiveAvgPool(4) in conv5's epilogue when the pool bins do not overlap and
// every 16-px fragment row of a 16x32 tile lies in one bin, a tile in at most 2 x 2 bins
inline bool conv4_pool_fused(int H, int W) { return H % 4 == 0 && W % 64 == 0 && H >= 64 && W >= 128; }

inline Ws make_ws(int es, int B, int H, int W) {
  Ws w;
  size_t o = 0;
  auto seg = [&](size_t bytes) {
    size_t r = o;
    o += align256(bytes);
    return r;
  };
  const size_t P = (size_t)B * H * W;
  const int slab_rows = std::max(std::max(chain_grid(B, H, W), 8 * chain_grid_v2(B, H, W, 0)),
                                 std::max(conv_grid(B, H, W), conv4_grid(B, H, W)));
  w.aff1 = seg(STEM_C * sizeof(float2));
  w.aff2 = seg(FUS_C * sizeof(float2));
  w.aff5 = seg(C5 * sizeof(float2));
  w.slab = seg((size_t)slab_rows * C5 * 2 * sizeof(float));
  w.att = seg(es == 2 ? (size_t)B * c4_ph(H) * c4_pw(W) * FUS_C * 2 : P * FUS_C * es);
  w.y = seg(es == 2 ? (size_t)conv4_tiles(B, H, W) * C4_TH * C4_TW * C5 * 2 : P * C5 * es);
  w.part = seg((size_t)B * 16 * POOL_SPLIT * C5 * sizeof(float));
  w.pooled = seg((size_t)B * C5 * 16 * sizeof(float));
  w.feat = seg((size_t)B * C6 * sizeof(float));
  w.h1 = seg((size_t)B * 128 * sizeof(float));
  w.fold = seg(es == 2 ? FOLD_BYTES : 0);
  w.stem = seg(es == 2 && stem_moments_ok(H, W) ? stem_ws(B, H, W).total : 0);
  w.total = o;
  return w;
}

template <typename T>
int ratio_forward(int training, float momentum, const float* depth3, long long bstride, int B, int H, int W,
                  const char* blob, const BnPtrs& bn, unsigned long long seed, unsigned long long* seed_ctr,
                  float* ratio, char* ws, int flags, hipStream_t s) {
  const Layout L = make_layout(sizeof(T));
  const Ws w = make_ws(sizeof(T), B, H, W);
  float2* aff1 = (float2*)(ws + w.aff1);
  float2* aff2 = (float2*)(ws + w.aff2);
  float2* aff5 = (float2*)(ws + w.aff5);
  float* slab = (float*)(ws + w.slab);
  T* att = (T*)(ws + w.att);
  T* y = (T*)(ws + w.y);
  float* part = (float*)(ws + w.part);
  float* pooled = (float*)(ws + w.pooled);
  float* feat = (float*)(ws + w.feat);
  float* h1 = (float*)(ws + w.h1);
  char* fold = ws + w.fold;
  const double P = (double)B * H * W;
  const bool v2 = sizeof(T) == 2;
  const int gch = v2 ? chain_grid_v2(B, H, W) : chain_grid(B, H, W);
  const int gch0 = v2 ? chain_grid_v2(B, H, W, 0) : gch;
  const int nslab_ch = v2 ? gch * 8 : gch;    // v2 writes one slab row per wave
  const int nslab_ch0 = v2 ? gch0 * 8 : gch;  // phase 0 (stem statistics)
  if (v2) {
    static const hipError_t attr[3] = {
        hipFuncSetAttribute((const void*)k_rp_chain_v2<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c2w_smem<0>()),
        hipFuncSetAttribute((const void*)k_rp_chain_v2<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c2w_smem<1>()),
        hipFuncSetAttribute((const void*)k_rp_chain_v2<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c2w_smem<2>())};
    for (int i = 0; i < 3; ++i)
      if (attr[i] != hipSuccess) return (int)attr[i];
  }
#define CHAIN_LAUNCH(PH, A1, A2, SL, OUT)                                                                          \
  do {                                                                                                            \
    if (RGBD_DIAG_ON && v2 && c2_stamps_on && PH < 2) {                                                           \
      static const hipError_t sattr = hipFuncSetAttribute((const void*)k_rp_chain_v2<PH, RGBD_DIAG_ON>,                  \
                                                          hipFuncAttributeMaxDynamicSharedMemorySize,             \
                                                          (int)c2w_smem<PH>());                                   \
      (void)sattr;                                                                                                \
      k_rp_chain_v2<PH, RGBD_DIAG_ON><<<PH == 0 ? gch0 : gch, 512, c2w_smem<PH>(), s>>>(                                 \
          depth3, bstride, B, H, W, blob, L, A1, A2, fold, SL, (bf16_t*)(OUT));                                   \
    } else if (v2)                                                                                                \
      k_rp_chain_v2<PH><<<PH == 0 ? gch0 : gch, 512, c2w_smem<PH>(), s>>>(depth3, bstride, B, H, W, blob, L, A1, A2, \
                                                                        fold, SL, (bf16_t*)(OUT));                \
    else                                                                                                          \
      k_rp_chain<T, PH><<<gch, 256, 0, s>>>(depth3, bstride, B, H, W, blob, L, A1, A2, SL, (T*)(OUT));            \
  } while (0)
  // stem BNs (scale1/2/3, 64 channels each, concatenated :1463)
  if (training && v2 && stem_moments_ok(H, W)) {  // bf16 train: the moments of the windows (no stem pass)
    // (+ the BN1 fold and conv5 v4's input padding)
    const int e = stem_bn_moments(depth3, bstride, B, H, W, blob, L, momentum, bn, aff1, fold, (bf16_t*)att,
                                  ws + w.stem, s);
    if (e != RGBD_OK) return e;
  } else {
    if (training) CHAIN_LAUNCH(0, nullptr, nullptr, slab, nullptr);
    k_bn_affine_stem<<<STEM_C, 256, 0, s>>>(slab, nslab_ch0, P, training, momentum, bn, aff1);
    if (v2) k_rp_fold<<<STEM_C, 256, 0, s>>>(blob, L, aff1, 1, fold);  // BN1 -> W1', b1'
    if (v2) k_c4_pad_zero<<<dim3(8, B * 4), 256, 0, s>>>((bf16_t*)att, H, W);
  }
  // fusion BN; train + bf16: phase 1 also stores its raw fusion output (in the conv5 output
  // buffer, which is dead until conv5) for k_rp_gate
  // flags & RGBD_RATIO_F_PHASE2: train mode through phase 2 instead of the gate kernel (a test
  // compares the two paths' gated features)
  const bool gate = v2 && training && !(flags & RGBD_RATIO_F_PHASE2);
  bf16_t* fus = (bf16_t*)y;
  if (training) CHAIN_LAUNCH(1, aff1, nullptr, slab, gate ? (void*)fus : nullptr);
  k_bn_affine<<<FUS_C, 256, 0, s>>>(slab, nslab_ch, FUS_C, 0, FUS_C, P, training, momentum, bn.p[12], bn.p[13], bn.p[14],
                                bn.p[15], aff2, v2 ? 1 : 0);  // chain v2 phase 1: channel-major
  if (v2 && !gate) k_rp_fold<<<FUS_C, 256, 0, s>>>(blob, L, aff2, 2, fold);  // BN2 -> W2', b2'
  // gated attention features
  {
    TimerScope ts("rp_chain", s);
    if (gate) {
      static const hipError_t gattr =
          hipFuncSetAttribute((const void*)k_rp_gate, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GT_SMEM);
      if (gattr != hipSuccess) return (int)gattr;
      const int gg = gate_grid(B, H, W);
      k_rp_gate<<<gg, 512, GT_SMEM, s>>>(fus, B, H, W, blob, L, aff2, (bf16_t*)att);
    } else {
      CHAIN_LAUNCH(2, aff1, aff2, nullptr, att);
    }
  }
  // conv5 + its BN statistics (train) / BN + ReLU + pool (eval, v4 MODE 1)
  int gcv;
  if constexpr (sizeof(T) == 2) {
    // eval: the BN affine from the running statistics first (the fused epilogue applies it)
    const int mode = training ? 0 : (conv4_pool_fused(H, W) ? 1 : 2);
    if (!training)
      k_bn_affine<<<C5, 256, 0, s>>>(slab, 0, C5, 0, C5, P, 0, momentum, bn.p[16], bn.p[17], bn.p[18], bn.p[19],
                                     aff5);
    {
      TimerScope ts("rp_conv3x3", s);
      gcv = conv4_grid(B, H, W);
      const int xcd = gcv % 16 == 0;
      float* ip = (float*)y;  // MODE 1: per-item bin partials (y is not written)
      auto go = [&](auto kern, float* out) {
        static const hipError_t sattr =
            hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)C4_SMEM);
        if (sattr != hipSuccess) return (int)sattr;
        kern<<<gcv, 512, C4_SMEM, s>>>((const bf16_t*)att, B, H, W, blob, L, aff5, (bf16_t*)y, out, xcd);
        return (int)hipSuccess;
      };
      const int e = mode == 0 ? go(k_rp_conv5_v4<0>, slab) : mode == 1 ? go(k_rp_conv5_v4<1>, ip) : go(k_rp_conv5_v4<2>, nullptr);
      if (e != hipSuccess) return e;
    }
    if (training)  // conv5 v4 MODE 0: channel-major
      k_bn_affine<<<C5, 256, 0, s>>>(slab, gcv, C5, 0, C5, P, training, momentum, bn.p[16], bn.p[17], bn.p[18],
                                     bn.p[19], aff5, 1);
    if (mode == 1) {
      k_rp_pool_finish_v4<<<dim3(16, B), 256, 0, s>>>((const float*)y, B, H, W, pooled);
    } else {
      if (H % 32 == 0 && W % 128 == 0)
        k_rp_bn_relu_pool_v4_tiles<<<dim3(16 * POOL_SPLIT, B), 256, 0, s>>>((const bf16_t*)y, H, W, aff5, part);
      else
        k_rp_bn_relu_pool_v4_frag<<<dim3(16 * POOL_SPLIT, B), 256, 0, s>>>((const bf16_t*)y, H, W, aff5, part);
      k_rp_pool_finish<<<ceil_div((long long)B * C5 * 16, 256), 256, 0, s>>>(part, B, H, W, pooled);
    }
  } else {
    {
      TimerScope ts("rp_conv3x3", s);
      gcv = conv_grid(B, H, W);
      k_rp_conv3x3<T><<<dim3(gcv, C5 / CV_BN), 256, 0, s>>>(att, B, H, W, blob, L, y, slab);
    }
    k_bn_affine<<<C5, 256, 0, s>>>(slab, gcv, C5, 0, C5, P, training, momentum, bn.p[16], bn.p[17], bn.p[18],
                                   bn.p[19], aff5);
    k_rp_bn_relu_pool<T><<<dim3(16 * POOL_SPLIT, B), 256, 0, s>>>(y, H, W, aff5, part);
    k_rp_pool_finish<<<ceil_div((long long)B * C5 * 16, 256), 256, 0, s>>>(part, B, H, W, pooled);
  }
  {
    static const hipError_t tattr =
        hipFuncSetAttribute((const void*)k_rp_tail_convbn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)TB_SMEM);
    if (tattr != hipSuccess) return (int)tattr;
    k_rp_tail_convbn<<<C6 / 2, 512, TB_SMEM, s>>>(pooled, B, training, momentum, blob, L, bn, feat);
  }
  k_rp_tail_fc1<<<128, 256, 0, s>>>(feat, B, training, blob, L, seed, seed_ctr, h1);
  k_rp_tail_head<<<1, 512, 0, s>>>(h1, B, training, blob, L, seed, seed_ctr, ratio);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // namespace

extern "C" {

#ifdef RGBD_DIAG
int rgbd_debug_chain_stamps(void* buf) {
  unsigned long long* p = (unsigned long long*)buf;
  const hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_c2_stamps), &p, sizeof(p));
  if (e != hipSuccess) return (int)e;
  c2_stamps_on = p != nullptr;
  return RGBD_OK;
}

int rgbd_debug_stem_lag_stamps(void* buf) {
  unsigned long long* p = (unsigned long long*)buf;
  const hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_sl_stamps), &p, sizeof(p));
  if (e != hipSuccess) return (int)e;
  sl_stamps_on = p != nullptr;
  return RGBD_OK;
}

int rgbd_debug_conv5_stamps(void* buf) {
  unsigned long long* p = (unsigned long long*)buf;
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_c4_stamps), &p, sizeof(p));
}
#endif

size_t rgbd_ratio_packed_size(int dtype) { return make_layout(dtype == RGBD_BF16 ? 2 : 4).total; }

int rgbd_ratio_pack(int dtype, const float* const* weights_host, void* packed, void* stream) {
  RGBD_REQUIRE(weights_host && packed, RGBD_E_ARG);
  WPtrs w;
  for (int i = 0; i < RGBD_RATIO_NW; ++i) {
    RGBD_REQUIRE(weights_host[i], RGBD_E_ARG);
    w.p[i] = weights_host[i];
  }
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_F32)
    k_rp_pack<float><<<1024, 256, 0, s>>>(w, (char*)packed, make_layout(4));
  else if (dtype == RGBD_BF16)
    k_rp_pack<bf16_t><<<1024, 256, 0, s>>>(w, (char*)packed, make_layout(2));
  else
    return RGBD_E_DTYPE;
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

size_t rgbd_ratio_features_offset(int dtype, int B, int H, int W) {
  return make_ws(dtype == RGBD_BF16 ? 2 : 4, B > 0 ? B : 1, H > 0 ? H : 1, W > 0 ? W : 1).att;
}


size_t rgbd_ratio_pooled_offset(int dtype, int B, int H, int W) {
  return make_ws(dtype == RGBD_BF16 ? 2 : 4, B > 0 ? B : 1, H > 0 ? H : 1, W > 0 ? W : 1).pooled;
}

size_t rgbd_ratio_workspace_size(int dtype, int B, int H, int W) {
  return make_ws(dtype == RGBD_BF16 ? 2 : 4, B > 0 ? B : 1, H > 0 ? H : 1, W > 0 ? W : 1).total;
}

int rgbd_ratio_forward(int dtype, int training, float momentum, const float* depth3, long long batch_stride,
                       int B, int H, int W, const void* packed, float* const* bn_host, unsigned long long seed,
                       unsigned long long* seed_counter, float* ratio, void* ws, void* stream) {
  return rgbd_ratio_forward_ex(dtype, training, momentum, depth3, batch_stride, B, H, W, packed, bn_host, seed,
                               seed_counter, ratio, ws, 0, stream);
}

int rgbd_ratio_forward_ex(int dtype, int training, float momentum, const float* depth3, long long batch_stride,
                          int B, int H, int W, const void* packed, float* const* bn_host, unsigned long long seed,
                          unsigned long long* seed_counter, float* ratio, void* ws, int flags, void* stream) {
  RGBD_REQUIRE((flags & ~RGBD_RATIO_F_PHASE2) == 0, RGBD_E_ARG);
  RGBD_REQUIRE(depth3 && packed && bn_host && ratio && ws, RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && H > 0 && W > 0, RGBD_E_ARG);
  RGBD_REQUIRE(B <= 32, RGBD_E_SHAPE);  // k_rp_tail_fc1 / k_rp_tail_head hold the batch in LDS
  RGBD_REQUIRE((long long)B * ((H + 7) / 8) * ((W + 31) / 32) < (1ll << 30), RGBD_E_SHAPE);  // 32-bit tile indices
  BnPtrs bn;
  for (int i = 0; i < RGBD_RATIO_NBN * 4; ++i) {
    RGBD_REQUIRE(bn_host[i], RGBD_E_ARG);
    bn.p[i] = bn_host[i];
  }
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_F32)
    return ratio_forward<float>(training, momentum, depth3, batch_stride, B, H, W, (const char*)packed, bn, seed,
                                seed_counter, ratio, (char*)ws, flags, s);
  if (dtype == RGBD_BF16)
    return ratio_forward<bf16_t>(training, momentum, depth3, batch_stride, B, H, W, (const char*)packed, bn, seed,
                                 seed_counter, ratio, (char*)ws, flags, s);
  return RGBD_E_DTYPE;
}

}  // extern "C"
