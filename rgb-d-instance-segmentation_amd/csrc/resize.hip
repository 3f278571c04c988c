// a11: the resizes of the reference's data map for frames that are not at model
// resolution (mask2former/utils/dataloader.py:405-414, map_10channel_case2):
//   * the image processor's PIL resize (Mask2FormerImageProcessor, PIL backend):
//     BILINEAR on the uint8 colour and depth-as-RGB images, NEAREST on the uint8 instance map;
//     restated from Pillow's libImaging/Resample.c and Geometry.c, bit-exact to Pillow;
//   * cv2.resize(depth, (h, w), INTER_LINEAR) of the 'L' depth (OpenCV 4 fixed-point linear
//     resize of 8-bit data; OpenCV is absent here: parity unpinned).
// Every table is computed on the device with the reference's double arithmetic (+, *, /, casts
// only: IEEE-identical to the host C), so nothing crosses PCIe and the calls stay capturable.
//
// PIL bilinear (Resample.c): per output index o along an axis of n_in -> n_out,
//   scale = n_in / n_out, fs = max(scale, 1), support = fs, center = (o + 0.5) scale,
//   xmin = max((int)(center - support + 0.5), 0), xmax = min((int)(center + support + 0.5), n_in),
//   w_x = max(0, 1 - |(x + xmin - center + 0.5) / fs|), normalised by their sum, then
//   k = (int)(w * 2^22 +- 0.5) (PRECISION_BITS 22);
//   out = clip8((2^21 + sum_x in[xmin + x] k_x) >> 22), horizontal pass first into uint8, then
//   vertical (ImagingResampleInner), each pass only when its size changes.
// PIL nearest (Geometry.c affine fast path): xx = 0.5 a0, index = (int)xx, xx += a0 per output,
//   a0 = n_in / n_out — walked sequentially (the accumulated double is what Pillow indexes with).
// cv2 linear: f = (d + 0.5) in / out - 0.5, s = floor(f), clamped to [0, in - 1] with f = 0 at
//   the borders, c1 = rint(f 2^11), c0 = 2^11 - c1; out = (h0 c0y + h1 c1y + 2^21) >> 22 with
//   h = in[s] c0x + in[s + 1] c1x.
// Bound: HBM (one pass over the frames; tables are O(H + W)).
#include <math.h>

#include "common.hpp"

namespace rgbd {
namespace {

constexpr int RS_KMAX = 32;  // coefficients per output (ksize = 2 ceil(max(scale, 1)) + 1)
constexpr int RS_PREC = 22;

// table per axis: [n_out] {xmin, count} int2 + [n_out][RS_KMAX] int32
__global__ void k_pil_coeffs(int n_in, int n_out, int2* __restrict__ bounds, int* __restrict__ kk) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= n_out) return;
  const double scale = (double)((float)n_in - 0.f) / n_out;
  const double fs = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * fs;
  const double center = 0.0 + (o + 0.5) * scale;
  const double ss = 1.0 / fs;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > n_in) xmax = n_in;
  xmax -= xmin;
  double w[RS_KMAX];
  double ww = 0.0;
  for (int x = 0; x < xmax && x < RS_KMAX; ++x) {
    double t = (x + xmin - center + 0.5) * ss;
    if (t < 0.0) t = -t;
    w[x] = t < 1.0 ? 1.0 - t : 0.0;
    ww += w[x];
  }
  for (int x = 0; x < RS_KMAX; ++x) {
    int k = 0;
    if (x < xmax) {
      double v = ww != 0.0 ? w[x] / ww : w[x];
      k = v < 0 ? (int)(-0.5 + v * (double)(1 << RS_PREC)) : (int)(0.5 + v * (double)(1 << RS_PREC));
    }
    kk[(long long)o * RS_KMAX + x] = k;
  }
  bounds[o] = make_int2(xmin, xmax);
}

__device__ __forceinline__ uint8_t clip8(int ss) {
  const int v = ss >> RS_PREC;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// horizontal pass: [B][H][W][C] -> [B][H][OW][C]
__global__ __launch_bounds__(256) void k_pil_h(const uint8_t* __restrict__ src, int B, int H, int W, int C, int OW,
                                                const int2* __restrict__ bounds, const int* __restrict__ kk,
                                                uint8_t* __restrict__ dst) {
  const long long n = (long long)B * H * OW * C;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long long p = i / C;
    const int ox = (int)(p % OW);
    const long long row = p / OW;  // b * H + y
    const int2 bd = bounds[ox];
    const int* k = kk + (long long)ox * RS_KMAX;
    const uint8_t* s = src + (row * W + bd.x) * C + c;
    int ss = 1 << (RS_PREC - 1);
    for (int x = 0; x < bd.y; ++x) ss += (int)s[(long long)x * C] * k[x];
    dst[i] = clip8(ss);
  }
}

// vertical pass: [B][H][OW][C] -> [B][OH][OW][C]
__global__ __launch_bounds__(256) void k_pil_v(const uint8_t* __restrict__ src, int B, int H, int OW, int C, int OH,
                                                const int2* __restrict__ bounds, const int* __restrict__ kk,
                                                uint8_t* __restrict__ dst) {
  const long long rowlen = (long long)OW * C;
  const long long n = (long long)B * OH * rowlen;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long q = i % rowlen;
    const long long br = i / rowlen;
    const int oy = (int)(br % OH), b = (int)(br / OH);
    const int2 bd = bounds[oy];
    const int* k = kk + (long long)oy * RS_KMAX;
    const uint8_t* s = src + ((long long)b * H + bd.x) * rowlen + q;
    int ss = 1 << (RS_PREC - 1);
    for (int y = 0; y < bd.y; ++y) ss += (int)s[(long long)y * rowlen] * k[y];
    dst[i] = clip8(ss);
  }
}

// PIL nearest index tables (one thread per axis walks the accumulation, as Pillow does)
__global__ void k_pil_nearest_idx(int in_h, int out_h, int in_w, int out_w, int* __restrict__ iy, int* __restrict__ ix) {
  const int axis = threadIdx.x;
  if (axis > 1) return;
  const int n_in = axis ? in_w : in_h, n_out = axis ? out_w : out_h;
  int* idx = axis ? ix : iy;
  const double a0 = (double)n_in / n_out;
  double xx = 0.5 * a0;
  for (int o = 0; o < n_out; ++o) {
    int v = (int)xx;
    idx[o] = v < 0 ? 0 : (v > n_in - 1 ? n_in - 1 : v);
    xx += a0;
  }
}

__global__ __launch_bounds__(256) void k_pil_nearest(const uint8_t* __restrict__ src, int B, int H, int W, int C,
                                                      int OH, int OW, const int* __restrict__ iy,
                                                      const int* __restrict__ ix, uint8_t* __restrict__ dst) {
  const long long n = (long long)B * OH * OW * C;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long long p = i / C;
    const int ox = (int)(p % OW);
    const long long r = p / OW;
    const int oy = (int)(r % OH), b = (int)(r / OH);
    dst[i] = src[(((long long)b * H + iy[oy]) * W + ix[ox]) * C + c];
  }
}

// cv2 INTER_LINEAR tables: int2 {s0, c1} per output index
__global__ void k_cv_coeffs(int n_in, int n_out, int2* __restrict__ t) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n_out) return;
  const double scale = (double)n_in / n_out;
  double f = (d + 0.5) * scale - 0.5;
  int s = (int)floor(f);
  f -= s;
  if (s < 0) {
    s = 0;
    f = 0.0;
  }
  if (s >= n_in - 1) {
    s = n_in - 1;
    f = 0.0;
  }
  t[d] = make_int2(s, (int)rint(f * 2048.0));
}

__global__ __launch_bounds__(256) void k_cv_linear(const uint8_t* __restrict__ src, int B, int H, int W, int OH, int OW,
                                                    const int2* __restrict__ ty, const int2* __restrict__ tx,
                                                    uint8_t* __restrict__ dst) {
  const long long n = (long long)B * OH * OW;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int ox = (int)(i % OW);
    const long long r = i / OW;
    const int oy = (int)(r % OH), b = (int)(r / OH);
    const int2 X = tx[ox], Y = ty[oy];
    const int x1 = X.x + 1 < W ? X.x + 1 : W - 1, y1 = Y.x + 1 < H ? Y.x + 1 : H - 1;
    const uint8_t* s0 = src + ((long long)b * H + Y.x) * W;
    const uint8_t* s1 = src + ((long long)b * H + y1) * W;
    const long long h0 = (long long)s0[X.x] * (2048 - X.y) + (long long)s0[x1] * X.y;
    const long long h1 = (long long)s1[X.x] * (2048 - X.y) + (long long)s1[x1] * X.y;
    long long v = (h0 * (2048 - Y.y) + h1 * Y.y + (1ll << 21)) >> 22;
    dst[i] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
  }
}

inline int grid_for(long long n) { return (int)std::min<long long>((n + 255) / 256, 65536); }

}  // namespace
}  // namespace rgbd

using namespace rgbd;

extern "C" {

size_t rgbd_resize_workspace_size(int B, int H, int W, int C, int out_h, int out_w) {
  const size_t tables = align256((size_t)(out_h + out_w) * (sizeof(int2) + RS_KMAX * sizeof(int))) +
                        align256((size_t)(out_h + out_w) * sizeof(int2));
  return tables + align256((size_t)B * H * out_w * C);
}

int rgbd_resize_pil_bilinear(const uint8_t* src, int B, int H, int W, int C, int out_h, int out_w, uint8_t* dst,
                             void* ws, void* stream) {
  RGBD_REQUIRE(src && dst && ws && B > 0 && H > 0 && W > 0 && out_h > 0 && out_w > 0 && (C == 1 || C == 3),
               RGBD_E_ARG);
  // ksize = 2 ceil(max(scale, 1)) + 1 <= RS_KMAX
  RGBD_REQUIRE(2 * (int)ceil(std::max(1.0, (double)H / out_h)) + 1 <= RS_KMAX &&
                   2 * (int)ceil(std::max(1.0, (double)W / out_w)) + 1 <= RS_KMAX,
               RGBD_E_SHAPE);
  hipStream_t s = (hipStream_t)stream;
  char* p = (char*)ws;
  int2* bh = (int2*)p;
  int* kh = (int*)(bh + out_w);
  int2* bv = (int2*)(kh + (size_t)out_w * RS_KMAX);
  int* kv = (int*)(bv + out_h);
  uint8_t* tmp = (uint8_t*)(p + align256((size_t)(out_h + out_w) * (sizeof(int2) + RS_KMAX * sizeof(int))) +
                            align256((size_t)(out_h + out_w) * sizeof(int2)));
  const bool need_h = out_w != W, need_v = out_h != H;
  if (!need_h && !need_v) {
    RGBD_CHECK_LAUNCH();
    return (int)hipMemcpyAsync(dst, src, (size_t)B * H * W * C, hipMemcpyDeviceToDevice, s);
  }
  if (need_h) {
    hipLaunchKernelGGL(k_pil_coeffs, dim3(ceil_div(out_w, 128)), dim3(128), 0, s, W, out_w, bh, kh);
    RGBD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_pil_h, dim3(grid_for((long long)B * H * out_w * C)), dim3(256), 0, s, src, B, H, W, C, out_w,
                       bh, kh, need_v ? tmp : dst);
    RGBD_CHECK_LAUNCH();
  }
  if (need_v) {
    hipLaunchKernelGGL(k_pil_coeffs, dim3(ceil_div(out_h, 128)), dim3(128), 0, s, H, out_h, bv, kv);
    RGBD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_pil_v, dim3(grid_for((long long)B * out_h * out_w * C)), dim3(256), 0, s,
                       need_h ? tmp : src, B, H, out_w, C, out_h, bv, kv, dst);
    RGBD_CHECK_LAUNCH();
  }
  return RGBD_OK;
}

int rgbd_resize_pil_nearest(const uint8_t* src, int B, int H, int W, int C, int out_h, int out_w, uint8_t* dst,
                            void* ws, void* stream) {
  RGBD_REQUIRE(src && dst && ws && B > 0 && H > 0 && W > 0 && out_h > 0 && out_w > 0 && C > 0, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  int* iy = (int*)ws;
  int* ix = iy + out_h;
  hipLaunchKernelGGL(k_pil_nearest_idx, dim3(1), dim3(64), 0, s, H, out_h, W, out_w, iy, ix);
  RGBD_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_pil_nearest, dim3(grid_for((long long)B * out_h * out_w * C)), dim3(256), 0, s, src, B, H, W,
                     C, out_h, out_w, iy, ix, dst);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_resize_cv2_linear(const uint8_t* src, int B, int H, int W, int out_h, int out_w, uint8_t* dst, void* ws,
                           void* stream) {
  RGBD_REQUIRE(src && dst && ws && B > 0 && H > 0 && W > 0 && out_h > 0 && out_w > 0, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  if (out_h == H && out_w == W)  // cv2.resize to the same size copies
    return (int)hipMemcpyAsync(dst, src, (size_t)B * H * W, hipMemcpyDeviceToDevice, s);
  int2* ty = (int2*)ws;
  int2* tx = ty + out_h;
  hipLaunchKernelGGL(k_cv_coeffs, dim3(ceil_div(out_h, 128)), dim3(128), 0, s, H, out_h, ty);
  RGBD_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_cv_coeffs, dim3(ceil_div(out_w, 128)), dim3(128), 0, s, W, out_w, tx);
  RGBD_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_cv_linear, dim3(grid_for((long long)B * out_h * out_w)), dim3(256), 0, s, src, B, H, W, out_h,
                     out_w, ty, tx, dst);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
