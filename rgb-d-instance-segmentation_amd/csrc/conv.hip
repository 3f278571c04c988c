// f2: the pixel decoder's and Swin's remaining convolutions as MFMA GEMMs (csrc/gemm.hip).
//
// Reference call sites: self.encoder(rgb) (custom_model.py:330: SwinPatchEmbeddings.projection,
// Conv2d(3, 96, 4, stride 4)) and self.decoder(backbone_features, ...) (custom_model.py:383:
// Mask2FormerPixelDecoder's input projections Conv2d(C, 256, 1) + GroupNorm, its FPN lateral
// Conv2d(96, 256, 1, bias=False) + GroupNorm, the FPN output Conv2d(256, 256, 3, padding 1,
// bias=False) + GroupNorm + ReLU and mask_projection Conv2d(256, 256, 1); transformers 5.15
// modeling_mask2former.py Mask2FormerPixelDecoder.__init__).
//
// A KxK convolution in NCHW is the batched GEMM
//   Y[b][o][p] = sum_k W[o][k] col[b][k][p] (+ bias[o]),   k = (c*KH + ky)*KW + kx
// with col the im2col of x (torch.nn.functional.unfold's row order, which is the flattened
// OIHW weight's column order).  1x1 convolutions need no col (col = x).  This file builds col:
//   3x3 stride 1, padding 1 (the FPN output convolution; also the transposed convolution of its
//     backward: dX = conv(dY, W flipped and transposed), so the same kernel serves dX);
//   4x4 stride 4, padding 0 (Swin's patch embedding: non-overlapping patches).
// The GEMMs themselves are rgbd_gemm (row-indexed bias, RGBD_BIAS_M).
#include "common.hpp"

namespace {

using namespace rgbd;

// 3x3, stride 1, pad 1.  Thread = (b, c, y, 8 consecutive x); it loads the 3 x 10 input values
// it needs (rows y-1..y+1, columns x-1..x+8, zero outside) and writes the 9 col rows' 8-pixel
// pieces (16-byte stores for bf16 when W % 8 == 0).
template <typename T>
__global__ __launch_bounds__(256) void k_im2col3(const T* __restrict__ x, int C, int H, int W, int xq,
                                                 long long total, T* __restrict__ col) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int q = (int)(i % xq);
  long long r = i / xq;
  const int y = (int)(r % H);
  r /= H;  // = b * C + c
  const int x0 = q * 8;
  const T* src = x + r * H * W;
  // all 30 loads unconditional (clamped addresses, zeroed after): behind per-element branches the
  // compiler waited for each one where it was issued, 30 memory round trips per thread
  T raw[3][10];
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int yc = min(max(y + dy - 1, 0), H - 1);
#pragma unroll
    for (int j = 0; j < 10; ++j) raw[dy][j] = src[(long long)yc * W + min(max(x0 + j - 1, 0), W - 1)];
  }
  float v[3][10];
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int yy = y + dy - 1;
    const bool row_ok = yy >= 0 && yy < H;
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const int xx = x0 + j - 1;
      v[dy][j] = (row_ok && xx >= 0 && xx < W) ? Num<T>::to_f(raw[dy][j]) : 0.f;
    }
  }
  const long long HW = (long long)H * W;
  T* dst = col + (r * 9) * HW + (long long)y * W + x0;  // row (c*3 + ky)*3 + kx of image b
  const bool full = x0 + 8 <= W;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int ky = t / 3, kx = t % 3;
    T* d = dst + t * HW;
    if constexpr (sizeof(T) == 2) {
      if (full && (W & 7) == 0) {
        *reinterpret_cast<uint4*>(d) =
            make_uint4(pack_bf16x2(v[ky][kx], v[ky][kx + 1]), pack_bf16x2(v[ky][kx + 2], v[ky][kx + 3]),
                       pack_bf16x2(v[ky][kx + 4], v[ky][kx + 5]), pack_bf16x2(v[ky][kx + 6], v[ky][kx + 7]));
        continue;
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (x0 + e < W) d[e] = Num<T>::from_f(v[ky][kx + e]);
  }
}

// 4x4, stride 4, pad 0 (H % 4 == W % 4 == 0): col[b][(c*4 + ky)*4 + kx][py * Wp + px] =
// x[b][c][4 py + ky][4 px + kx].  Thread = (b, c, y, px): one 4-element input run -> 4 col rows.
template <typename T>
__global__ __launch_bounds__(256) void k_patchify4(const T* __restrict__ x, int C, int H, int W, long long total,
                                                   T* __restrict__ col) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int Wp = W / 4, Hp = H / 4;
  const int px = (int)(i % Wp);
  long long r = i / Wp;
  const int y = (int)(r % H);
  r /= H;  // b * C + c
  const int py = y >> 2, ky = y & 3;
  const T* s = x + (r * H + y) * (long long)W + 4 * px;
  const long long HWp = (long long)Hp * Wp;
  T* d = col + (r * 16 + ky * 4) * HWp + (long long)py * Wp + px;
#pragma unroll
  for (int kx = 0; kx < 4; ++kx) d[kx * HWp] = s[kx];
}

template <typename T>
int im2col_t(const void* x, int B, int C, int H, int W, int kernel, void* col, hipStream_t s) {
  if (kernel == 3) {
    const int xq = (W + 7) / 8;
    const long long total = (long long)B * C * H * xq;
    hipLaunchKernelGGL(k_im2col3<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, (const T*)x, C, H, W, xq,
                       total, (T*)col);
  } else {
    const long long total = (long long)B * C * H * (W / 4);
    hipLaunchKernelGGL(k_patchify4<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, (const T*)x, C, H, W,
                       total, (T*)col);
  }
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // namespace

extern "C" {

int rgbd_im2col(int dtype, const void* x, int B, int C, int H, int W, int kernel, void* col, void* stream) {
  RGBD_REQUIRE(x && col && B > 0 && C > 0 && H > 0 && W > 0, RGBD_E_ARG);
  RGBD_REQUIRE(kernel == 3 || (kernel == 4 && H % 4 == 0 && W % 4 == 0), RGBD_E_SHAPE);
  RGBD_REQUIRE((long long)B * C * H * W * (kernel == 3 ? 9 : 1) < (1ll << 40), RGBD_E_SHAPE);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_BF16) return im2col_t<bf16_t>(x, B, C, H, W, kernel, col, s);
  if (dtype == RGBD_F32) return im2col_t<float>(x, B, C, H, W, kernel, col, s);
  return RGBD_E_DTYPE;
}

}  // extern "C"
