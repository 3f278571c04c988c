// f4: mask IoU of the segm mean-average-precision metric (the reference's Evaluator,
// mask2former/utils/model_essential_part.py:56-157, torchmetrics MeanAveragePrecision(iou_type=
// "segm") over pycocotools' maskApi rleIou).  The IoU of every (detection, ground truth) pair of
// an image is the pairs' intersection over union of their pixel sets; here the masks are packed
// into bitmaps once (one u64 per 64 consecutive pixels) with their areas, and a pair's
// intersection is a popcount over the AND of two bitmaps — HBM / L2-bound integer work, no GEMM.
#include "common.hpp"

using namespace rgbd;

namespace {

// One thread per 64-pixel word: 64 bytes of the {0, nonzero} uint8 mask (four 16-byte loads when
// the row is 16-byte aligned) -> one u64; per-mask area by a block reduction + one atomic.
__global__ __launch_bounds__(256) void k_pack_bits(const uint8_t* __restrict__ masks, long long npx, int words,
                                                   unsigned long long* __restrict__ bits, int* __restrict__ area) {
  const int m = blockIdx.y;
  const long long w = (long long)blockIdx.x * 256 + threadIdx.x;
  const uint8_t* src = masks + (long long)m * npx;
  unsigned long long v = 0ull;
  if (w < words) {
    const long long p0 = w * 64;
    const bool vec = (npx % 16) == 0 && p0 + 64 <= npx && (((uintptr_t)src & 15) == 0);
    if (vec) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 x = *reinterpret_cast<const uint4*>(src + p0 + 16 * q);
        const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int b = 0; b < 4; ++b)
            if ((xs[k] >> (8 * b)) & 0xffu) v |= 1ull << (16 * q + 4 * k + b);
      }
    } else {
      for (int j = 0; j < 64 && p0 + j < npx; ++j)
        if (src[p0 + j]) v |= 1ull << j;
    }
    bits[(long long)m * words + w] = v;
  }
  int c = __popcll(v);
  c = (int)wave_sum((float)c);  // <= 64 * 64: exact in float
  __shared__ int red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(area + m, red[0] + red[1] + red[2] + red[3]);
}

// One workgroup per (a, b) pair: popcount of the AND over the words, fixed-order reduction.
__global__ __launch_bounds__(256) void k_mask_inter(const unsigned long long* __restrict__ a, int na,
                                                    const unsigned long long* __restrict__ b, int nb, int words,
                                                    int* __restrict__ inter) {
  const int i = blockIdx.y, j = blockIdx.x;
  const unsigned long long* pa = a + (long long)i * words;
  const unsigned long long* pb = b + (long long)j * words;
  int c = 0;
  for (int w = threadIdx.x; w < words; w += 256) c += __popcll(pa[w] & pb[w]);
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  __shared__ int red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) inter[(long long)i * nb + j] = red[0] + red[1] + red[2] + red[3];
}

}  // namespace

extern "C" {

int rgbd_pack_mask_bits(const uint8_t* masks, int n, long long npx, unsigned long long* bits, int* area,
                        void* stream) {
  RGBD_REQUIRE(n >= 0 && npx > 0, RGBD_E_ARG);
  if (n == 0) return RGBD_OK;
  RGBD_REQUIRE(masks && bits && area, RGBD_E_ARG);
  RGBD_REQUIRE(n <= 65535, RGBD_E_SHAPE);
  const long long words = (npx + 63) / 64;
  RGBD_REQUIRE(words < (1ll << 31), RGBD_E_SHAPE);
  hipStream_t s = (hipStream_t)stream;
  const hipError_t e = hipMemsetAsync(area, 0, sizeof(int) * (size_t)n, s);
  if (e != hipSuccess) return (int)e;
  k_pack_bits<<<dim3((unsigned)((words + 255) / 256), n), 256, 0, s>>>(masks, npx, (int)words, bits, area);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_mask_intersections(const unsigned long long* a, int na, const unsigned long long* b, int nb, long long npx,
                            int* inter, void* stream) {
  RGBD_REQUIRE(na >= 0 && nb >= 0 && npx > 0, RGBD_E_ARG);
  if (na == 0 || nb == 0) return RGBD_OK;
  RGBD_REQUIRE(a && b && inter && na <= 65535 && nb <= 65535, RGBD_E_ARG);
  const long long words = (npx + 63) / 64;
  k_mask_inter<<<dim3(nb, na), 256, 0, (hipStream_t)stream>>>(a, na, b, nb, (int)words, inter);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
