// a11, label half: the instance channel of the annotation -> mask_labels / class_labels, as
// map_10channel_case2 gets them from Mask2FormerImageProcessor (reference
// mask2former/utils/dataloader.py:391-423 -> transformers convert_segmentation_map_to_binary_masks):
//   labels = sorted unique instance ids minus ignore_index; mask_labels[i] = (map == labels[i]).
// Two HBM-bound passes over u8 maps: a per-image 256-bit presence bitmap (read back by the host,
// 32 B per image, to size the ragged outputs and look up the class ids), then the float32 masks,
// 16 pixels per thread (one 16-byte map load, four 16-byte stores).
#include "common.hpp"

using namespace rgbd;

namespace {

__global__ __launch_bounds__(256) void k_instance_presence(const uint8_t* __restrict__ inst, long long HW,
                                                           uint32_t* __restrict__ presence) {
  __shared__ uint32_t bits[8];
  const int b = blockIdx.y;
  if (threadIdx.x < 8) bits[threadIdx.x] = 0u;
  __syncthreads();
  const uint8_t* m = inst + b * HW;
  uint32_t local[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  const long long n16 = HW >> 4;
  for (long long q = blockIdx.x * 256ll + threadIdx.x; q < n16; q += 256ll * gridDim.x) {
    const uint4 v = reinterpret_cast<const uint4*>(m)[q];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const uint32_t id = (w[e >> 2] >> (8 * (e & 3))) & 0xffu;
#pragma unroll
      for (int k = 0; k < 8; ++k) local[k] |= (id >> 5) == (uint32_t)k ? 1u << (id & 31) : 0u;
    }
  }
  for (long long p = (n16 << 4) + blockIdx.x * 256ll + threadIdx.x; p < HW; p += 256ll * gridDim.x) {
    const uint32_t id = m[p];
    local[id >> 5] |= 1u << (id & 31);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint32_t v = local[k];
    for (int o = 32; o > 0; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o);
    if ((threadIdx.x & 63) == 0 && v) atomicOr(&bits[k], v);
  }
  __syncthreads();
  if (threadIdx.x < 8 && bits[threadIdx.x]) atomicOr(&presence[b * 8 + threadIdx.x], bits[threadIdx.x]);
}

__global__ __launch_bounds__(256) void k_instance_masks(const uint8_t* __restrict__ inst, long long HW,
                                                        const int* __restrict__ ids, const int* __restrict__ img,
                                                        float* __restrict__ masks) {
  const int j = blockIdx.y;
  const uint32_t id = (uint32_t)ids[j];
  const uint8_t* m = inst + img[j] * HW;
  float* out = masks + j * HW;
  const long long n16 = HW >> 4;
  for (long long q = blockIdx.x * 256ll + threadIdx.x; q < n16; q += 256ll * gridDim.x) {
    const uint4 v = reinterpret_cast<const uint4*>(m)[q];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float f[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) f[e] = ((w[k] >> (8 * e)) & 0xffu) == id ? 1.f : 0.f;
      reinterpret_cast<float4*>(out)[4 * q + k] = make_float4(f[0], f[1], f[2], f[3]);
    }
  }
  for (long long p = (n16 << 4) + blockIdx.x * 256ll + threadIdx.x; p < HW; p += 256ll * gridDim.x)
    out[p] = (uint32_t)m[p] == id ? 1.f : 0.f;
}

}  // namespace

extern "C" {

int rgbd_instance_presence(const uint8_t* instance_map, int B, int H, int W, uint32_t* presence, void* stream) {
  RGBD_REQUIRE(instance_map && presence && B > 0 && H > 0 && W > 0, RGBD_E_ARG);
  const long long HW = (long long)H * W;
  RGBD_REQUIRE(((uintptr_t)instance_map & 15) == 0 && (HW % 16 == 0 || B == 1), RGBD_E_SHAPE);
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(presence, 0, (size_t)B * 8 * sizeof(uint32_t), s);
  if (e != hipSuccess) return (int)e;
  const int gx = (int)std::min<long long>(std::max<long long>(1, (HW / 16 + 255) / 256), 64);
  k_instance_presence<<<dim3(gx, B), 256, 0, s>>>(instance_map, HW, presence);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_instance_masks(const uint8_t* instance_map, int H, int W, const int* ids, const int* image_of, int n,
                        float* masks, void* stream) {
  RGBD_REQUIRE(instance_map && ids && image_of && masks && n >= 0 && H > 0 && W > 0, RGBD_E_ARG);
  if (n == 0) return RGBD_OK;
  const long long HW = (long long)H * W;
  RGBD_REQUIRE(((uintptr_t)instance_map & 15) == 0 && ((uintptr_t)masks & 15) == 0 && HW % 16 == 0, RGBD_E_SHAPE);
  const int gx = (int)std::min<long long>(std::max<long long>(1, (HW / 16 + 255) / 256), 512);
  k_instance_masks<<<dim3(gx, n), 256, 0, (hipStream_t)stream>>>(instance_map, HW, ids, image_of, masks);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
