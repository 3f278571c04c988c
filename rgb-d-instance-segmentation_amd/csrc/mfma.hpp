// MFMA fragment helpers shared by the implicit-GEMM kernels.
//
// Both precisions use the 16x16 output tile (C/D map: col = lane&15, row = 4*(lane>>4)+reg)
// and the same per-lane K slice: lane (r = lane&15, g = lane>>4) holds 8 consecutive
// reduction elements k = 8g .. 8g+7 of a 32-wide K step for its A row / B column.
//   bf16: one v_mfma_f32_16x16x32_bf16 (lane map A[r][8g+j], B[8g+j][r]  — exact match)
//   f32 : eight v_mfma_f32_16x16x4_f32; step j uses element j, i.e. the instruction's
//         k index l>>4 = g stands for reduction element 8g+j.  A and B apply the same
//         permutation, so the sum is the same 32-term dot product (exact f32 products,
//         f32 accumulation: the parity mode).
#pragma once
#include "common.hpp"

namespace rgbd {

typedef __attribute__((ext_vector_type(8))) __bf16 mbf16x8;

template <typename T> struct Frag;

template <> struct Frag<bf16_t> {
  uint4 v;  // 8 x bf16
  __device__ __forceinline__ void load(const bf16_t* p) { v = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void zero() { v = make_uint4(0u, 0u, 0u, 0u); }
  __device__ __forceinline__ void select(bool keep) {
    if (!keep) zero();
  }
  // element setters: j must be a compile-time constant after unrolling (switch keeps the
  // fragment in registers; a pointer into it would force scratch)
  __device__ __forceinline__ void set(int j, float f) { set_raw(j, f32_to_bf16(f)); }
  __device__ __forceinline__ void set_raw(int j, bf16_t h) {
    const uint32_t hv = h;
    switch (j >> 1) {
      case 0: v.x = (j & 1) ? ((v.x & 0xffffu) | (hv << 16)) : ((v.x & 0xffff0000u) | hv); break;
      case 1: v.y = (j & 1) ? ((v.y & 0xffffu) | (hv << 16)) : ((v.y & 0xffff0000u) | hv); break;
      case 2: v.z = (j & 1) ? ((v.z & 0xffffu) | (hv << 16)) : ((v.z & 0xffff0000u) | hv); break;
      default: v.w = (j & 1) ? ((v.w & 0xffffu) | (hv << 16)) : ((v.w & 0xffff0000u) | hv); break;
    }
  }
  __device__ __forceinline__ void to8(float (&f)[8]) const {
    f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
    f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
    f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
  }
  __device__ __forceinline__ void from8(const float (&f)[8]) {
    v = make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]), pack_bf16x2(f[6], f[7]));
  }
};

template <> struct Frag<float> {
  float4 lo, hi;  // 8 x f32
  __device__ __forceinline__ void load(const float* p) {
    lo = *reinterpret_cast<const float4*>(p);
    hi = *reinterpret_cast<const float4*>(p + 4);
  }
  __device__ __forceinline__ void zero() {
    lo = make_float4(0.f, 0.f, 0.f, 0.f);
    hi = lo;
  }
  __device__ __forceinline__ void select(bool keep) {
    if (!keep) zero();
  }
  __device__ __forceinline__ void set(int j, float f) {
    switch (j) {
      case 0: lo.x = f; break;
      case 1: lo.y = f; break;
      case 2: lo.z = f; break;
      case 3: lo.w = f; break;
      case 4: hi.x = f; break;
      case 5: hi.y = f; break;
      case 6: hi.z = f; break;
      default: hi.w = f; break;
    }
  }
  __device__ __forceinline__ void to8(float (&f)[8]) const {
    f[0] = lo.x; f[1] = lo.y; f[2] = lo.z; f[3] = lo.w;
    f[4] = hi.x; f[5] = hi.y; f[6] = hi.z; f[7] = hi.w;
  }
  __device__ __forceinline__ void from8(const float (&f)[8]) {
    lo = make_float4(f[0], f[1], f[2], f[3]);
    hi = make_float4(f[4], f[5], f[6], f[7]);
  }
};

__device__ __forceinline__ void mma(f32x4& acc, const Frag<bf16_t>& a, const Frag<bf16_t>& b) {
  mbf16x8 av, bv;
  __builtin_memcpy(&av, &a.v, 16);
  __builtin_memcpy(&bv, &b.v, 16);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
}

__device__ __forceinline__ void mma(f32x4& acc, const Frag<float>& a, const Frag<float>& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo.x, b.lo.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo.y, b.lo.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo.z, b.lo.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo.w, b.lo.w, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi.x, b.hi.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi.y, b.hi.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi.z, b.hi.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi.w, b.hi.w, acc, 0, 0, 0);
}

}  // namespace rgbd
