// Shared helpers for the gfx950 kernels of librgbd_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "../../include/rgbd_hip.h"

#define RGBD_CHECK_LAUNCH()                                  \
  do {                                                       \
    hipError_t e__ = hipGetLastError();                      \
    if (e__ != hipSuccess) return (int)e__;                  \
  } while (0)

#define RGBD_REQUIRE(cond, code) \
  do {                           \
    if (!(cond)) return (code);  \
  } while (0)

namespace rgbd {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

// Buffer descriptor over [base, base + bytes) built from wave-uniform values (readfirstlane of the
// pointer halves, so no waterfall loop around each access), for write-through hand-offs: 16-byte
// buffer stores / loads with aux WT_SC1 carry sc1 (they bypass this CU's L1 and write through the
// XCD's L2), the form MI355X_MICROARCH.md's visibility table (row 1) admits without fences.
constexpr int WT_SC1 = 16;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* base, int bytes) {
  const uintptr_t p = (uintptr_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
}

typedef uint16_t bf16_t;  // raw bfloat16 storage (same bits as torch.bfloat16)

__device__ __forceinline__ float bf16_to_f32(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);  // round-to-nearest-even, NaN-preserving
  return *reinterpret_cast<bf16_t*>(&b);
}

// Two floats -> packed bf16x2 (low = a) with one v_cvt_pk_bf16_f32 (round-to-nearest-even).
typedef float rgbd_f2v __attribute__((ext_vector_type(2)));
typedef __bf16 rgbd_b2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  const rgbd_f2v f = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, rgbd_b2v));
}

template <typename T> struct Num;
template <> struct Num<float> {
  static __device__ __forceinline__ float load(const float* p) { return *p; }
  static __device__ __forceinline__ float to_f(float v) { return v; }
  static __device__ __forceinline__ float from_f(float v) { return v; }
};
template <> struct Num<bf16_t> {
  static __device__ __forceinline__ float to_f(bf16_t v) { return bf16_to_f32(v); }
  static __device__ __forceinline__ bf16_t from_f(float v) { return f32_to_bf16(v); }
};

// Order-preserving float <-> uint32 key (for atomicMin/atomicMax on floats of any sign).
__device__ __forceinline__ uint32_t f32_key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_f32(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

// Correctly rounded float32 division / sqrt.  HIP's default f32 `/` and sqrtf are not
// IEEE-rounded on gfx950 (measured: 28 of 256 quotients off by 1 ulp vs numpy), so every
// op that must match numpy bit-for-bit goes through double: for / and sqrt of float32
// operands, rounding the f64 result to f32 is exact rounding (53 >= 2*24+2 bits).
__device__ __forceinline__ float div_rn(float a, float b) { return (float)((double)a / (double)b); }
__device__ __forceinline__ float sqrt_rn(float a) { return (float)__builtin_sqrt((double)a); }

__device__ __forceinline__ float wave_min(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Hide a loop-invariant pointer from LICM: without it hipcc hoists every weight-fragment load
// of a persistent tile loop out of the loop and spills them all to scratch.
template <class P>
__device__ __forceinline__ P opaque(P p) {
  uintptr_t u = (uintptr_t)p;
  asm volatile("" : "+s"(u));
  return (P)u;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// outstanding global loads/stores (__syncthreads() also drains vmcnt, which would serialise
// every register-prefetched global load and every epilogue store with the barrier).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// One LDS-DMA wave instruction: 64 lanes x 16 B from per-lane global sources to
// lds_base + 16 * lane (lds_base wave-uniform; it goes through M0).
__device__ __forceinline__ void dma_lds16(const void* gsrc, uint32_t lds_base) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_base)
               : "memory");
}

// Ring-pipeline hand-off: this wave's DMA pieces older than the newest N have landed and its LDS
// reads are done, then the workgroup barrier (no compiler-visible global loads may be in flight
// in such a loop: they share vmcnt with the DMA).
template <int N>
__device__ __forceinline__ void vm_wait_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// vm_wait_barrier for a run-time count (wave-uniform); counts past 23 wait for 23 (more waiting,
// never less).
__device__ __forceinline__ void vm_wait_barrier_dyn(int n) {
  switch (n) {
#define RGBD_VMW_CASE(k) \
  case k:                \
    vm_wait_barrier<k>(); \
    break;
    RGBD_VMW_CASE(0) RGBD_VMW_CASE(1) RGBD_VMW_CASE(2) RGBD_VMW_CASE(3) RGBD_VMW_CASE(4) RGBD_VMW_CASE(5)
    RGBD_VMW_CASE(6) RGBD_VMW_CASE(7) RGBD_VMW_CASE(8) RGBD_VMW_CASE(9) RGBD_VMW_CASE(10) RGBD_VMW_CASE(11)
    RGBD_VMW_CASE(12) RGBD_VMW_CASE(13) RGBD_VMW_CASE(14) RGBD_VMW_CASE(15) RGBD_VMW_CASE(16) RGBD_VMW_CASE(17)
    RGBD_VMW_CASE(18) RGBD_VMW_CASE(19) RGBD_VMW_CASE(20) RGBD_VMW_CASE(21) RGBD_VMW_CASE(22)
#undef RGBD_VMW_CASE
    default:
      vm_wait_barrier<23>();
      break;
  }
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace rgbd
