// Per-CU copy throughput from L2 / MALL / HBM: LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
// instruction) vs register loads (global_load_dwordx4), one 512-thread workgroup per CU (the
// workgroup claims 96 KiB of LDS so no second one fits), each wave issuing `depth` 1-KiB pieces
// and then waiting for all of them, `iters` times.  Every workgroup walks its own window of the
// source buffer (a footprint of `foot` bytes over all workgroups: 1 MiB stays in L2, 64 MiB in
// the Infinity Cache, 2 GiB streams from HBM).  Prints GB/s per CU and bytes per clock per CU.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/bin/dma_bw tools/native/dma_bw.hip
//   tools/bin/dma_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__device__ __forceinline__ void dma16(const void* g, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(lds)
               : "memory");
}

// mode 0: LDS-DMA; mode 1: register loads.  window = bytes per workgroup (multiple of 8 KiB)
template <int MODE, int DEPTH>
__global__ __launch_bounds__(512, 1) void k_bw(const char* __restrict__ src, long long window, int shared, int iters,
                                               unsigned* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const char* base = src + (shared ? 0ll : (long long)blockIdx.x * window);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem + wave * (DEPTH * 1024);
  long long off = (long long)wave * DEPTH * 1024;
  uint4 x = make_uint4(0u, 0u, 0u, 0u);
  for (int it = 0; it < iters; ++it) {
    if (off + 8ll * DEPTH * 1024 > window) off = (long long)wave * DEPTH * 1024;
    if constexpr (MODE == 0) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) dma16(base + off + d * 1024 + lane * 16, lds0 + d * 1024);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      uint4 v[DEPTH];
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) v[d] = *(const uint4*)(base + off + d * 1024 + lane * 16);
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        x.x ^= v[d].x;
        x.y ^= v[d].y;
        x.z ^= v[d].z;
        x.w ^= v[d].w;
      }
    }
    off += 8ll * DEPTH * 1024;
  }
  if (x.x == 0x12345678u && x.y == 0x9abcdef0u) sink[threadIdx.x] = x.z ^ x.w;  // keeps the loads live
}

template <int MODE, int DEPTH>
void run(const char* src, long long foot, int nwg, unsigned* sink, int clk_mhz) {
  // foot < 1 MiB: every workgroup reads the same window (L2-resident on every XCD)
  const int shared = foot < (1 << 20);
  const long long per = shared ? foot : foot / nwg;
  const long long window = per / (8 * DEPTH * 1024) * (8 * DEPTH * 1024);
  if (window < 8ll * DEPTH * 1024) return;
  const int iters = 400;
  CK(hipFuncSetAttribute((const void*)k_bw<MODE, DEPTH>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 2; ++w) k_bw<MODE, DEPTH><<<nwg, 512, 96 * 1024>>>(src, window, shared, iters, sink);
  CK(hipEventRecord(e0));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) k_bw<MODE, DEPTH><<<nwg, 512, 96 * 1024>>>(src, window, shared, iters, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = (double)reps * nwg * iters * 8.0 * DEPTH * 1024;
  (void)window;
  const double per_cu = bytes / (ms * 1e-3) / nwg;
  printf("%-9s depth %2d  footprint %9.3f MiB: %7.1f GB/s per CU  %5.1f B/clk per CU (at %d MHz)  chip %6.2f TB/s\n",
         MODE == 0 ? "LDS-DMA" : "register", DEPTH, foot / 1048576.0, per_cu / 1e9, per_cu / (clk_mhz * 1e6), clk_mhz,
         bytes / (ms * 1e-3) / 1e12);
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int nwg = p.multiProcessorCount;
  const int clk = p.clockRate / 1000;
  printf("%s, %d CUs, %d MHz\n", p.gcnArchName, nwg, clk);
  const long long maxfoot = 2ll << 30;
  char* src;
  CK(hipMalloc(&src, maxfoot));
  CK(hipMemset(src, 1, maxfoot));
  unsigned* sink;
  CK(hipMalloc(&sink, 512 * sizeof(unsigned)));
  const long long foots[3] = {576ll * 1024, 64ll << 20, maxfoot};
  for (long long f : foots) {
    run<0, 1>(src, f, nwg, sink, clk);
    run<0, 4>(src, f, nwg, sink, clk);
    run<0, 9>(src, f, nwg, sink, clk);
    run<1, 1>(src, f, nwg, sink, clk);
    run<1, 4>(src, f, nwg, sink, clk);
    run<1, 9>(src, f, nwg, sink, clk);
  }
  CK(hipFree(src));
  CK(hipFree(sink));
  return 0;
}
