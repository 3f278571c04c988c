// f1 / f2: the dense layers of the Mask2Former decoder, pixel decoder and Swin
// backbone — nn.Linear forward and backward — as one MFMA GEMM family with fused epilogues.
//
// Reference call sites (transformers 5.15 modeling_mask2former.py / modeling_swin.py):
//   decoder layer   self_attn q/k/v/out_proj (:1480-1483), fc1 -> relu -> fc2 (:1711-1714)
//   pixel decoder   value_proj / sampling_offsets / attention_weights / output_proj
//                   (:862-868), fc1 -> relu -> fc2 of each encoder layer (:1030-1036)
//   Swin-T          qkv (query/key/value), attention output dense, intermediate dense -> gelu,
//                   output dense, patch-merging reduction (modeling_swin.py:420-424, 540, 560,
//                   574, 344)
//
// C[M][N] = act(sum_k op(A)[m][k] op(B)[k][n] + bias[n]) (+ R[m][n]), batched, with
//   A: a_t = 0 -> stored [M][lda] (K contiguous: activations); a_t = 1 -> [K][lda] (M
//      contiguous: dY^T of a weight gradient)
//   B: b_t = 0 -> stored [N][ldb] (K contiguous: nn.Linear's weight); b_t = 1 -> [K][ldb]
//      (N contiguous: the weight in dX = dY W, the activations in dW = dY^T X)
// so the three GEMMs of a linear layer are (a_t, b_t) = (0, 0) forward, (0, 1) dX, (1, 1) dW.
//
// Tiling: 256 threads = 4 waves, workgroup tile TM x TN (128 x 128 or 64 x 64), wave tile
// (TM/2) x (TN/2) of 16x16 MFMA fragments, K staged per 128-byte step (64 bf16 / 32 f32) into
// double-buffered LDS through registers (the next step's 16-byte global loads are in flight
// during the current step's MFMAs; one barrier per step).  K-contiguous tiles are [rows][128 B]
// with 16-byte chunk c at slot c ^ (row & 7); M/N-contiguous tiles are [k][rows] read back
// k-major with ds_read_b64_tr_b16 (bf16, 32-byte blocks XOR-swizzled by row bits 0-1 and 3)
// or ds_read_b32 (f32, 64-byte blocks swizzled by row bit 3) — the layouts of mask_predict.hip.
// The MFMA's A operand is the N side and its B operand the M side, so a lane's four accumulator
// registers are four consecutive n of one row m: 8-byte (bf16) / 16-byte (f32) stores.
// bf16: v_mfma_f32_16x16x32_bf16, float32 sums; f32: v_mfma_f32_16x16x4_f32 (exact products).
// Split-K (splits > 1): per split a float32 partial tile into the workspace, then one pass sums
// the splits in order (deterministic) and applies the epilogue.
#include "common.hpp"
#include "mfma.hpp"

#include <algorithm>
#include <type_traits>

namespace rgbd {
namespace {

typedef __attribute__((ext_vector_type(4))) short g_v4s;
typedef __attribute__((ext_vector_type(4))) unsigned int v4u;

constexpr int G_THREADS = 256;

template <typename T> struct GCfg;
template <> struct GCfg<bf16_t> {
  static constexpr int KS = 64;    // K elements per stage (128 bytes)
  static constexpr int VEC = 8;    // elements per 16-byte chunk
  static constexpr int TROW = 256; // bytes per k row of an M/N-contiguous tile (128 elements)
  static __device__ __forceinline__ int toff(int row, int byte) {
    const int swz = (row & 3) | (((row >> 3) & 1) << 2);
    return row * TROW + (((byte >> 5) ^ swz) << 5) + (byte & 31);
  }
};
template <> struct GCfg<float> {
  static constexpr int KS = 32;
  static constexpr int VEC = 4;
  static constexpr int TROW = 512;
  static __device__ __forceinline__ int toff(int row, int byte) {
    return row * TROW + (((byte >> 6) ^ ((row >> 3) & 1)) << 6) + (byte & 63);
  }
};

__device__ __forceinline__ int koff(int row, int chunk) { return row * 128 + 16 * (chunk ^ (row & 7)); }

// fragment i (rows 16i..16i+15 of the tile) of k-step ks from a K-contiguous tile
__device__ __forceinline__ Frag<bf16_t> frag_k(const char* s, int i, int ks, int lane) {
  const int row = 16 * i + (lane & 15), g = lane >> 4;
  Frag<bf16_t> f;
  f.v = *reinterpret_cast<const uint4*>(s + koff(row, 4 * ks + g));
  return f;
}
__device__ __forceinline__ Frag<float> frag_k_f32(const char* s, int i, int lane) {
  const int row = 16 * i + (lane & 15), g = lane >> 4;
  Frag<float> f;
  f.lo = *reinterpret_cast<const float4*>(s + koff(row, 2 * g));
  f.hi = *reinterpret_cast<const float4*>(s + koff(row, 2 * g + 1));
  return f;
}
// the same fragment from an M/N-contiguous tile [k][rows] (transposed reads)
__device__ __forceinline__ Frag<bf16_t> frag_t(const char* s, int i, int ks, int lane) {
  using Cfg = GCfg<bf16_t>;
  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int row0 = 32 * ks + 8 * g + q4, row1 = row0 + 4;
  const int byte = (16 * i + 4 * p4) * 2;
  g_v4s t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) g_v4s*)(s + Cfg::toff(row0, byte)));
  g_v4s t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) g_v4s*)(s + Cfg::toff(row1, byte)));
  Frag<bf16_t> f;
  f.v = make_uint4((uint32_t)(uint16_t)t0.x | ((uint32_t)(uint16_t)t0.y << 16),
                   (uint32_t)(uint16_t)t0.z | ((uint32_t)(uint16_t)t0.w << 16),
                   (uint32_t)(uint16_t)t1.x | ((uint32_t)(uint16_t)t1.y << 16),
                   (uint32_t)(uint16_t)t1.z | ((uint32_t)(uint16_t)t1.w << 16));
  return f;
}
__device__ __forceinline__ Frag<float> frag_t_f32(const char* s, int i, int lane) {
  using Cfg = GCfg<float>;
  const int r = lane & 15, g = lane >> 4;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const float*>(s + Cfg::toff(8 * g + j, (16 * i + r) * 4));
  Frag<float> f;
  f.from8(v);
  return f;
}

// One operand's stage: ROWS (M or N) x KS (K) elements through registers into LDS.
// KC: stored [row][ld] with K contiguous; else [k][ld] with the rows contiguous.
template <typename T, bool KC, int ROWS>
struct GStage {
  using Cfg = GCfg<T>;
  static constexpr int KS = Cfg::KS, VEC = Cfg::VEC;
  static constexpr int CHUNKS = ROWS * KS / VEC;             // 16-byte chunks per stage
  static constexpr int PER = (CHUNKS + G_THREADS - 1) / G_THREADS;
  static constexpr int CPR = KC ? KS / VEC : ROWS / VEC;     // chunks per stored row
  uint4 v[PER];

  // rows [row0, row0 + ROWS) of nrows, k [k0, k0 + KS) of klim; VL: 16-byte loads allowed
  template <bool VL>
  __device__ __forceinline__ void load(const T* __restrict__ base, long long ld, int row0, int nrows, int k0,
                                       int klim, int tid) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = tid + G_THREADS * u;
      v[u] = make_uint4(0u, 0u, 0u, 0u);
      if (CHUNKS % G_THREADS != 0 && c >= CHUNKS) continue;
      const int major = c / CPR, minor = (c % CPR) * VEC;
      const int row = KC ? row0 + major : row0 + minor;  // first row of the chunk
      const int k = KC ? k0 + minor : k0 + major;        // first k of the chunk
      const T* src = KC ? base + (long long)row * ld + k : base + (long long)k * ld + row;
      if constexpr (VL) {
        if (KC ? (row < nrows && k < klim) : (k < klim && row < nrows)) v[u] = *reinterpret_cast<const uint4*>(src);
      } else {
        T e[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const bool ok = KC ? (row < nrows && k + j < klim) : (k < klim && row + j < nrows);
          e[j] = ok ? src[j] : T(0);
        }
        __builtin_memcpy(&v[u], e, 16);
      }
    }
  }
  __device__ __forceinline__ void store(char* s, int tid) const {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = tid + G_THREADS * u;
      if (CHUNKS % G_THREADS != 0 && c >= CHUNKS) continue;
      const int major = c / CPR, minor = c % CPR;
      if (KC)
        *reinterpret_cast<uint4*>(s + koff(major, minor)) = v[u];
      else
        *reinterpret_cast<uint4*>(s + Cfg::toff(major, minor * 16)) = v[u];
    }
  }
  static constexpr int bytes() { return KC ? ROWS * 128 : KS * Cfg::TROW; }
};

template <typename T, bool KC>
__device__ __forceinline__ Frag<T> gfrag(const char* s, int i, int ks, int lane) {
  if constexpr (sizeof(T) == 2)
    return KC ? frag_k(s, i, ks, lane) : frag_t(s, i, ks, lane);
  else
    return KC ? frag_k_f32(s, i, lane) : frag_t_f32(s, i, lane);
}

struct GArgs {
  int M, N, K;
  const void* A;
  long long lda, sa;
  const void* B;
  long long ldb, sb;
  const float* bias;
  int act, bias_m;
  const void* R;
  long long ldr, sr;
  void* C;
  long long ldc, sc;
  int c_f32;    // C stored as float32
  int r_f32;    // R read as float32
  int c_round;  // values rounded to bf16 before the float32 store (c_f32 = 2)
  int splits, kchunk;
  float* part;  // split-K partials [batch*splits][M][N]
  int vec_a, vec_b;
};

__device__ __forceinline__ float g_act(float v, int act) {
  if (act == RGBD_ACT_RELU) return fmaxf(v, 0.f);
  if (act == RGBD_ACT_GELU) return 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
  return v;
}

// R in C's dtype: float32 when C is written as float32, else the operand dtype
template <typename T>
__device__ __forceinline__ float g_r(const GArgs& a, long long ridx) {
  return a.r_f32 ? reinterpret_cast<const float*>(a.R)[ridx] : Num<T>::to_f(reinterpret_cast<const T*>(a.R)[ridx]);
}

// epilogue of one value: act(v + bias) (+ R) | v * (R > 0); bias indexed by n (nn.Linear) or,
// with bias_m, by m (a 1x1 / im2col convolution's output channel in NCHW)
template <typename T>
__device__ __forceinline__ float g_epi(float v, int m, int n, long long ridx, const GArgs& a) {
  if (a.act == RGBD_ACT_RELU_GRAD) return g_r<T>(a, ridx) > 0.f ? v : 0.f;
  if (a.bias) v += a.bias[a.bias_m ? m : n];
  v = g_act(v, a.act);
  if (a.R) v += g_r<T>(a, ridx);
  return v;
}

template <typename T>
__device__ __forceinline__ void g_store(const GArgs& a, int bz, int m, int n0, const float (&v)[4]) {
  // four consecutive n of row m
  if (a.c_f32) {
    float* c = reinterpret_cast<float*>(a.C) + (long long)bz * a.sc + (long long)m * a.ldc + n0;
    float w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) w[e] = a.c_round ? bf16_to_f32(f32_to_bf16(v[e])) : v[e];
    if (n0 + 3 < a.N && ((a.ldc | n0) & 3) == 0 && (((uintptr_t)a.C) & 15) == 0 && (a.sc & 3) == 0)
      *reinterpret_cast<float4*>(c) = make_float4(w[0], w[1], w[2], w[3]);
    else
      for (int e = 0; e < 4; ++e)
        if (n0 + e < a.N) c[e] = w[e];
  } else {
    T* c = reinterpret_cast<T*>(a.C) + (long long)bz * a.sc + (long long)m * a.ldc + n0;
    if constexpr (sizeof(T) == 2) {
      if (n0 + 3 < a.N && ((a.ldc | n0) & 3) == 0 && (((uintptr_t)a.C) & 7) == 0 && (a.sc & 3) == 0) {
        *reinterpret_cast<uint2*>(c) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
        return;
      }
    }
    for (int e = 0; e < 4; ++e)
      if (n0 + e < a.N) c[e] = Num<T>::from_f(v[e]);
  }
}

// Epilogue staging: the float32 accumulator tile [TM][TN] in LDS, 16-byte chunk c of row m at
// slot c ^ (m & (chunks - 1)) (conflict-free writes from the MFMA layout, conflict-free row reads).
template <int TN>
__device__ __forceinline__ int coff(int m, int chunk) {
  constexpr int CH = TN / 4;
  return (m * CH + (chunk ^ (m & (CH - 1)))) * 16;
}

// 8 consecutive outputs n0..n0+7 of row m: epilogue, store (16-byte stores when aligned)
template <typename T>
__device__ __forceinline__ void g_store8(const GArgs& a, int b, int bz, int m, int n0, float (&v)[8], bool vec_c) {
  if (a.splits > 1) {  // float32 partial of this split, ld = N
    float* p = a.part + ((long long)bz * a.M + m) * a.N + n0;
    if (vec_c && n0 + 8 <= a.N) {
      *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      for (int e = 0; e < 8; ++e)
        if (n0 + e < a.N) p[e] = v[e];
    }
    return;
  }
  const long long rbase = (long long)b * a.sr + (long long)m * a.ldr + n0;
  if (vec_c && n0 + 8 <= a.N && (a.R || a.bias)) {
    // whole row piece: the residual / bias values loaded together (wide loads) before use; per
    // element behind `n0 + e < N` each load was its own memory round trip.  Same arithmetic as
    // g_epi.  (vec_c implies 16-byte aligned R rows.)
    float rr[8], bb[8];
    if (a.R) {
      if (a.r_f32) {
        const float4 x = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(a.R) + rbase);
        const float4 y = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(a.R) + rbase + 4);
        rr[0] = x.x; rr[1] = x.y; rr[2] = x.z; rr[3] = x.w; rr[4] = y.x; rr[5] = y.y; rr[6] = y.z; rr[7] = y.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) rr[e] = Num<T>::to_f(reinterpret_cast<const T*>(a.R)[rbase + e]);
      }
    }
    if (a.bias && a.act != RGBD_ACT_RELU_GRAD) {
#pragma unroll
      for (int e = 0; e < 8; ++e) bb[e] = a.bias[a.bias_m ? m : n0 + e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (a.act == RGBD_ACT_RELU_GRAD) {
        v[e] = rr[e] > 0.f ? v[e] : 0.f;
        continue;
      }
      if (a.bias) v[e] += bb[e];
      v[e] = g_act(v[e], a.act);
      if (a.R) v[e] += rr[e];
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (n0 + e < a.N) v[e] = g_epi<T>(v[e], m, n0 + e, rbase + e, a);
  }
  if (a.c_f32) {
    float* c = reinterpret_cast<float*>(a.C) + (long long)b * a.sc + (long long)m * a.ldc + n0;
    if (a.c_round) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = bf16_to_f32(f32_to_bf16(v[e]));
    }
    if (vec_c && n0 + 8 <= a.N) {
      *reinterpret_cast<float4*>(c) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(c + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      for (int e = 0; e < 8; ++e)
        if (n0 + e < a.N) c[e] = v[e];
    }
  } else {
    T* c = reinterpret_cast<T*>(a.C) + (long long)b * a.sc + (long long)m * a.ldc + n0;
    if constexpr (sizeof(T) == 2) {
      if (vec_c && n0 + 8 <= a.N) {
        *reinterpret_cast<uint4*>(c) = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                                  pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
        return;
      }
    }
    for (int e = 0; e < 8; ++e)
      if (n0 + e < a.N) c[e] = Num<T>::from_f(v[e]);
  }
}

// The staged accumulator tile's epilogue for one batch entry, no split: thread = 8 columns of NR
// rows.  The bias (the same 8 columns for every row) and every row's residual are loaded before
// any use, then g_store8's arithmetic (bias, act, + R) and 16-byte stores.  One row at a time,
// each row's bias / residual loads were a memory round trip of their own (the bias epilogue took
// a (50400 x 1024, K 256) forward from 69 to 130 us).  Returns false (nothing done) outside the
// vector shape: the caller's per-row path then runs.
template <typename T, int TM, int TN, int NT>
__device__ __forceinline__ bool g_epi_rows(const GArgs& a, const char* smem, int tid, int b, int m_base, int n_base,
                                           bool vec_c) {
  constexpr int TPR = TN / 8, RPP = NT / TPR, NR = TM / RPP;
  const int nl = (tid % TPR) * 8, n0 = n_base + nl;
  if (!(a.splits == 1 && vec_c && !a.bias_m && n0 + 8 <= a.N && (((uintptr_t)a.bias) & 15) == 0)) return false;
  float bb[8];
  if (a.bias && a.act != RGBD_ACT_RELU_GRAD) {
    const float4 x = *reinterpret_cast<const float4*>(a.bias + n0), y = *reinterpret_cast<const float4*>(a.bias + n0 + 4);
    bb[0] = x.x; bb[1] = x.y; bb[2] = x.z; bb[3] = x.w; bb[4] = y.x; bb[5] = y.y; bb[6] = y.z; bb[7] = y.w;
  }
  float rr[NR][8];
  if (a.R) {
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      const int m = m_base + tid / TPR + q * RPP;
      const long long rb = (long long)b * a.sr + (long long)(m < a.M ? m : 0) * a.ldr + n0;
      if (a.r_f32) {
        const float4 x = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(a.R) + rb);
        const float4 y = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(a.R) + rb + 4);
        rr[q][0] = x.x; rr[q][1] = x.y; rr[q][2] = x.z; rr[q][3] = x.w;
        rr[q][4] = y.x; rr[q][5] = y.y; rr[q][6] = y.z; rr[q][7] = y.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) rr[q][e] = Num<T>::to_f(reinterpret_cast<const T*>(a.R)[rb + e]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NR; ++q) {
    const int ml = tid / TPR + q * RPP, m = m_base + ml;
    if (m >= a.M) continue;
    const f32x4 lo = *reinterpret_cast<const f32x4*>(smem + coff<TN>(ml, nl / 4));
    const f32x4 hi = *reinterpret_cast<const f32x4*>(smem + coff<TN>(ml, nl / 4 + 1));
    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (a.act == RGBD_ACT_RELU_GRAD) {
        v[e] = rr[q][e] > 0.f ? v[e] : 0.f;
        continue;
      }
      if (a.bias) v[e] += bb[e];
      v[e] = g_act(v[e], a.act);
      if (a.R) v[e] += rr[q][e];
    }
    if (a.c_f32) {
      float* c = reinterpret_cast<float*>(a.C) + (long long)b * a.sc + (long long)m * a.ldc + n0;
      if (a.c_round) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = bf16_to_f32(f32_to_bf16(v[e]));
      }
      *reinterpret_cast<float4*>(c) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(c + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      T* c = reinterpret_cast<T*>(a.C) + (long long)b * a.sc + (long long)m * a.ldc + n0;
      if constexpr (sizeof(T) == 2) {
        *reinterpret_cast<uint4*>(c) = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                                  pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) c[e] = Num<T>::from_f(v[e]);
      }
    }
  }
  return true;
}

template <typename T, int TM, int TN, bool AT, bool BT, bool VEC>
__global__ __launch_bounds__(G_THREADS) __attribute__((amdgpu_waves_per_eu(2, 4))) void k_gemm(GArgs a) {
  using Cfg = GCfg<T>;
  constexpr int KS = Cfg::KS;
  using SA = GStage<T, !AT, TM>;
  using SB = GStage<T, !BT, TN>;
  constexpr int A_BYTES = SA::bytes(), B_BYTES = SB::bytes();
  constexpr int FM = TM / 32, FN = TN / 32;  // fragments per wave (2 x 2 waves)
  constexpr int SMEM = 2 * (A_BYTES + B_BYTES) > TM * TN * 4 ? 2 * (A_BYTES + B_BYTES) : TM * TN * 4;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int n_base = blockIdx.x * TN, m_base = blockIdx.y * TM;
  const int bz = blockIdx.z, b = bz / a.splits, sp = bz % a.splits;
  const int kbeg = sp * a.kchunk, kend = min(a.K, kbeg + a.kchunk);
  const T* Ab = reinterpret_cast<const T*>(a.A) + (long long)b * a.sa;
  const T* Bb = reinterpret_cast<const T*>(a.B) + (long long)b * a.sb;

  f32x4 acc[FN][FM];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < FM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // K stages through PD register sets and two LDS buffers: the loads of stage kt + PD are issued
  // while stage kt is multiplied and are stored to LDS PD - 1 stages later (the barrier between
  // stages waits for LDS traffic only; loads stay in flight across it).  PD = 2 for the 128 x 128
  // tiles (register budget); PD = 4 for the 64 x 64 tiles of small GEMMs, whose stages are short
  // and otherwise each wait for a load issued only one stage earlier.
  constexpr int PD = TM == 64 ? 4 : 2;
  SA ra[PD];
  SB rb[PD];
  const int nk = kend > kbeg ? (kend - kbeg + KS - 1) / KS : 0;
  auto load = [&](SA& ra, SB& rb, int kt) {
    const int k0 = kbeg + kt * KS;
    ra.template load<VEC>(Ab, a.lda, m_base, a.M, k0, kend, tid);
    rb.template load<VEC>(Bb, a.ldb, n_base, a.N, k0, kend, tid);
  };
  auto put = [&](const SA& ra, const SB& rb, int buf) {
    char* d = smem + buf * (A_BYTES + B_BYTES);
    ra.store(d, tid);
    rb.store(d + A_BYTES, tid);
  };
  auto compute = [&](int buf) {
    const char* s_a = smem + buf * (A_BYTES + B_BYTES);
    const char* s_b = s_a + A_BYTES;
    // one k-step's fragments live at a time (both unrolled, the 128 x 128 bf16 tile spills)
#pragma unroll 1
    for (int ks = 0; ks < KS / 32; ++ks) {
      Frag<T> fm[FM], fn[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fm[i] = gfrag<T, !AT>(s_a, wm * FM + i, ks, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) fn[j] = gfrag<T, !BT>(s_b, wn * FN + j, ks, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i) mma(acc[j][i], fn[j], fm[i]);
    }
  };
#pragma unroll
  for (int j = 0; j < PD; ++j)
    if (j < nk) load(ra[j], rb[j], j);
  if (nk > 0) put(ra[0], rb[0], 0);
  lds_barrier();
  // step kt: register set kt % PD went to LDS buffer kt % 2 before the last barrier and takes
  // stage kt + PD now; set (kt + 1) % PD goes to the other buffer after the multiply
  auto step = [&](auto J, int kt) {
    constexpr int j = decltype(J)::value;
    if (kt + PD < nk) load(ra[j], rb[j], kt + PD);
    compute(j & 1);
    if (kt + 1 < nk) put(ra[(j + 1) % PD], rb[(j + 1) % PD], (j + 1) & 1);
    lds_barrier();
  };
  for (int kt = 0; kt < nk; kt += PD) {
    step(std::integral_constant<int, 0>{}, kt);
    if (kt + 1 >= nk) break;
    step(std::integral_constant<int, 1>{}, kt + 1);
    if constexpr (PD == 4) {
      if (kt + 2 >= nk) break;
      step(std::integral_constant<int, 2>{}, kt + 2);
      if (kt + 3 >= nk) break;
      step(std::integral_constant<int, 3>{}, kt + 3);
    }
  }

  // epilogue: accumulators -> LDS (float32 tile) -> rows of 8 outputs per thread, coalesced
  // 16-byte stores.  lane (r, g): acc[j][i][e] = C[m = 16 (wm FM + i) + r][n = 16 (wn FN + j) + 4 g + e]
  {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int ml = 16 * (wm * FM + i) + r, ch = 4 * (wn * FN + j) + g;
        *reinterpret_cast<f32x4*>(smem + coff<TN>(ml, ch)) = acc[j][i];
      }
  }
  lds_barrier();
  const bool vec_c = a.splits > 1 ? (a.N % 4 == 0)
                                  : ((a.N % 8 == 0) && (((uintptr_t)a.C) % 16 == 0) && (a.ldc % 8 == 0) &&
                                     (a.sc % 8 == 0) && (!a.R || (a.ldr % 8 == 0 && a.sr % 8 == 0 && ((uintptr_t)a.R) % 16 == 0)));
  if (g_epi_rows<T, TM, TN, G_THREADS>(a, smem, tid, b, m_base, n_base, vec_c)) return;
  constexpr int TPR = TN / 8, RPP = G_THREADS / TPR;  // threads per row, rows per pass
  const int nl = (tid % TPR) * 8;
#pragma unroll 1
  for (int ml = tid / TPR; ml < TM; ml += RPP) {
    const int m = m_base + ml, n0 = n_base + nl;
    if (m >= a.M || n0 >= a.N) continue;
    const f32x4 lo = *reinterpret_cast<const f32x4*>(smem + coff<TN>(ml, nl / 4));
    const f32x4 hi = *reinterpret_cast<const f32x4*>(smem + coff<TN>(ml, nl / 4 + 1));
    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    g_store8<T>(a, b, bz, m, n0, v, vec_c);
  }
}

// split-K reduction (splits summed in order) + epilogue; thread = 4 consecutive n
template <typename T>
__global__ __launch_bounds__(256) void k_gemm_splitk_reduce(GArgs a, int batch) {
  const long long quads_per_row = (a.N + 3) / 4;
  const long long total = (long long)batch * a.M * quads_per_row;
  for (long long t = blockIdx.x * 256ll + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int b = (int)(t / ((long long)a.M * quads_per_row));
    const long long rem = t % ((long long)a.M * quads_per_row);
    const int m = (int)(rem / quads_per_row), n0 = (int)(rem % quads_per_row) * 4;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    const long long rbase = (long long)b * a.sr + (long long)m * a.ldr + n0;
    if ((a.N & 3) == 0 && (((uintptr_t)a.part) & 15) == 0) {
      // whole quads (16-byte aligned partial rows): one load per split, no branches, so the
      // splits' loads and the epilogue's residual / bias loads are in flight together (behind
      // per-element branches each was a memory round trip); same summation order
#pragma unroll 4
      for (int s = 0; s < a.splits; ++s) {
        const float4 q = *reinterpret_cast<const float4*>(a.part + (((long long)b * a.splits + s) * a.M + m) * a.N + n0);
        v[0] += q.x;
        v[1] += q.y;
        v[2] += q.z;
        v[3] += q.w;
      }
      float rr[4], bb[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        rr[e] = a.R ? g_r<T>(a, rbase + e) : 0.f;
        bb[e] = a.bias && a.act != RGBD_ACT_RELU_GRAD ? a.bias[a.bias_m ? m : n0 + e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (a.act == RGBD_ACT_RELU_GRAD) {
          v[e] = rr[e] > 0.f ? v[e] : 0.f;
          continue;
        }
        if (a.bias) v[e] += bb[e];
        v[e] = g_act(v[e], a.act);
        if (a.R) v[e] += rr[e];
      }
    } else {
      for (int s = 0; s < a.splits; ++s) {
        const float* p = a.part + (((long long)b * a.splits + s) * a.M + m) * a.N + n0;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (n0 + e < a.N) v[e] += p[e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (n0 + e < a.N) v[e] = g_epi<T>(v[e], m, n0 + e, rbase + e, a);
    }
    g_store<T>(a, b, m, n0, v);
  }
}

// bias gradient: out[n] = sum_m y[m][n], float32, fixed order, in one launch.  The rows in
// chunks sized so that the launch has about CS_TARGET blocks (at least 32 rows per chunk, at most
// CS_MAXCH chunks): a [50400 x 256] bias gradient gets 256 chunks, not one block per CU quarter.
// Block = 256 columns x one chunk, 256 threads = 32 column groups of 8 (one 16-byte load per row
// when aligned, four rows in flight) x 8 row lanes folded through LDS in fixed order -> the
// chunk's partial, stored write-through (sc1); the last chunk of a column block to take its ticket
// (agent-scope counter, after every partial store drained) sums the partials in chunk order with
// the same 8-row-lane x 32-column-group split (loads sc1, MI355X_MICROARCH.md visibility table,
// row 1), then rearms the ticket.  Deterministic for a given shape.
constexpr int CS_MAXCH = 256, CS_TARGET = 1024;

inline int cs_chunks(int rows, int N) {
  const int nbx = std::max(1, ceil_div(N, 256));
  return std::min({CS_MAXCH, std::max(1, ceil_div(rows, 32)), std::max(1, ceil_div(CS_TARGET, nbx))});
}
// the tickets occupy a fixed head of the workspace whatever N is, so calls of different widths on
// one workspace never see each other's partials as tickets
constexpr int CS_MAXBLK = 1024;  // column blocks: N <= 262 144
inline size_t cs_ticket_bytes(int) { return CS_MAXBLK * sizeof(int); }

template <typename T>
__global__ __launch_bounds__(256) void k_colsum(const T* __restrict__ y, int rows, int N, long long ld, int chunk,
                                                int vec, int* __restrict__ tickets, float* __restrict__ part,
                                                float* __restrict__ out) {
  __shared__ float red[8][256];
  __shared__ int last_s;
  const int cg = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c0 = blockIdx.x * 256 + 8 * cg;
  const int r0 = blockIdx.y * chunk, r1 = min(rows, r0 + chunk);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < N) {
    if (vec && c0 + 8 <= N) {
#pragma unroll 8
      for (int m = r0 + rl; m < r1; m += 8) {
        Frag<T> f;
        f.load(y + (long long)m * ld + c0);
        float v[8];
        f.to8(v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[j];
      }
    } else {
      for (int m = r0 + rl; m < r1; m += 8) {
        const T* row = y + (long long)m * ld + c0;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += c0 + j < N ? Num<T>::to_f(row[j]) : 0.f;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][8 * cg + j] = acc[j];
  __syncthreads();
  const int nch = gridDim.y;
  const __amdgpu_buffer_rsrc_t prs = wt_rsrc(part, nch * N * (int)sizeof(float));
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c < N) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][threadIdx.x];
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(t), prs, (blockIdx.y * N + c) * 4, 0, WT_SC1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last_s = __hip_atomic_fetch_add(tickets + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nch - 1;
  __syncthreads();
  if (!last_s) return;
  // the chunks' partials: row lane rl takes chunks rl, rl + 8, ... (in order), then the 8 lanes
  // fold in fixed order
  float t8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if ((N & 3) == 0 && c0 + 8 <= N) {
    // two 16-byte loads per partial row, eight rows' loads in flight
#pragma unroll 8
    for (int k = rl; k < nch; k += 8) {
      const v4u a = __builtin_amdgcn_raw_buffer_load_b128(prs, (k * N + c0) * 4, 0, WT_SC1);
      const v4u b = __builtin_amdgcn_raw_buffer_load_b128(prs, (k * N + c0 + 4) * 4, 0, WT_SC1);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t8[j] += __uint_as_float(a[j]);
        t8[4 + j] += __uint_as_float(b[j]);
      }
    }
  } else {
#pragma unroll 4
    for (int k = rl; k < nch; k += 8)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (c0 + j < N) t8[j] += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(prs, (k * N + c0 + j) * 4, 0, WT_SC1));
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][8 * cg + j] = t8[j];
  __syncthreads();
  if (c < N) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][threadIdx.x];
    out[c] = t;
  }
  if (threadIdx.x == 0) tickets[blockIdx.x] = 0;  // rearmed for the next call on this workspace
}

// ---- bf16, both operands K-contiguous (forward: X [M][K] W [N][K]; dX with the weight
// transposed), batch 1, no split: the conv5 recipe (ratio.hip k_rp_conv3x3_v3) on a plain
// GEMM.  512 threads = 8 waves as 2 (M) x 4 (N), wave tile (TM/2) x (TN/4); K staged 64 at a
// time (128-byte rows, 16-byte chunk c at slot c ^ (row & 7)) by LDS-DMA straight from global
// memory (global_load_lds_dwordx4: no VGPR staging, no ds_write) into an S-stage ring issued
// S - 1 stages ahead, one barrier per stage; rows past M / N and chunks past K read a zero line.  The
// blockIdx -> tile map keeps the N tiles of one M tile on one XCD (workgroup i runs on XCD
// i % 8), so X is fetched from HBM once and re-read from that XCD's L2.  Epilogue: the
// accumulator tile through LDS, 16-byte row stores with bias / act / residual / ReLU-mask.
__device__ uint4 g_zero_line[4];  // 64 zero bytes (never written)

__device__ __forceinline__ void gl_dma16(const void* gsrc, uint32_t lds_base) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_base)
               : "memory");
}

constexpr int GL_THREADS = 512;
template <int TM, int TN, int S>
struct GlCfg {
  static constexpr int FM = TM / 32, FN = TN / 64;  // fragments per wave: 2 (M) x 4 (N) waves
  static constexpr int A_BYTES = TM * 128, B_BYTES = TN * 128, STAGE = A_BYTES + B_BYTES;
  static constexpr int PIECES = STAGE / 1024, PER_WAVE = PIECES / 8;
  static constexpr int SMEM = S * STAGE > TM * TN * 4 ? S * STAGE : TM * TN * 4;
  static_assert(PIECES % 8 == 0 && SMEM <= 163840, "LDS-DMA GEMM tile");
};

// s_waitcnt immediate (gfx9 encoding): vmcnt(vm), lgkmcnt(lgkm), expcnt not waited
constexpr int gl_waitcnt(int vm, int lgkm) { return (vm & 15) | (7 << 4) | ((lgkm & 15) << 8) | ((vm >> 4) << 14); }

// TT: both operands stored [K][rows] with the rows contiguous (a_t = b_t = 1: a weight gradient
// dY^T X, K = tokens), split-K over blockIdx.y.  Stages of 64 k-rows x 256 bytes per operand,
// read back k-major with ds_read_tr16_b64 (frag_t, GCfg<bf16_t>::toff's 32-byte-block swizzle
// applied on the DMA's per-lane source addresses).
template <int TM, int TN, int S, bool TT = false>
__global__ __launch_bounds__(GL_THREADS, S == 2 ? 2 : 1) void k_gemm_lds(GArgs a) {
  using C = GlCfg<TM, TN, S>;
  static_assert(!TT || (TM == 128 && TN == 128), "TT stages: 128 columns = 256-byte rows");
  constexpr int FM = C::FM, FN = C::FN;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  // tile of this workgroup: XCD-major over consecutive tiles (n fastest)
  const int ntn = (a.N + TN - 1) / TN;
  const int T = ntn * ((a.M + TM - 1) / TM), full = T / 8 * 8;
  const int bid = blockIdx.x;
  const int t = bid < full ? (bid % 8) * (full / 8) + bid / 8 : bid;
  const int m_base = (t / ntn) * TM, n_base = (t % ntn) * TN;
  const bf16_t* A = reinterpret_cast<const bf16_t*>(a.A);
  const bf16_t* B = reinterpret_cast<const bf16_t*>(a.B);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const int sp = TT ? (int)blockIdx.y : 0;
  const int kbeg = TT ? sp * a.kchunk : 0, kend = TT ? min(a.K, kbeg + a.kchunk) : a.K;
  const int nk = kend > kbeg ? (kend - kbeg + 63) / 64 : 0;

  auto issue = [&](int kt, int buf) {
    const int k0 = kbeg + kt * 64;
#pragma unroll
    for (int u = 0; u < C::PER_WAVE; ++u) {
      const int p = wave * C::PER_WAVE + u;
      const bool is_a = p < C::A_BYTES / 1024;
      const void* src = g_zero_line;
      if constexpr (TT) {
        // piece = 4 k-rows x 256 B; lane -> row 4p + lane/16, physical 16-byte slot lane%16 of the
        // row, which holds logical 32-byte block (slot/2) ^ swz(row)
        const int row = (is_a ? p : p - C::A_BYTES / 1024) * 4 + (lane >> 4);
        const int slot = lane & 15;
        const int swz = (row & 3) | (((row >> 3) & 1) << 2);
        const int col = (((slot >> 1) ^ swz) << 4) + 8 * (slot & 1);
        const int gk = k0 + row, gc = (is_a ? m_base : n_base) + col;
        if (gk < kend && gc < (is_a ? a.M : a.N))
          src = is_a ? (const void*)(A + (long long)gk * a.lda + gc) : (const void*)(B + (long long)gk * a.ldb + gc);
      } else {
        // piece p of a stage: 8 rows of A (p < TM / 8) or of B; lane -> row p*8 + lane/8, slot lane%8
        const int row = (is_a ? p : p - TM / 8) * 8 + (lane >> 3);
        const int q = (lane & 7) ^ (row & 7);
        const int gr = (is_a ? m_base : n_base) + row, k = k0 + 8 * q;
        if (gr < (is_a ? a.M : a.N) && k < a.K)
          src = is_a ? (const void*)(A + (long long)gr * a.lda + k) : (const void*)(B + (long long)gr * a.ldb + k);
      }
      gl_dma16(src, lds0 + buf * C::STAGE + p * 1024);
    }
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < FM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // stages 0 .. S-2 ahead; stage kt + S - 1 is issued at the start of step kt
#pragma unroll
  for (int j = 0; j < S - 1; ++j)
    if (j < nk) issue(j, j);
  if (S == 3 && nk > 1)
    __builtin_amdgcn_s_waitcnt(gl_waitcnt(C::PER_WAVE, 15));
  else
    __builtin_amdgcn_s_waitcnt(gl_waitcnt(0, 15));
  __syncthreads();
#pragma unroll 1
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + S - 1 < nk;
    if (more) issue(kt + S - 1, (kt + S - 1) % S);
    const char* sa = smem + (kt % S) * C::STAGE;
    const char* sb = sa + C::A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      Frag<bf16_t> fm[FM], fn[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fm[i] = TT ? frag_t(sa, wm * FM + i, ks, lane) : frag_k(sa, wm * FM + i, ks, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) fn[j] = TT ? frag_t(sb, wn * FN + j, ks, lane) : frag_k(sb, wn * FN + j, ks, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i) mma(acc[j][i], fn[j], fm[i]);
    }
    // the next stage landed (this wave's pieces; the barrier covers the others'), reads done
    if (S == 3 && more)
      __builtin_amdgcn_s_waitcnt(gl_waitcnt(C::PER_WAVE, 0));
    else
      __builtin_amdgcn_s_waitcnt(gl_waitcnt(0, 0));
    __builtin_amdgcn_s_barrier();
  }

  // epilogue as k_gemm's: lane (r, g): acc[j][i][e] = C[m = 16 (wm FM + i) + r][n = 16 (wn FN + j) + 4 g + e]
  {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int ml = 16 * (wm * FM + i) + r, ch = 4 * (wn * FN + j) + g;
        *reinterpret_cast<f32x4*>(smem + coff<TN>(ml, ch)) = acc[j][i];
      }
  }
  __syncthreads();
  const bool vec_c = a.splits > 1 ? (a.N % 4 == 0)
                                  : ((a.N % 8 == 0) && (((uintptr_t)a.C) % 16 == 0) && (a.ldc % 8 == 0) &&
                                     (!a.R || (a.ldr % 8 == 0 && ((uintptr_t)a.R) % 16 == 0)));
  constexpr int TPR = TN / 8, RPP = GL_THREADS / TPR;
  const int nl = (tid % TPR) * 8;
  if (g_epi_rows<bf16_t, TM, TN, GL_THREADS>(a, smem, tid, 0, m_base, n_base, vec_c)) return;
#pragma unroll 1
  for (int ml = tid / TPR; ml < TM; ml += RPP) {
    const int m = m_base + ml, n0 = n_base + nl;
    if (m >= a.M || n0 >= a.N) continue;
    const f32x4 lo = *reinterpret_cast<const f32x4*>(smem + coff<TN>(ml, nl / 4));
    const f32x4 hi = *reinterpret_cast<const f32x4*>(smem + coff<TN>(ml, nl / 4 + 1));
    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    g_store8<bf16_t>(a, 0, sp, m, n0, v, vec_c);  // splits > 1: the split's float32 partial
  }
}

template <int TM, int TN, int S, bool TT = false>
int launch_lds(const GArgs& a, hipStream_t s) {
  using C = GlCfg<TM, TN, S>;
  static const hipError_t attr = hipFuncSetAttribute((const void*)k_gemm_lds<TM, TN, S, TT>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, C::SMEM);
  if (attr != hipSuccess) return (int)attr;
  const int T = ceil_div(a.N, TN) * ceil_div(a.M, TM);
  k_gemm_lds<TM, TN, S, TT><<<dim3(T, TT ? a.splits : 1), GL_THREADS, C::SMEM, s>>>(a);
  RGBD_CHECK_LAUNCH();
  if (TT && a.splits > 1) {
    const long long quads = (long long)a.M * ((a.N + 3) / 4);
    const int blocks = (int)std::min<long long>((quads + 255) / 256, 4096);
    hipLaunchKernelGGL(k_gemm_splitk_reduce<bf16_t>, dim3(blocks), dim3(256), 0, s, a, 1);
    RGBD_CHECK_LAUNCH();
  }
  return RGBD_OK;
}

template <typename T, int TM, int TN, bool AT, bool BT>
void launch_t(const GArgs& a, int batch, hipStream_t s) {
  dim3 grid(ceil_div(a.N, TN), ceil_div(a.M, TM), batch * a.splits);
  if (a.vec_a && a.vec_b)
    hipLaunchKernelGGL((k_gemm<T, TM, TN, AT, BT, true>), grid, dim3(G_THREADS), 0, s, a);
  else
    hipLaunchKernelGGL((k_gemm<T, TM, TN, AT, BT, false>), grid, dim3(G_THREADS), 0, s, a);
}

template <typename T, int TM, int TN>
void launch_layout(const GArgs& a, int at, int bt, int batch, hipStream_t s) {
  if (!at && !bt) launch_t<T, TM, TN, false, false>(a, batch, s);
  else if (!at && bt) launch_t<T, TM, TN, false, true>(a, batch, s);
  else if (at && !bt) launch_t<T, TM, TN, true, false>(a, batch, s);
  else launch_t<T, TM, TN, true, true>(a, batch, s);
}

template <typename T>
int gemm_t(GArgs a, int at, int bt, int batch, hipStream_t s) {
  if constexpr (sizeof(T) == 2) {
    // the LDS-DMA kernel: bf16, both operands K-contiguous and 16-byte aligned, one GEMM, no split
    if (!at && !bt && batch == 1 && a.splits == 1 && a.vec_a && a.vec_b && a.K % 8 == 0 && !a.bias_m &&
        a.M >= 1024) {
      // 128 x 128 tiles with a 2-stage ring (64 KB of LDS: two workgroups per CU, one's prologue
      // and epilogue under the other's MFMAs); measured 1.2-1.6x faster than one workgroup per
      // CU with a 3-stage ring on the drop-in model's shapes (profiles/r04_v3/micro_gemm_lds.txt)
      return launch_lds<128, 128, 2>(a, s);
    }
    // weight gradients (both operands token-major): the LDS-DMA kernel with transposed fragment
    // reads (profiles/r04_v5/micro_gemm_dw_tt_ab.txt)
    if (at && bt && batch == 1 && a.vec_a && a.vec_b && a.M % 8 == 0 && a.N % 8 == 0 && !a.bias_m && !a.R &&
        a.K >= 1024)
      return launch_lds<128, 128, 2, true>(a, s);
  }
  // 128 x 128 tiles when they give the chip enough workgroups, else 64 x 64
  const long long big = (long long)ceil_div(a.N, 128) * ceil_div(a.M, 128) * batch * a.splits;
  if (big >= 256)
    launch_layout<T, 128, 128>(a, at, bt, batch, s);
  else
    launch_layout<T, 64, 64>(a, at, bt, batch, s);
  RGBD_CHECK_LAUNCH();
  if (a.splits > 1) {
    const long long quads = (long long)batch * a.M * ((a.N + 3) / 4);
    const int blocks = (int)std::min<long long>((quads + 255) / 256, 4096);
    hipLaunchKernelGGL(k_gemm_splitk_reduce<T>, dim3(blocks), dim3(256), 0, s, a, batch);
    RGBD_CHECK_LAUNCH();
  }
  return RGBD_OK;
}

}  // namespace
}  // namespace rgbd

using namespace rgbd;

extern "C" {

size_t rgbd_gemm_workspace_size(int M, int N, int batch, int splits) {
  if (splits <= 1) return 0;
  return (size_t)batch * splits * M * N * sizeof(float);
}

int rgbd_gemm(int dtype, int a_t, int b_t, int M, int N, int K, const void* A, long long lda, long long sa,
              const void* B, long long ldb, long long sb, const float* bias, int act, const void* R, long long ldr,
              long long sr, void* C, long long ldc, long long sc, int c_f32, int batch, int splits, void* ws,
              void* stream) {
  RGBD_REQUIRE(A && B && C && M > 0 && N > 0 && K > 0 && batch > 0 && splits > 0, RGBD_E_ARG);
  RGBD_REQUIRE(dtype == RGBD_F32 || dtype == RGBD_BF16, RGBD_E_ARG);
  const int bias_m = (act & RGBD_BIAS_M) != 0;
  act &= ~RGBD_BIAS_M;
  RGBD_REQUIRE(act >= RGBD_ACT_NONE && act <= RGBD_ACT_RELU_GRAD, RGBD_E_ARG);
  RGBD_REQUIRE(act != RGBD_ACT_RELU_GRAD || (R && !bias), RGBD_E_ARG);
  RGBD_REQUIRE(splits == 1 || ws, RGBD_E_ARG);
  RGBD_REQUIRE(lda >= (a_t ? M : K) && ldb >= (b_t ? N : K) && ldc >= N && (!R || ldr >= N), RGBD_E_SHAPE);
  const int esz = dtype == RGBD_BF16 ? 2 : 4, vec = 16 / esz;
  const int ks = dtype == RGBD_BF16 ? 64 : 32;
  GArgs a;
  a.M = M; a.N = N; a.K = K;
  a.A = A; a.lda = lda; a.sa = sa;
  a.B = B; a.ldb = ldb; a.sb = sb;
  a.bias = bias; a.act = act; a.bias_m = bias_m;
  a.R = R; a.ldr = ldr; a.sr = sr;
  RGBD_REQUIRE(c_f32 >= 0 && c_f32 <= 2, RGBD_E_ARG);
  a.C = C; a.ldc = ldc; a.sc = sc; a.c_f32 = c_f32 || dtype == RGBD_F32;
  a.r_f32 = a.c_f32 && !(c_f32 == 2 && dtype == RGBD_BF16);
  a.c_round = c_f32 == 2 && dtype == RGBD_BF16;
  a.splits = splits;
  a.kchunk = ((K + splits - 1) / splits + ks - 1) / ks * ks;
  a.part = (float*)ws;
  // 16-byte loads: the contiguous extent, the leading dimension, the batch stride and the base
  // all multiples of 16 bytes
  auto vec_ok = [&](const void* p, long long ld, long long st, int extent) {
    return (((uintptr_t)p) & 15) == 0 && ld % vec == 0 && (batch == 1 || st % vec == 0) && extent % vec == 0;
  };
  a.vec_a = vec_ok(A, lda, sa, a_t ? M : K);
  a.vec_b = vec_ok(B, ldb, sb, b_t ? N : K);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_BF16) return gemm_t<bf16_t>(a, a_t, b_t, batch, s);
  return gemm_t<float>(a, a_t, b_t, batch, s);
}

size_t rgbd_colsum_workspace_size(int rows, int N) {
  if (rows <= 0 || N <= 0) return 256;
  return cs_ticket_bytes(N) + (size_t)cs_chunks(rows, N) * N * sizeof(float);
}

int rgbd_colsum(int dtype, const void* y, int rows, int N, long long ld, float* out, void* ws, void* stream) {
  RGBD_REQUIRE(y && out && ws && rows > 0 && N > 0 && ld >= N, RGBD_E_ARG);
  RGBD_REQUIRE(dtype == RGBD_F32 || dtype == RGBD_BF16, RGBD_E_DTYPE);
  RGBD_REQUIRE(ceil_div(N, 256) <= CS_MAXBLK && (long long)cs_chunks(rows, N) * N * (long long)sizeof(float) < (1ll << 31),
               RGBD_E_SHAPE);
  hipStream_t s = (hipStream_t)stream;
  const int nch = cs_chunks(rows, N);
  const int chunk = ceil_div(rows, nch);
  const int esz = dtype == RGBD_BF16 ? 2 : 4;
  const int vec = (((uintptr_t)y) % 16 == 0) && ((ld * esz) % 16 == 0);
  int* tickets = (int*)ws;
  float* part = (float*)((char*)ws + cs_ticket_bytes(N));
  dim3 grid(ceil_div(N, 256), nch);
  if (dtype == RGBD_BF16)
    hipLaunchKernelGGL(k_colsum<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)y, rows, N, ld, chunk, vec, tickets,
                       part, out);
  else
    hipLaunchKernelGGL(k_colsum<float>, grid, dim3(256), 0, s, (const float*)y, rows, N, ld, chunk, vec, tickets, part,
                       out);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
