// f1: the masked cross-attention core of the Mask2Former decoder layers (gfx950; float32 or
// bfloat16 operands, float32 arithmetic).
//
// Reference (third-party, in the model the reference trains, custom_model.py:37-53):
// transformers 5.15 Mask2FormerMaskedAttentionDecoderLayer.forward_post (modeling_mask2former.py
// :1640-1647) calls nn.MultiheadAttention with the mask predictor's boolean attention mask
// (:2048-2055); torch's math path computes, per (batch*head) bh,
//     S = (q * head_dim^-1/2) k^T + where(mask, -inf, 0),  P = softmax(S),  O = P v
// (L = the level's pixels).  The in / out projections stay the module's GEMMs (library, genuine
// dense contractions); this file is the non-GEMM part.  Layout is sequence-major, as the
// projections produce it (no head transposes): q / o [Q][BH][32], k / v [L][BH][32], the
// per-row lse / delta [Q][BH]; the mask is the predictor's [BH][Q][L] bytes.
//
// Shapes here are few queries (100) against many keys (300 .. 19 200 per level), so the forward
// and dQ split the work over KEY ranges (flash-decoding style) to fill 256 CUs; partials are merged
// in split order (no atomics anywhere: the backward is deterministic).  The kernels run on fp32
// MFMA (v_mfma_f32_16x16x4_f32, exact f32 products and sums) over operands of type T: float32, or
// bfloat16 under torch.autocast (the projections then produce bf16 q / k / v; each element is
// widened exactly on load, so the core adds no rounding of its own beyond torch's bf16 path —
// the outputs o / dq / dk / dv are rounded to T once; lse and delta stay float32):
//   k_attn_fwd_mfma     wave = 16 queries; S^T = K q_scaled^T, online softmax per query column,
//                       O^T += V^T P^T with P^T taken straight from the accumulators; partial
//                       (max, sum, o) per split -> k_attn_merge (also writes the row log-sum-exp)
//   k_attn_bwd_kv_mfma  wave = 16 keys over all queries; S, dP, then dV^T += dO^T P, dK^T +=
//                       q_scaled^T dS, K / V tiles held in registers
//   k_attn_bwd_q_mfma   the forward's tiling: dq^T += K^T dS^T, partial per split -> k_attn_dq_sum
#include <cmath>

#include "common.hpp"

using namespace rgbd;

namespace {

constexpr int HD = 32;      // head dim (hidden 256 / 8 heads)
constexpr int QW = 64;      // queries per forward / dQ workgroup (4 waves x 16)
constexpr int KS = 64;      // key-split granularity

template <typename T>
struct AttnArgs {
  const T* q;            // [Q][BH][HD] (unscaled)
  const T* k;            // [L][BH][HD]
  const T* v;            // [L][BH][HD]
  const uint8_t* mask;   // [BH][Q][L] bool, true = not allowed
  T* o;                  // [Q][BH][HD]
  float* lse;            // [Q][BH] log-sum-exp of the scaled, masked scores
  float* part_o;         // [nsplit][Q][BH][HD]
  float* part_ml;        // [nsplit][Q][BH][2] = (max, sum)
  int BH, Q, L;
  int nsplit, span;      // key range of split s: [s*span, min(L, (s+1)*span)), span % KS == 0
  float scale;
  bool vec_mask;         // mask rows 16-byte aligned (L % 16 == 0)
};

// K / V tile staging for the MFMA forward and dQ: 64 keys x 32 dims of each, two float4 per
// thread per matrix, loaded one tile ahead into registers so the global loads overlap the
// current tile's MFMAs.
struct KVTile {
  float4 k[2], v[2];
};

// 4 consecutive elements (16-byte aligned float4, or 8-byte aligned bf16 x4) widened to float
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 ld4(const bf16_t* p) {
  const uint2 w = *reinterpret_cast<const uint2*>(p);
  return make_float4(__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u), __uint_as_float(w.y << 16),
                     __uint_as_float(w.y & 0xffff0000u));
}
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const bf16_t* p) { return bf16_to_f32(*p); }
__device__ __forceinline__ void st4(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}
__device__ __forceinline__ void st4(bf16_t* p, float a, float b, float c, float d) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf16x2(a, b), pack_bf16x2(c, d));
}
__device__ __forceinline__ void st1(float* p, float v) { *p = v; }
__device__ __forceinline__ void st1(bf16_t* p, float v) { *p = f32_to_bf16(v); }

template <typename T>
__device__ __forceinline__ void kv_load(KVTile& t, const T* K, const T* V, int k0, int ke, int BH, int bh, int tid) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = tid + 256 * j, row = idx >> 3, c = idx & 7, key = k0 + row;
    const bool ok = key < ke;
    // unconditional loads of a clamped key (zeroed after): behind the branch the compiler waited
    // for each load where it was issued, and the next tile's "prefetch" blocked the current one
    const long long off = ((long long)(ok ? key : ke - 1) * BH + bh) * HD + 4 * c;
    const float4 kk = ld4(K + off), vv = ld4(V + off);
    t.k[j] = ok ? kk : make_float4(0.f, 0.f, 0.f, 0.f);
    t.v[j] = ok ? vv : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

__device__ __forceinline__ void kv_store(float (*sk)[HD + 1], float (*sv)[HD + 1], const KVTile& t, int tid) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = tid + 256 * j, row = idx >> 3, c = idx & 7;
    sk[row][4 * c] = t.k[j].x; sk[row][4 * c + 1] = t.k[j].y; sk[row][4 * c + 2] = t.k[j].z; sk[row][4 * c + 3] = t.k[j].w;
    sv[row][4 * c] = t.v[j].x; sv[row][4 * c + 1] = t.v[j].y; sv[row][4 * c + 2] = t.v[j].z; sv[row][4 * c + 3] = t.v[j].w;
  }
}

// Forward on fp32 MFMA: a wave owns 16 queries (a workgroup 64), keys of the split staged 64 at a
// time in LDS; per 16-key block
//   S^T = K . q_scaled^T                     (16k x 16q, 8 MFMAs; q_scaled^T is the register-held
//                                             B operand; lane l holds key (l>>4)*4+i, query l&15)
//   online softmax per query column          (max / sum over i, then across the 4 lane groups)
//   O^T += V^T . P^T                         (32d x 16q, 8 MFMAs; P^T feeds the B operand from the
//                                             accumulators, chunk i contracts keys (l>>4)*4+i)
// Every accumulator of a lane belongs to its query column, so the rescale is a per-lane multiply.
typedef float f4m __attribute__((ext_vector_type(4)));

template <typename T>
__global__ __launch_bounds__(256) void k_attn_fwd_mfma(AttnArgs<T> a) {
  __shared__ float sk[64][HD + 1];
  __shared__ float sv[64][HD + 1];
  const int split = blockIdx.x, bh = blockIdx.y, tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int lc = l & 15, lg = l >> 4;
  const int qrow = blockIdx.z * 64 + w * 16 + lc;
  const bool qv = qrow < a.Q;
  float qb[8];  // B operand: q_scaled^T [d = 4c + lg][query lc]
#pragma unroll
  for (int c = 0; c < 8; ++c) qb[c] = ld1(a.q + ((long long)(qv ? qrow : 0) * a.BH + bh) * HD + 4 * c + lg);  // together
#pragma unroll
  for (int c = 0; c < 8; ++c) qb[c] = qv ? qb[c] * a.scale : 0.f;
  f4m o[2] = {f4m{0.f, 0.f, 0.f, 0.f}, f4m{0.f, 0.f, 0.f, 0.f}};
  float m = -INFINITY, lsum = 0.f;
  const int kb = split * a.span, ke = min(a.L, kb + a.span);
  const uint8_t* mrow = a.mask ? a.mask + ((long long)bh * a.Q + (qv ? qrow : 0)) * a.L : nullptr;
  KVTile nxt;
  if (kb < ke) kv_load(nxt, a.k, a.v, kb, ke, a.BH, bh, tid);
  for (int k0 = kb; k0 < ke; k0 += 64) {
    __syncthreads();
    kv_store(sk, sv, nxt, tid);
    __syncthreads();
    if (k0 + 64 < ke) kv_load(nxt, a.k, a.v, k0 + 64, ke, a.BH, bh, tid);
    const int kn = min(64, ke - k0);
    for (int r0 = 0; r0 < kn; r0 += 16) {
      f4m S = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 8; ++c) S = __builtin_amdgcn_mfma_f32_16x16x4f32(sk[r0 + lc][4 * c + lg], qb[c], S, 0, 0, 0);
      // this lane's 4 keys: k0 + r0 + lg*4 + i, query qrow
      const int kbase = k0 + r0 + lg * 4;
      uint32_t mb = 0;
      if (!a.mask) {
        // no mask (the decoder's self-attention): only keys past the range are excluded
      } else if (a.vec_mask && kbase + 4 <= ke) {
        mb = *reinterpret_cast<const uint32_t*>(mrow + kbase);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) mb |= (kbase + i < ke ? (uint32_t)mrow[kbase + i] : 1u) << (8 * i);
      }
      float sc[4];
      float bmax = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool masked = !qv || kbase + i >= ke || ((mb >> (8 * i)) & 0xffu);
        sc[i] = masked ? -INFINITY : S[i];
        bmax = fmaxf(bmax, sc[i]);
      }
      bmax = fmaxf(bmax, __shfl_xor(bmax, 16));
      bmax = fmaxf(bmax, __shfl_xor(bmax, 32));
      const float mn = fmaxf(m, bmax);
      float p[4], bsum = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        p[i] = sc[i] == -INFINITY ? 0.f : expf(sc[i] - mn);
        bsum += p[i];
      }
      bsum += __shfl_xor(bsum, 16);
      bsum += __shfl_xor(bsum, 32);
      if (mn != -INFINITY) {
        const float alpha = expf(m - mn);  // m == -inf -> 0 (o, lsum are 0 then)
        lsum = lsum * alpha + bsum;
        o[0] *= alpha;
        o[1] *= alpha;
        m = mn;
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          o[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(sv[r0 + lg * 4 + i][h * 16 + lc], p[i], o[h], 0, 0, 0);
    }
  }
  if (!qv) return;
  // accumulators: row = d = h*16 + lg*4 + j, col = query lc
  const long long row = ((long long)split * a.Q + qrow) * a.BH + bh;
  float* po = a.part_o + row * HD;
#pragma unroll
  for (int h = 0; h < 2; ++h)
    *reinterpret_cast<float4*>(po + h * 16 + lg * 4) = make_float4(o[h][0], o[h][1], o[h][2], o[h][3]);
  if (lg == 0) *reinterpret_cast<float2*>(a.part_ml + row * 2) = make_float2(m, lsum);
}

// One 32-lane group per (q, bh) row: merge the splits' partials; o = sum_s e_s o_s / sum_s e_s l_s.
template <typename T>
__global__ __launch_bounds__(256) void k_attn_merge(AttnArgs<T> a) {
  const long long rows = (long long)a.Q * a.BH;
  const long long r = blockIdx.x * 8ll + (threadIdx.x >> 5);
  const int d = threadIdx.x & 31;
  if (r >= rows) return;
  float M = -INFINITY;
  for (int s = 0; s < a.nsplit; ++s) M = fmaxf(M, a.part_ml[(s * rows + r) * 2]);
  float Ls = 0.f, acc = 0.f;
  if (M != -INFINITY) {
    for (int s = 0; s < a.nsplit; ++s) {
      const float ms = a.part_ml[(s * rows + r) * 2];
      if (ms == -INFINITY) continue;
      const float e = expf(ms - M);
      Ls = __builtin_fmaf(e, a.part_ml[(s * rows + r) * 2 + 1], Ls);
      acc = __builtin_fmaf(e, a.part_o[(s * rows + r) * HD + d], acc);
    }
  }
  // a fully masked row: 0 / 0 = NaN, as torch's softmax gives
  st1(a.o + r * HD + d, M == -INFINITY ? __builtin_nanf("") : acc / Ls);
  if (d == 0) a.lse[r] = M == -INFINITY ? INFINITY : M + logf(Ls);
}

template <typename T>
struct AttnBwdArgs {
  const T* q;
  const T* k;
  const T* v;
  const uint8_t* mask;
  const float* lse;     // [Q][BH]
  const float* delta;   // [Q][BH] = rowsum(dO * O)
  const T* dout;        // [Q][BH][HD]
  const float* qs;      // [Q][BH][HD] = q * scale (k_attn_delta)
  T* dq;                // [Q][BH][HD]
  T* dk;                // [L][BH][HD]
  T* dv;                // [L][BH][HD]
  float* part_dq;       // [nsplit][Q][BH][HD]
  int BH, Q, L;
  int nsplit, span;
  float scale;
  bool vec_mask;
};

// One 32-lane group per (q, bh) row: delta = sum_d dO * O, and q_scaled = q * scale (fp32, as
// torch forms it) for the dK / dV kernel's LDS staging.
template <typename T>
__global__ __launch_bounds__(256) void k_attn_delta(AttnBwdArgs<T> a, const T* __restrict__ o, float* delta,
                                                    float* qs) {
  const long long rows = (long long)a.Q * a.BH;
  const long long r = blockIdx.x * 8ll + (threadIdx.x >> 5);
  const int d = threadIdx.x & 31;
  float v = 0.f;
  if (r < rows) {
    v = ld1(o + r * HD + d) * ld1(a.dout + r * HD + d);
    qs[r * HD + d] = ld1(a.q + r * HD + d) * a.scale;
  }
  for (int s = 16; s > 0; s >>= 1) v += __shfl_xor(v, s, 32);
  if (r < rows && d == 0) delta[r] = v;
}

// dK / dV on fp32 MFMA (v_mfma_f32_16x16x4_f32, exact f32): a wave owns 16 keys, a workgroup 64;
// per block of 16 queries
//   S = q_scaled . K^T, dP = dO . V^T                 (16q x 16k, 8 + 8 MFMAs over the 32 dims)
//   P = exp(S - lse), dS = P (dP - delta)              (in the accumulator layout: lane l holds
//                                                       query (l>>4)*4+i, key l&15)
//   dV^T += dO^T . P, dK^T += q_scaled^T . dS          (32d x 16k, 8 + 8 MFMAs; P / dS feed the B
//                                                       operand straight from the accumulators:
//                                                       chunk i contracts queries (l>>4)*4+i)
// The K / V tiles stay in registers for the whole loop; q_scaled and dO are staged 64 queries at
// a time in LDS (rows padded to 33 floats).
typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int QB = 64;

template <typename T>
__global__ __launch_bounds__(256) void k_attn_bwd_kv_mfma(AttnBwdArgs<T> a) {
  __shared__ float sq[QB][HD + 1];
  __shared__ float sdo[QB][HD + 1];
  __shared__ float slse[QB], sdel[QB];
  const int bh = blockIdx.y, tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int lc = l & 15, lg = l >> 4;
  const int key0 = blockIdx.x * 64 + w * 16, keyl = key0 + lc;
  const bool kv = keyl < a.L;
  float kb[8], vb[8];  // B operands: K^T / V^T [d = 4c + lg][key lc]
#pragma unroll
  for (int c = 0; c < 8; ++c) {  // loads together (clamped key), zeroed after
    kb[c] = ld1(a.k + ((long long)(kv ? keyl : 0) * a.BH + bh) * HD + 4 * c + lg);
    vb[c] = ld1(a.v + ((long long)(kv ? keyl : 0) * a.BH + bh) * HD + 4 * c + lg);
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    kb[c] = kv ? kb[c] : 0.f;
    vb[c] = kv ? vb[c] : 0.f;
  }
  f4v dv[2] = {f4v{0.f, 0.f, 0.f, 0.f}, f4v{0.f, 0.f, 0.f, 0.f}};
  f4v dk[2] = {f4v{0.f, 0.f, 0.f, 0.f}, f4v{0.f, 0.f, 0.f, 0.f}};
  const uint8_t* mcol = a.mask ? a.mask + (long long)bh * a.Q * a.L + (kv ? keyl : 0) : nullptr;
  for (int qb0 = 0; qb0 < a.Q; qb0 += QB) {
    __syncthreads();
    for (int i = tid; i < QB * HD; i += 256) {
      const int r = i / HD, d = i % HD, qrow = qb0 + r;
      const bool ok = qrow < a.Q;
      const long long o = ((long long)(ok ? qrow : 0) * a.BH + bh) * HD + d;
      const float qv2 = a.qs[o], dv2 = ld1(a.dout + o);
      sq[r][d] = ok ? qv2 : 0.f;
      sdo[r][d] = ok ? dv2 : 0.f;
    }
    if (tid < QB) {
      const int qrow = qb0 + tid;
      const long long o = (long long)(qrow < a.Q ? qrow : 0) * a.BH + bh;
      const float lv = a.lse[o], dl = a.delta[o];
      slse[tid] = qrow < a.Q ? lv : 0.f;
      sdel[tid] = qrow < a.Q ? dl : 0.f;
    }
    __syncthreads();
    const int qn = min(QB, a.Q - qb0);
    for (int r0 = 0; r0 < qn; r0 += 16) {
      f4v S = {0.f, 0.f, 0.f, 0.f}, DP = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        S = __builtin_amdgcn_mfma_f32_16x16x4f32(sq[r0 + lc][4 * c + lg], kb[c], S, 0, 0, 0);
        DP = __builtin_amdgcn_mfma_f32_16x16x4f32(sdo[r0 + lc][4 * c + lg], vb[c], DP, 0, 0, 0);
      }
      float p[4], ds[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rr = r0 + lg * 4 + i, qq = qb0 + rr;
        const bool masked = !kv || qq >= a.Q || (mcol && mcol[(long long)(qq < a.Q ? qq : 0) * a.L]);
        p[i] = masked ? 0.f : expf(S[i] - slse[rr]);
        ds[i] = p[i] * (DP[i] - sdel[rr]);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = r0 + lg * 4 + i;
          dv[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(sdo[rr][h * 16 + lc], p[i], dv[h], 0, 0, 0);
          dk[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(sq[rr][h * 16 + lc], ds[i], dk[h], 0, 0, 0);
        }
    }
  }
  if (!kv) return;
  // accumulators: row = d = h*16 + lg*4 + j, col = key lc
  T* dkr = a.dk + ((long long)keyl * a.BH + bh) * HD;
  T* dvr = a.dv + ((long long)keyl * a.BH + bh) * HD;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    st4(dkr + h * 16 + lg * 4, dk[h][0], dk[h][1], dk[h][2], dk[h][3]);
    st4(dvr + h * 16 + lg * 4, dv[h][0], dv[h][1], dv[h][2], dv[h][3]);
  }
}

// dQ on fp32 MFMA, the forward's tiling: per 16-key block S^T = K . q_scaled^T and
// dP^T = V . dO^T (8 + 8 MFMAs), dS^T = exp(S^T - lse) (dP^T - delta) in the accumulator layout,
// then dq^T += K^T . dS^T (8 MFMAs, dS^T as the B operand); partial per key split.
template <typename T>
__global__ __launch_bounds__(256) void k_attn_bwd_q_mfma(AttnBwdArgs<T> a) {
  __shared__ float sk[64][HD + 1];
  __shared__ float sv[64][HD + 1];
  const int split = blockIdx.x, bh = blockIdx.y, tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int lc = l & 15, lg = l >> 4;
  const int qrow = blockIdx.z * 64 + w * 16 + lc;
  const bool qv = qrow < a.Q;
  float qb[8], db[8];  // B operands: q_scaled^T, dO^T [d = 4c + lg][query lc]
#pragma unroll
  for (int c = 0; c < 8; ++c) {  // loads together (clamped query), zeroed after
    qb[c] = ld1(a.q + ((long long)(qv ? qrow : 0) * a.BH + bh) * HD + 4 * c + lg);
    db[c] = ld1(a.dout + ((long long)(qv ? qrow : 0) * a.BH + bh) * HD + 4 * c + lg);
  }
  const float lse0 = a.lse[(long long)(qv ? qrow : 0) * a.BH + bh];
  const float del0 = a.delta[(long long)(qv ? qrow : 0) * a.BH + bh];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    qb[c] = qv ? qb[c] * a.scale : 0.f;
    db[c] = qv ? db[c] : 0.f;
  }
  const float lse = qv ? lse0 : 0.f;
  const float del = qv ? del0 : 0.f;
  f4m g[2] = {f4m{0.f, 0.f, 0.f, 0.f}, f4m{0.f, 0.f, 0.f, 0.f}};
  const int kb = split * a.span, ke = min(a.L, kb + a.span);
  const uint8_t* mrow = a.mask ? a.mask + ((long long)bh * a.Q + (qv ? qrow : 0)) * a.L : nullptr;
  KVTile nxt;
  if (kb < ke) kv_load(nxt, a.k, a.v, kb, ke, a.BH, bh, tid);
  for (int k0 = kb; k0 < ke; k0 += 64) {
    __syncthreads();
    kv_store(sk, sv, nxt, tid);
    __syncthreads();
    if (k0 + 64 < ke) kv_load(nxt, a.k, a.v, k0 + 64, ke, a.BH, bh, tid);
    const int kn = min(64, ke - k0);
    for (int r0 = 0; r0 < kn; r0 += 16) {
      f4m S = {0.f, 0.f, 0.f, 0.f}, DP = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        S = __builtin_amdgcn_mfma_f32_16x16x4f32(sk[r0 + lc][4 * c + lg], qb[c], S, 0, 0, 0);
        DP = __builtin_amdgcn_mfma_f32_16x16x4f32(sv[r0 + lc][4 * c + lg], db[c], DP, 0, 0, 0);
      }
      const int kbase = k0 + r0 + lg * 4;
      uint32_t mb = 0;
      if (!a.mask) {
        // no mask (the decoder's self-attention): only keys past the range are excluded
      } else if (a.vec_mask && kbase + 4 <= ke) {
        mb = *reinterpret_cast<const uint32_t*>(mrow + kbase);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) mb |= (kbase + i < ke ? (uint32_t)mrow[kbase + i] : 1u) << (8 * i);
      }
      float ds[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool masked = !qv || kbase + i >= ke || ((mb >> (8 * i)) & 0xffu);
        ds[i] = masked ? 0.f : expf(S[i] - lse) * (DP[i] - del);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          g[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(sk[r0 + lg * 4 + i][h * 16 + lc], ds[i], g[h], 0, 0, 0);
    }
  }
  if (!qv) return;
  float* pg = a.part_dq + (((long long)split * a.Q + qrow) * a.BH + bh) * HD;
#pragma unroll
  for (int h = 0; h < 2; ++h)
    *reinterpret_cast<float4*>(pg + h * 16 + lg * 4) = make_float4(g[h][0], g[h][1], g[h][2], g[h][3]);
}

// dq = scale * sum over splits (split order, deterministic)
template <typename T>
__global__ __launch_bounds__(256) void k_attn_dq_sum(AttnBwdArgs<T> a) {
  const long long n = (long long)a.Q * a.BH * HD;
  const long long i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  float acc = 0.f;
  for (int s = 0; s < a.nsplit; ++s) acc += a.part_dq[s * n + i];
  st1(a.dq + i, acc * a.scale);
}

// Key splits: ~1024 x (Q / 128) workgroups (swept 512..4096 at B=8, L=4800: fewer splits make the
// merge cheaper, more leave the MFMA kernels no faster), >= KS keys each.
void split_keys(int BH, int Q, int L, int* nsplit, int* span) {
  const long long base = (long long)BH * ((Q + 127) / 128);
  const int max_split = (L + KS - 1) / KS;
  const long long target = 1024;
  int ns = (int)std::min<long long>(max_split, std::max<long long>(1, (target + base - 1) / base));
  int sp = (L + ns - 1) / ns;
  sp = (sp + KS - 1) / KS * KS;
  *span = sp;
  *nsplit = (L + sp - 1) / sp;
}

bool attn_shape_ok(const void* q, const void* k, const void* v, int BH, int Q, int L, int head_dim) {
  return head_dim == HD && BH > 0 && Q > 0 && L > 0 && ((uintptr_t)q % 16) == 0 && ((uintptr_t)k % 16) == 0 &&
         ((uintptr_t)v % 16) == 0;
}

template <typename T>
int attn_fwd(const void* q, const void* k, const void* v, const uint8_t* mask, int BH, int Q, int L, float scale,
             void* out, float* lse, void* ws, hipStream_t s);
template <typename T>
int attn_bwd(const void* q, const void* k, const void* v, const uint8_t* mask, const void* out, const float* lse,
             const void* dout, int BH, int Q, int L, float scale, void* dq, void* dk, void* dv, void* ws,
             hipStream_t s);

size_t attn_align(size_t x) { return (x + 255) / 256 * 256; }

bool mask_vec(const uint8_t* mask, int L) { return mask && (L % 16) == 0 && ((uintptr_t)mask % 16) == 0; }

template <typename T>
int attn_fwd(const void* q, const void* k, const void* v, const uint8_t* mask, int BH, int Q, int L, float scale,
             void* out, float* lse, void* ws, hipStream_t s) {
  AttnArgs<T> a = {(const T*)q, (const T*)k, (const T*)v, mask, (T*)out, lse, nullptr, nullptr, BH, Q, L, 0, 0,
                   scale, mask_vec(mask, L)};
  split_keys(BH, Q, L, &a.nsplit, &a.span);
  const size_t rows = (size_t)a.nsplit * Q * BH;
  a.part_o = (float*)ws;
  a.part_ml = (float*)((char*)ws + attn_align(rows * HD * sizeof(float)));
  k_attn_fwd_mfma<T><<<dim3(a.nsplit, BH, (Q + QW - 1) / QW), 256, 0, s>>>(a);
  const long long orows = (long long)Q * BH;
  k_attn_merge<T><<<(unsigned)((orows + 7) / 8), 256, 0, s>>>(a);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

template <typename T>
int attn_bwd(const void* q, const void* k, const void* v, const uint8_t* mask, const void* out, const float* lse,
             const void* dout, int BH, int Q, int L, float scale, void* dq, void* dk, void* dv, void* ws,
             hipStream_t s) {
  const long long rows = (long long)BH * Q;
  float* delta = (float*)ws;
  float* qs = (float*)((char*)ws + attn_align((size_t)rows * sizeof(float)));
  AttnBwdArgs<T> a = {(const T*)q, (const T*)k, (const T*)v, mask, lse, delta, (const T*)dout, qs, (T*)dq, (T*)dk,
                      (T*)dv, nullptr, BH, Q, L, 0, 0, scale, mask_vec(mask, L)};
  split_keys(BH, Q, L, &a.nsplit, &a.span);
  a.part_dq = (float*)((char*)qs + attn_align((size_t)rows * HD * sizeof(float)));
  k_attn_delta<T><<<(unsigned)((rows + 7) / 8), 256, 0, s>>>(a, (const T*)out, delta, qs);
  k_attn_bwd_kv_mfma<T><<<dim3((L + 63) / 64, BH), 256, 0, s>>>(a);
  k_attn_bwd_q_mfma<T><<<dim3(a.nsplit, BH, (Q + QW - 1) / QW), 256, 0, s>>>(a);
  k_attn_dq_sum<T><<<(unsigned)((rows * HD + 255) / 256), 256, 0, s>>>(a);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // namespace

extern "C" {

size_t rgbd_masked_attn_fwd_workspace_size(int BH, int Q, int L) {
  if (BH <= 0 || Q <= 0 || L <= 0) return 256;
  int ns, sp;
  split_keys(BH, Q, L, &ns, &sp);
  const size_t rows = (size_t)ns * Q * BH;
  return attn_align(rows * HD * sizeof(float)) + attn_align(rows * 2 * sizeof(float));
}

int rgbd_masked_attn_fwd(int dtype, const void* q, const void* k, const void* v, const uint8_t* mask, int BH, int Q,
                         int L, int head_dim, float scale, void* out, float* lse, void* ws, void* stream) {
  RGBD_REQUIRE(q && k && v && out && lse && ws && BH > 0 && Q > 0 && L > 0, RGBD_E_ARG);
  RGBD_REQUIRE(attn_shape_ok(q, k, v, BH, Q, L, head_dim) && ((uintptr_t)out % 16) == 0, RGBD_E_SHAPE);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_F32) return attn_fwd<float>(q, k, v, mask, BH, Q, L, scale, out, lse, ws, s);
  if (dtype == RGBD_BF16) return attn_fwd<bf16_t>(q, k, v, mask, BH, Q, L, scale, out, lse, ws, s);
  return RGBD_E_DTYPE;
}

size_t rgbd_masked_attn_bwd_workspace_size(int BH, int Q, int L) {
  if (BH <= 0 || Q <= 0 || L <= 0) return 256;
  int ns, sp;
  split_keys(BH, Q, L, &ns, &sp);
  return attn_align((size_t)Q * BH * sizeof(float)) + attn_align((size_t)Q * BH * HD * sizeof(float)) +
         attn_align((size_t)ns * Q * BH * HD * sizeof(float));
}

int rgbd_masked_attn_bwd(int dtype, const void* q, const void* k, const void* v, const uint8_t* mask, const void* out,
                         const float* lse, const void* dout, int BH, int Q, int L, int head_dim, float scale,
                         void* dq, void* dk, void* dv, void* ws, void* stream) {
  RGBD_REQUIRE(q && k && v && out && lse && dout && dq && dk && dv && ws && BH > 0 && Q > 0 && L > 0,
               RGBD_E_ARG);
  RGBD_REQUIRE(attn_shape_ok(q, k, v, BH, Q, L, head_dim) && ((uintptr_t)dout % 16) == 0 && ((uintptr_t)out % 16) == 0 &&
                   ((uintptr_t)dk % 16) == 0 && ((uintptr_t)dv % 16) == 0,
               RGBD_E_SHAPE);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_F32) return attn_bwd<float>(q, k, v, mask, out, lse, dout, BH, Q, L, scale, dq, dk, dv, ws, s);
  if (dtype == RGBD_BF16) return attn_bwd<bf16_t>(q, k, v, mask, out, lse, dout, BH, Q, L, scale, dq, dk, dv, ws, s);
  return RGBD_E_DTYPE;
}

}  // extern "C"
