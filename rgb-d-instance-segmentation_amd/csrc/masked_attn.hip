// f1: the masked cross-attention core of the Mask2Former decoder layers (gfx950, float32).
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
// in split order (no atomics anywhere: the backward is deterministic).  Default kernels run on fp32
// MFMA (v_mfma_f32_16x16x4_f32, exact f32 products and sums):
//   k_attn_fwd_mfma     wave = 16 queries; S^T = K q_scaled^T, online softmax per query column,
//                       O^T += V^T P^T with P^T taken straight from the accumulators; partial
//                       (max, sum, o) per split -> k_attn_merge (also writes the row log-sum-exp)
//   k_attn_bwd_kv_mfma  wave = 16 keys over all queries; S, dP, then dV^T += dO^T P, dK^T +=
//                       q_scaled^T dS, K / V tiles held in registers
//   k_attn_bwd_q_mfma   the forward's tiling: dq^T += K^T dS^T, partial per split -> k_attn_dq_sum
// The earlier packed-fp32 VALU kernels (thread per query / per key, K / V rows as scalar loads)
// stay selectable with RGBD_ATTN_FWD=valu / RGBD_ATTN_KV=valu (A/B and diagnosis).
#include <cmath>
#include <cstdlib>

#include "common.hpp"

using namespace rgbd;

namespace {

constexpr int HD = 32;      // head dim (hidden 256 / 8 heads)
constexpr int QW = 128;     // queries per forward / dQ workgroup (one per thread)
constexpr int KS = 64;      // key-split granularity
constexpr int KC = 16;      // keys per online-softmax chunk
constexpr int KVW = 256;    // keys per dK / dV workgroup (one per thread)

struct AttnArgs {
  const float* q;        // [Q][BH][HD] (unscaled)
  const float* k;        // [L][BH][HD]
  const float* v;        // [L][BH][HD]
  const uint8_t* mask;   // [BH][Q][L] bool, true = not allowed
  float* o;              // [Q][BH][HD]
  float* lse;            // [Q][BH] log-sum-exp of the scaled, masked scores
  float* part_o;         // [nsplit][Q][BH][HD]
  float* part_ml;        // [nsplit][Q][BH][2] = (max, sum)
  int BH, Q, L;
  int nsplit, span;      // key range of split s: [s*span, min(L, (s+1)*span)), span % KS == 0
  float scale;
  bool vec_mask;         // mask rows 16-byte aligned (L % 16 == 0)
};

// Rows of K / V (forward, dQ) and of q_scaled / dO (dK / dV) are the same for every lane of a
// wave: they are read through the constant address space, so they arrive as scalar loads into
// SGPRs and feed the FMAs as scalar operands — no LDS staging, no broadcast traffic.
typedef const float __attribute__((address_space(4))) cfloat;

__device__ __forceinline__ const cfloat* uniform_row(const float* base, long long row, int BH, int bh) {
  return (const cfloat*)(base + (row * BH + bh) * HD);
}

// Packed fp32 (v_pk_fma_f32): a 32-wide row is 16 float pairs; dot products keep two partial
// sums (even / odd dims) added at the end.
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int HP = HD / 2;

__device__ __forceinline__ f2 pair(const cfloat* row, int c) { return f2{row[2 * c], row[2 * c + 1]}; }

__device__ __forceinline__ float dot_row(const f2 (&x)[HP], const cfloat* row) {
  f2 acc = {0.f, 0.f};
#pragma unroll
  for (int c = 0; c < HP; ++c) acc = __builtin_elementwise_fma(x[c], pair(row, c), acc);
  return acc.x + acc.y;
}

__device__ __forceinline__ void axpy_row(f2 (&acc)[HP], float a, const cfloat* row) {
  const f2 a2 = {a, a};
#pragma unroll
  for (int c = 0; c < HP; ++c) acc[c] = __builtin_elementwise_fma(a2, pair(row, c), acc[c]);
}

__device__ __forceinline__ void load_row(f2 (&x)[HP], const float* row, bool ok, float mul) {
#pragma unroll
  for (int c = 0; c < HP; ++c) {
    const float2 t = ok ? *reinterpret_cast<const float2*>(row + 2 * c) : make_float2(0.f, 0.f);
    x[c] = f2{t.x * mul, t.y * mul};
  }
}

__device__ __forceinline__ void store_row(float* row, const f2 (&x)[HP]) {
#pragma unroll
  for (int c = 0; c < HD / 4; ++c)
    *reinterpret_cast<float4*>(row + 4 * c) = make_float4(x[2 * c].x, x[2 * c].y, x[2 * c + 1].x, x[2 * c + 1].y);
}

// bit j = key c0 + j masked (or past ke), from the lane's own mask row: one 16-byte load when
// the row is 16-byte aligned (vec), else byte loads.
__device__ __forceinline__ uint32_t mask_bits16(const uint8_t* mrow, int c0, int ke, bool vec) {
  uint32_t bits = 0;
  if (vec && c0 + KC <= ke) {
    const uint4 w = *reinterpret_cast<const uint4*>(mrow + c0);
    const uint32_t x[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int b = 0; b < 4; ++b) bits |= ((x[i] >> (8 * b)) & 1u) << (4 * i + b);
  } else {
    for (int j = 0; j < KC; ++j)
      if (c0 + j >= ke || mrow[c0 + j]) bits |= 1u << j;
  }
  return bits;
}

// grid (nsplit, BH, ceil(Q / QW)), QW threads
__global__ __launch_bounds__(QW) void k_attn_fwd(AttnArgs a) {
  const int split = blockIdx.x, bh = blockIdx.y, tid = threadIdx.x;
  const int qrow = blockIdx.z * QW + tid;
  const bool qv = qrow < a.Q;
  f2 qr[HP], o[HP];
  load_row(qr, a.q + ((long long)qrow * a.BH + bh) * HD, qv, a.scale);  // q * scale, as torch forms it
#pragma unroll
  for (int c = 0; c < HP; ++c) o[c] = f2{0.f, 0.f};
  const int kb = split * a.span, ke = min(a.L, kb + a.span);
  const uint8_t* mrow = a.mask + ((long long)bh * a.Q + (qv ? qrow : 0)) * a.L;
  float m = -INFINITY, l = 0.f;
  uint32_t next_bits = kb < ke ? mask_bits16(mrow, kb, ke, a.vec_mask) : 0u;
  for (int c0 = kb; c0 < ke; c0 += KC) {
    const uint32_t bits = next_bits;  // mask bits one chunk ahead, so the load latency overlaps a chunk
    if (c0 + KC < ke) next_bits = mask_bits16(mrow, c0 + KC, ke, a.vec_mask);
    float s[KC];
    float cmax = -INFINITY;
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      s[j] = -INFINITY;
      if (c0 + j < ke) {
        const float acc = dot_row(qr, uniform_row(a.k, c0 + j, a.BH, bh));
        if (!((bits >> j) & 1u)) s[j] = acc;
      }
      cmax = fmaxf(cmax, s[j]);
    }
    if (cmax != -INFINITY) {  // else the whole chunk is masked for this query
      const float mn = fmaxf(m, cmax);
      const float alpha = expf(m - mn);  // m == -inf -> 0 (l, o are 0 then)
      l *= alpha;
#pragma unroll
      for (int c = 0; c < HP; ++c) o[c] *= alpha;
      m = mn;
    }
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      if (c0 + j >= ke) break;
      const float p = s[j] == -INFINITY ? 0.f : expf(s[j] - m);  // masked: exactly 0, as torch's softmax
      l += p;
      axpy_row(o, p, uniform_row(a.v, c0 + j, a.BH, bh));
    }
  }
  if (!qv) return;
  const long long row = ((long long)split * a.Q + qrow) * a.BH + bh;
  store_row(a.part_o + row * HD, o);
  *reinterpret_cast<float2*>(a.part_ml + row * 2) = make_float2(m, l);
}

// K / V tile staging for the MFMA forward and dQ: 64 keys x 32 dims of each, two float4 per
// thread per matrix, loaded one tile ahead into registers so the global loads overlap the
// current tile's MFMAs.
struct KVTile {
  float4 k[2], v[2];
};

__device__ __forceinline__ void kv_load(KVTile& t, const float* K, const float* V, int k0, int ke, int BH, int bh,
                                        int tid) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = tid + 256 * j, row = idx >> 3, c = idx & 7, key = k0 + row;
    const bool ok = key < ke;
    const long long off = ((long long)key * BH + bh) * HD + 4 * c;
    t.k[j] = ok ? *reinterpret_cast<const float4*>(K + off) : make_float4(0.f, 0.f, 0.f, 0.f);
    t.v[j] = ok ? *reinterpret_cast<const float4*>(V + off) : make_float4(0.f, 0.f, 0.f, 0.f);
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

__global__ __launch_bounds__(256) void k_attn_fwd_mfma(AttnArgs a) {
  __shared__ float sk[64][HD + 1];
  __shared__ float sv[64][HD + 1];
  const int split = blockIdx.x, bh = blockIdx.y, tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int lc = l & 15, lg = l >> 4;
  const int qrow = blockIdx.z * 64 + w * 16 + lc;
  const bool qv = qrow < a.Q;
  float qb[8];  // B operand: q_scaled^T [d = 4c + lg][query lc]
#pragma unroll
  for (int c = 0; c < 8; ++c) qb[c] = qv ? a.q[((long long)qrow * a.BH + bh) * HD + 4 * c + lg] * a.scale : 0.f;
  f4m o[2] = {f4m{0.f, 0.f, 0.f, 0.f}, f4m{0.f, 0.f, 0.f, 0.f}};
  float m = -INFINITY, lsum = 0.f;
  const int kb = split * a.span, ke = min(a.L, kb + a.span);
  const uint8_t* mrow = a.mask + ((long long)bh * a.Q + (qv ? qrow : 0)) * a.L;
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
      if (a.vec_mask && kbase + 4 <= ke) {
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
__global__ __launch_bounds__(256) void k_attn_merge(AttnArgs a) {
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
  a.o[r * HD + d] = M == -INFINITY ? __builtin_nanf("") : acc / Ls;
  if (d == 0) a.lse[r] = M == -INFINITY ? INFINITY : M + logf(Ls);
}

struct AttnBwdArgs {
  const float* q;
  const float* k;
  const float* v;
  const uint8_t* mask;
  const float* lse;     // [Q][BH]
  const float* delta;   // [Q][BH] = rowsum(dO * O)
  const float* dout;    // [Q][BH][HD]
  const float* qs;      // [Q][BH][HD] = q * scale (k_attn_delta)
  float* dq;            // [Q][BH][HD]
  float* dk;            // [L][BH][HD]
  float* dv;            // [L][BH][HD]
  float* part_dq;       // [nsplit][Q][BH][HD]
  int BH, Q, L;
  int nsplit, span;
  float scale;
  bool vec_mask;
};

// One 32-lane group per (q, bh) row: delta = sum_d dO * O, and q_scaled = q * scale (fp32, as
// torch forms it) for the dK / dV kernel's scalar reads.
__global__ __launch_bounds__(256) void k_attn_delta(AttnBwdArgs a, const float* __restrict__ o, float* delta,
                                                    float* qs) {
  const long long rows = (long long)a.Q * a.BH;
  const long long r = blockIdx.x * 8ll + (threadIdx.x >> 5);
  const int d = threadIdx.x & 31;
  float v = 0.f;
  if (r < rows) {
    v = o[r * HD + d] * a.dout[r * HD + d];
    qs[r * HD + d] = a.q[r * HD + d] * a.scale;
  }
  for (int s = 16; s > 0; s >>= 1) v += __shfl_xor(v, s, 32);
  if (r < rows && d == 0) delta[r] = v;
}

// grid (ceil(L / KVW), BH), KVW threads: thread = key; q_scaled / dO rows of each query are
// wave-uniform scalar reads.
__global__ __launch_bounds__(KVW) void k_attn_bwd_kv(AttnBwdArgs a) {
  const int bh = blockIdx.y, tid = threadIdx.x;
  const int key = blockIdx.x * KVW + tid;
  const bool kv = key < a.L;
  f2 kr[HP], vr[HP], dk[HP], dv[HP];
  load_row(kr, a.k + ((long long)key * a.BH + bh) * HD, kv, 1.f);
  load_row(vr, a.v + ((long long)key * a.BH + bh) * HD, kv, 1.f);
#pragma unroll
  for (int c = 0; c < HP; ++c) dk[c] = dv[c] = f2{0.f, 0.f};
  const cfloat* lse = (const cfloat*)a.lse;
  const cfloat* del = (const cfloat*)a.delta;
  const uint8_t* mcol = a.mask + (long long)bh * a.Q * a.L + (kv ? key : 0);
  for (int q0 = 0; q0 < a.Q; q0 += 16) {
    // the next 16 queries' mask bytes for this key, all loads in flight at once
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (q0 + j < a.Q && (!kv || mcol[(long long)(q0 + j) * a.L])) bits |= 1u << j;
    const int qn = min(16, a.Q - q0);
#pragma unroll 2
    for (int j = 0; j < qn; ++j) {
      const int qi = q0 + j;
      const cfloat* qr = uniform_row(a.qs, qi, a.BH, bh);
      const cfloat* dor = uniform_row(a.dout, qi, a.BH, bh);
      const float s = dot_row(kr, qr);
      const float dp = dot_row(vr, dor);
      const float p = ((bits >> j) & 1u) ? 0.f : expf(s - lse[(long long)qi * a.BH + bh]);
      const float ds = p * (dp - del[(long long)qi * a.BH + bh]);
      axpy_row(dv, p, dor);
      axpy_row(dk, ds, qr);  // dK = dS^T (q * scale)
    }
  }
  if (!kv) return;
  store_row(a.dk + ((long long)key * a.BH + bh) * HD, dk);
  store_row(a.dv + ((long long)key * a.BH + bh) * HD, dv);
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

__global__ __launch_bounds__(256) void k_attn_bwd_kv_mfma(AttnBwdArgs a) {
  __shared__ float sq[QB][HD + 1];
  __shared__ float sdo[QB][HD + 1];
  __shared__ float slse[QB], sdel[QB];
  const int bh = blockIdx.y, tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int lc = l & 15, lg = l >> 4;
  const int key0 = blockIdx.x * 64 + w * 16, keyl = key0 + lc;
  const bool kv = keyl < a.L;
  float kb[8], vb[8];  // B operands: K^T / V^T [d = 4c + lg][key lc]
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    kb[c] = kv ? a.k[((long long)keyl * a.BH + bh) * HD + 4 * c + lg] : 0.f;
    vb[c] = kv ? a.v[((long long)keyl * a.BH + bh) * HD + 4 * c + lg] : 0.f;
  }
  f4v dv[2] = {f4v{0.f, 0.f, 0.f, 0.f}, f4v{0.f, 0.f, 0.f, 0.f}};
  f4v dk[2] = {f4v{0.f, 0.f, 0.f, 0.f}, f4v{0.f, 0.f, 0.f, 0.f}};
  const uint8_t* mcol = a.mask + (long long)bh * a.Q * a.L + (kv ? keyl : 0);
  for (int qb0 = 0; qb0 < a.Q; qb0 += QB) {
    __syncthreads();
    for (int i = tid; i < QB * HD; i += 256) {
      const int r = i / HD, d = i % HD, qrow = qb0 + r;
      const bool ok = qrow < a.Q;
      sq[r][d] = ok ? a.qs[((long long)qrow * a.BH + bh) * HD + d] : 0.f;
      sdo[r][d] = ok ? a.dout[((long long)qrow * a.BH + bh) * HD + d] : 0.f;
    }
    if (tid < QB) {
      const int qrow = qb0 + tid;
      slse[tid] = qrow < a.Q ? a.lse[(long long)qrow * a.BH + bh] : 0.f;
      sdel[tid] = qrow < a.Q ? a.delta[(long long)qrow * a.BH + bh] : 0.f;
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
        const bool masked = !kv || qq >= a.Q || mcol[(long long)(qq < a.Q ? qq : 0) * a.L];
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
  float* dkr = a.dk + ((long long)keyl * a.BH + bh) * HD;
  float* dvr = a.dv + ((long long)keyl * a.BH + bh) * HD;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    *reinterpret_cast<float4*>(dkr + h * 16 + lg * 4) = make_float4(dk[h][0], dk[h][1], dk[h][2], dk[h][3]);
    *reinterpret_cast<float4*>(dvr + h * 16 + lg * 4) = make_float4(dv[h][0], dv[h][1], dv[h][2], dv[h][3]);
  }
}

// grid (nsplit, BH, ceil(Q / QW)), QW threads: thread = query; partial sum_k ds k over the split.
__global__ __launch_bounds__(QW) void k_attn_bwd_q(AttnBwdArgs a) {
  const int split = blockIdx.x, bh = blockIdx.y, tid = threadIdx.x;
  const int qrow = blockIdx.z * QW + tid;
  const bool qv = qrow < a.Q;
  f2 qr[HP], dor[HP], g[HP];
  load_row(qr, a.q + ((long long)qrow * a.BH + bh) * HD, qv, a.scale);
  load_row(dor, a.dout + ((long long)qrow * a.BH + bh) * HD, qv, 1.f);
#pragma unroll
  for (int c = 0; c < HP; ++c) g[c] = f2{0.f, 0.f};
  const float lse = qv ? a.lse[(long long)qrow * a.BH + bh] : 0.f;
  const float del = qv ? a.delta[(long long)qrow * a.BH + bh] : 0.f;
  const int kb = split * a.span, ke = min(a.L, kb + a.span);
  const uint8_t* mrow = a.mask + ((long long)bh * a.Q + (qv ? qrow : 0)) * a.L;
  uint32_t next_bits = kb < ke ? mask_bits16(mrow, kb, ke, a.vec_mask) : 0u;
  for (int c0 = kb; c0 < ke; c0 += KC) {
    const uint32_t bits = next_bits;  // mask bits one chunk ahead, so the load latency overlaps a chunk
    if (c0 + KC < ke) next_bits = mask_bits16(mrow, c0 + KC, ke, a.vec_mask);
#pragma unroll 4
    for (int j = 0; j < KC; ++j) {
      if (c0 + j >= ke) break;
      const cfloat* kr = uniform_row(a.k, c0 + j, a.BH, bh);
      const float s = dot_row(qr, kr);
      const float dp = dot_row(dor, uniform_row(a.v, c0 + j, a.BH, bh));
      const float ds = ((bits >> j) & 1u) ? 0.f : expf(s - lse) * (dp - del);
      axpy_row(g, ds, kr);
    }
  }
  if (!qv) return;
  store_row(a.part_dq + (((long long)split * a.Q + qrow) * a.BH + bh) * HD, g);
}

// dQ on fp32 MFMA, the forward's tiling: per 16-key block S^T = K . q_scaled^T and
// dP^T = V . dO^T (8 + 8 MFMAs), dS^T = exp(S^T - lse) (dP^T - delta) in the accumulator layout,
// then dq^T += K^T . dS^T (8 MFMAs, dS^T as the B operand); partial per key split.
__global__ __launch_bounds__(256) void k_attn_bwd_q_mfma(AttnBwdArgs a) {
  __shared__ float sk[64][HD + 1];
  __shared__ float sv[64][HD + 1];
  const int split = blockIdx.x, bh = blockIdx.y, tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int lc = l & 15, lg = l >> 4;
  const int qrow = blockIdx.z * 64 + w * 16 + lc;
  const bool qv = qrow < a.Q;
  float qb[8], db[8];  // B operands: q_scaled^T, dO^T [d = 4c + lg][query lc]
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    qb[c] = qv ? a.q[((long long)qrow * a.BH + bh) * HD + 4 * c + lg] * a.scale : 0.f;
    db[c] = qv ? a.dout[((long long)qrow * a.BH + bh) * HD + 4 * c + lg] : 0.f;
  }
  const float lse = qv ? a.lse[(long long)qrow * a.BH + bh] : 0.f;
  const float del = qv ? a.delta[(long long)qrow * a.BH + bh] : 0.f;
  f4m g[2] = {f4m{0.f, 0.f, 0.f, 0.f}, f4m{0.f, 0.f, 0.f, 0.f}};
  const int kb = split * a.span, ke = min(a.L, kb + a.span);
  const uint8_t* mrow = a.mask + ((long long)bh * a.Q + (qv ? qrow : 0)) * a.L;
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
      if (a.vec_mask && kbase + 4 <= ke) {
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
__global__ __launch_bounds__(256) void k_attn_dq_sum(AttnBwdArgs a) {
  const long long n = (long long)a.Q * a.BH * HD;
  const long long i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  float acc = 0.f;
  for (int s = 0; s < a.nsplit; ++s) acc += a.part_dq[s * n + i];
  a.dq[i] = acc * a.scale;
}

// Key splits: ~1024 x (Q / 128) workgroups (swept 512..4096 at B=8, L=4800: fewer splits make the
// merge cheaper, more leave the MFMA kernels no faster), >= KS keys each.
void split_keys(int BH, int Q, int L, int* nsplit, int* span) {
  const long long base = (long long)BH * ((Q + QW - 1) / QW);
  const int max_split = (L + KS - 1) / KS;
  static const long long target = [] {  // workgroups to aim for (RGBD_ATTN_WG_TARGET, tuning)
    const char* e = getenv("RGBD_ATTN_WG_TARGET");
    return e ? std::max(1LL, atoll(e)) : 1024LL;
  }();
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

size_t attn_align(size_t x) { return (x + 255) / 256 * 256; }

bool mask_vec(const uint8_t* mask, int L) { return (L % 16) == 0 && ((uintptr_t)mask % 16) == 0; }

}  // namespace

extern "C" {

size_t rgbd_masked_attn_fwd_workspace_size(int BH, int Q, int L) {
  if (BH <= 0 || Q <= 0 || L <= 0) return 256;
  int ns, sp;
  split_keys(BH, Q, L, &ns, &sp);
  const size_t rows = (size_t)ns * Q * BH;
  return attn_align(rows * HD * sizeof(float)) + attn_align(rows * 2 * sizeof(float));
}

int rgbd_masked_attn_fwd(const float* q, const float* k, const float* v, const uint8_t* mask, int BH, int Q, int L,
                         int head_dim, float scale, float* out, float* lse, void* ws, void* stream) {
  RGBD_REQUIRE(q && k && v && mask && out && lse && ws && BH > 0 && Q > 0 && L > 0, RGBD_E_ARG);
  RGBD_REQUIRE(attn_shape_ok(q, k, v, BH, Q, L, head_dim) && ((uintptr_t)out % 16) == 0, RGBD_E_SHAPE);
  hipStream_t s = (hipStream_t)stream;
  AttnArgs a = {q, k, v, mask, out, lse, nullptr, nullptr, BH, Q, L, 0, 0, scale, mask_vec(mask, L)};
  split_keys(BH, Q, L, &a.nsplit, &a.span);
  const size_t rows = (size_t)a.nsplit * Q * BH;
  a.part_o = (float*)ws;
  a.part_ml = (float*)((char*)ws + attn_align(rows * HD * sizeof(float)));
  static const char* fwd_env = getenv("RGBD_ATTN_FWD");  // "valu": the thread-per-query kernel
  if (fwd_env && fwd_env[0] == 'v')
    k_attn_fwd<<<dim3(a.nsplit, BH, (Q + QW - 1) / QW), QW, 0, s>>>(a);
  else
    k_attn_fwd_mfma<<<dim3(a.nsplit, BH, (Q + 63) / 64), 256, 0, s>>>(a);
  const long long orows = (long long)Q * BH;
  k_attn_merge<<<(unsigned)((orows + 7) / 8), 256, 0, s>>>(a);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

size_t rgbd_masked_attn_bwd_workspace_size(int BH, int Q, int L) {
  if (BH <= 0 || Q <= 0 || L <= 0) return 256;
  int ns, sp;
  split_keys(BH, Q, L, &ns, &sp);
  return attn_align((size_t)Q * BH * sizeof(float)) + attn_align((size_t)Q * BH * HD * sizeof(float)) +
         attn_align((size_t)ns * Q * BH * HD * sizeof(float));
}

int rgbd_masked_attn_bwd(const float* q, const float* k, const float* v, const uint8_t* mask, const float* out,
                         const float* lse, const float* dout, int BH, int Q, int L, int head_dim, float scale,
                         float* dq, float* dk, float* dv, void* ws, void* stream) {
  RGBD_REQUIRE(q && k && v && mask && out && lse && dout && dq && dk && dv && ws && BH > 0 && Q > 0 && L > 0,
               RGBD_E_ARG);
  RGBD_REQUIRE(attn_shape_ok(q, k, v, BH, Q, L, head_dim) && ((uintptr_t)dout % 16) == 0 && ((uintptr_t)out % 16) == 0 &&
                   ((uintptr_t)dk % 16) == 0 && ((uintptr_t)dv % 16) == 0,
               RGBD_E_SHAPE);
  hipStream_t s = (hipStream_t)stream;
  const long long rows = (long long)BH * Q;
  float* delta = (float*)ws;
  float* qs = (float*)((char*)ws + attn_align((size_t)rows * sizeof(float)));
  AttnBwdArgs a = {q, k, v, mask, lse, delta, dout, qs, dq, dk, dv, nullptr, BH, Q, L, 0, 0, scale,
                   mask_vec(mask, L)};
  split_keys(BH, Q, L, &a.nsplit, &a.span);
  a.part_dq = (float*)((char*)qs + attn_align((size_t)rows * HD * sizeof(float)));
  k_attn_delta<<<(unsigned)((rows + 7) / 8), 256, 0, s>>>(a, out, delta, qs);
  static const char* kv_env = getenv("RGBD_ATTN_KV");  // "valu": the thread-per-key kernel
  if (kv_env && kv_env[0] == 'v')
    k_attn_bwd_kv<<<dim3((L + KVW - 1) / KVW, BH), KVW, 0, s>>>(a);
  else
    k_attn_bwd_kv_mfma<<<dim3((L + 63) / 64, BH), 256, 0, s>>>(a);
  if (kv_env && kv_env[0] == 'v')
    k_attn_bwd_q<<<dim3(a.nsplit, BH, (Q + QW - 1) / QW), QW, 0, s>>>(a);
  else
    k_attn_bwd_q_mfma<<<dim3(a.nsplit, BH, (Q + 63) / 64), 256, 0, s>>>(a);
  k_attn_dq_sum<<<(unsigned)((rows * HD + 255) / 256), 256, 0, s>>>(a);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
