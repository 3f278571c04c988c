// f1: the Mask2Former mask predictor's dense work on gfx950.
//
// Reference: Mask2FormerMaskPredictor.forward (transformers 5.15 modeling_mask2former.py:2040-2056),
// called 10x per forward by Mask2FormerMaskedAttentionDecoder (:1896, :1929):
//   outputs_mask   = einsum("bqc,bchw->bqhw", mask_embeddings, pixel_embeddings)      (:2046)
//   attention_mask = interpolate(outputs_mask, target, bilinear, align_corners=False)  (:2048)
//                      .sigmoid().flatten(2).unsqueeze(1).repeat(1, heads, 1, 1)
//                      .flatten(0, 1) < 0.5                                            (:2052-2053)
//
// k_mask_logits: out[b][q][p] = sum_c emb[b][q][c] * pix[b][c][p] as an MFMA GEMM with the
// pixels as the M operand.  Per workgroup: one image, 64 pixels x 128 queries, 4 waves, wave w
// owns query fragments 2w, 2w+1 (16 queries each) for all 4 pixel fragments.  The NCHW pixel
// embeddings arrive channel-major, so a 64-channel x 128-pixel chunk is staged in LDS with
// coalesced 16-byte loads and read back k-major: bf16 with ds_read_b64_tr_b16 (32-byte column
// blocks XOR-swizzled by row bits 0-1 and 3, conflict-free), f32 with ds_read_b32 (64-byte blocks
// swizzled by row bit 3).  The query embeddings (tiny, L2-resident) are the B operand straight
// from global memory (8 consecutive channels per lane).  The accumulator holds 4 consecutive
// pixels of one query per lane: one 16-byte (f32) / 8-byte (bf16) store each.
// Bound: HBM.  Per pixel the kernel reads C elements of the pixel embedding and writes Q logits:
// (256 + 100) x 4 B = 1424 B/px in f32, 712 B/px in bf16, for 51 200 FLOP/px (36-72 FLOP/B, far
// below the ~310 FLOP/B ridge).
//
// k_mask_attention: the bilinear resample (torch upsample_bilinear2d, align_corners=False, no
// antialias: source = max(scale*(dst+0.5)-0.5, 0), scale = in/out), the sigmoid and the < 0.5
// binarisation per (b, q, target pixel), written once per head as bytes (torch.bool).
#include "common.hpp"
#include "mfma.hpp"

#include <algorithm>

namespace rgbd {
namespace {

constexpr int ML_TP = 128;  // pixels per workgroup (max; the launch picks TP = 64 or 128)
constexpr int ML_TQ = 128;  // queries per workgroup
constexpr int ML_KC = 64;   // channels per LDS chunk

typedef __attribute__((ext_vector_type(4))) short ml_v4s;

template <typename T> struct MlCfg;
template <> struct MlCfg<bf16_t> {
  static constexpr int ROW = ML_TP * 2;  // 256-byte rows (the TP = 64 variant uses the first half)
  static constexpr int VEC = 8;          // pixels per 16-byte chunk
  // 32-byte block index XOR (row bits 0-1, 3): the 8 rows of a transposed read's 32-lane half
  // land on 8 distinct blocks
  static __device__ __forceinline__ int off(int row, int byte) {
    const int swz = (row & 3) | (((row >> 3) & 1) << 2);
    return row * ROW + ((((byte >> 5) ^ swz)) << 5) + (byte & 31);
  }
};
template <> struct MlCfg<float> {
  static constexpr int ROW = ML_TP * 4;  // 512-byte rows
  static constexpr int VEC = 4;
  static __device__ __forceinline__ int off(int row, int byte) {
    return row * ROW + ((((byte >> 6) ^ ((row >> 3) & 1))) << 6) + (byte & 63);
  }
};

// A fragment (pixels x 32 channels) of pixel fragment mi, k-step ks of the staged chunk
__device__ __forceinline__ Frag<bf16_t> ml_afrag(const char* s, int mi, int ks, int lane) {
  using Cfg = MlCfg<bf16_t>;
  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int row0 = 32 * ks + 8 * g + q4, row1 = row0 + 4;
  const int byte = (16 * mi + 4 * p4) * 2;
  ml_v4s t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) ml_v4s*)(s + Cfg::off(row0, byte)));
  ml_v4s t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) ml_v4s*)(s + Cfg::off(row1, byte)));
  Frag<bf16_t> f;
  f.v = make_uint4((uint32_t)(uint16_t)t0.x | ((uint32_t)(uint16_t)t0.y << 16),
                   (uint32_t)(uint16_t)t0.z | ((uint32_t)(uint16_t)t0.w << 16),
                   (uint32_t)(uint16_t)t1.x | ((uint32_t)(uint16_t)t1.y << 16),
                   (uint32_t)(uint16_t)t1.z | ((uint32_t)(uint16_t)t1.w << 16));
  return f;
}
__device__ __forceinline__ Frag<float> ml_afrag_f32(const char* s, int mi, int ks, int lane) {
  using Cfg = MlCfg<float>;
  const int r = lane & 15, g = lane >> 4;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const float*>(s + Cfg::off(32 * ks + 8 * g + j, (16 * mi + r) * 4));
  Frag<float> f;
  f.from8(v);
  return f;
}

template <typename T, int TP>
__global__ __launch_bounds__(256) void k_mask_logits(const T* __restrict__ emb, const T* __restrict__ pix, int Q, int C,
                                                      int P, T* __restrict__ out) {
  using Cfg = MlCfg<T>;
  __shared__ __attribute__((aligned(16))) char smem[ML_KC * Cfg::ROW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, g = lane >> 4;
  constexpr int MI = TP / 16;
  const int p0 = blockIdx.x * TP, qb = blockIdx.y * ML_TQ, b = blockIdx.z;
  const int qf0 = qb + 32 * wave;          // first query of this wave's two fragments
  const bool live0 = qf0 < Q, live1 = qf0 + 16 < Q;
  const T* pb = pix + (long long)b * C * P;
  const T* eb = emb + (long long)b * Q * C;
  const bool vec = (P % Cfg::VEC) == 0;

  f32x4 acc[MI][2];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) acc[mi][0] = acc[mi][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  // pixel-embedding chunk kc0 -> registers (16-byte pieces; rows past C / pixels past P zero).
  // The next chunk's loads are issued right after the current one is in LDS, so they are in
  // flight during the current chunk's MFMAs.
  constexpr int CH_PER_ROW = Cfg::ROW / 16 * TP / ML_TP, NCH = ML_KC * CH_PER_ROW, NPT = NCH / 256;
  static_assert(NCH % 256 == 0, "chunk pieces per thread");
  auto load_chunk = [&](int kc0, uint4 (&v)[NPT]) {
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int i = tid + 256 * u, row = i / CH_PER_ROW, ch = i % CH_PER_ROW;
      const int c = kc0 + row, pp = p0 + ch * Cfg::VEC;
      v[u] = make_uint4(0u, 0u, 0u, 0u);
      if (c < C) {
        const T* src = pb + (long long)c * P + pp;
        if (vec) {
          if (pp < P) v[u] = *reinterpret_cast<const uint4*>(src);
        } else {
          T e[Cfg::VEC];
#pragma unroll
          for (int j = 0; j < Cfg::VEC; ++j) e[j] = pp + j < P ? src[j] : T(0);
          __builtin_memcpy(&v[u], e, 16);
        }
      }
    }
  };
  uint4 stage[NPT];
  load_chunk(0, stage);
  for (int kc0 = 0; kc0 < C; kc0 += ML_KC) {
    // query-embedding fragments of this chunk (B operand): emb[q][kc0 + 32 ks + 8 g + 0..7]
    Frag<T> fb[2][2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int nj = 0; nj < 2; ++nj) {
        const int q = qf0 + 16 * nj + r, c = kc0 + 32 * ks + 8 * g;
        if (q < Q && c < C)
          fb[ks][nj].load(eb + (long long)q * C + c);
        else
          fb[ks][nj].zero();
      }
    __syncthreads();  // previous chunk's LDS reads done
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int i = tid + 256 * u;
      *reinterpret_cast<uint4*>(smem + Cfg::off(i / CH_PER_ROW, (i % CH_PER_ROW) * 16)) = stage[u];
    }
    __syncthreads();
    if (kc0 + ML_KC < C) load_chunk(kc0 + ML_KC, stage);
    if (live0) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) {
          Frag<T> fa;
          if constexpr (sizeof(T) == 2)
            fa = ml_afrag(smem, mi, ks, lane);
          else
            fa = ml_afrag_f32(smem, mi, ks, lane);
          mma(acc[mi][0], fa, fb[ks][0]);
          if (live1) mma(acc[mi][1], fa, fb[ks][1]);
        }
      }
    }
  }
  if (!live0) return;
  // epilogue: lane holds pixels 16 mi + 4 g + 0..3 of query qf0 + 16 nj + r
  T* ob = out + (long long)b * Q * P;
#pragma unroll
  for (int nj = 0; nj < 2; ++nj) {
    const int q = qf0 + 16 * nj + r;
    if (q >= Q) continue;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int p = p0 + 16 * mi + 4 * g;
      T* dst = ob + (long long)q * P + p;
      const f32x4 a = acc[mi][nj];
      if (p + 3 < P && (P & 3) == 0) {
        if constexpr (sizeof(T) == 4)
          *reinterpret_cast<float4*>(dst) = make_float4(a[0], a[1], a[2], a[3]);
        else
          *reinterpret_cast<uint2*>(dst) = make_uint2(pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3]));
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (p + e < P) dst[e] = Num<T>::from_f(a[e]);
      }
    }
  }
}

// torch area_pixel_compute_source_index (align_corners=False, non-cubic)
__device__ __forceinline__ float ml_src(float scale, int dst) {
  const float s = scale * ((float)dst + 0.5f) - 0.5f;
  return s < 0.f ? 0.f : s;
}

template <typename T>
__global__ __launch_bounds__(256) void k_mask_attention(const T* __restrict__ logits, int BQ, int Q, int H, int W,
                                                         int th, int tw, int heads, float rh, float rw,
                                                         uint8_t* __restrict__ attn) {
  const long long n = (long long)BQ * th * tw;
  const int tp = th * tw;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int t = (int)(i % tp);
    const long long bq = i / tp;
    const int ty = t / tw, tx = t % tw;
    const float sy = ml_src(rh, ty), sx = ml_src(rw, tx);
    const int y0 = (int)sy, x0 = (int)sx;
    const int yp = y0 < H - 1 ? 1 : 0, xp = x0 < W - 1 ? 1 : 0;
    const float l1y = sy - (float)y0, l0y = 1.f - l1y, l1x = sx - (float)x0, l0x = 1.f - l1x;
    const T* src = logits + bq * H * W;
    const float v00 = Num<T>::to_f(src[y0 * W + x0]), v01 = Num<T>::to_f(src[y0 * W + x0 + xp]);
    const float v10 = Num<T>::to_f(src[(y0 + yp) * W + x0]), v11 = Num<T>::to_f(src[(y0 + yp) * W + x0 + xp]);
    float v = l0y * (l0x * v00 + l1x * v01) + l1y * (l0x * v10 + l1x * v11);
    v = Num<T>::to_f(Num<T>::from_f(v));                 // interpolate's output dtype
    float s = 1.f / (1.f + expf(-v));
    s = Num<T>::to_f(Num<T>::from_f(s));                 // sigmoid's output dtype
    const uint8_t m = s < 0.5f ? 1 : 0;
    const long long b = bq / Q, q = bq % Q;
    for (int h = 0; h < heads; ++h) attn[((b * heads + h) * Q + q) * tp + t] = m;
  }
}

// The masked-attention decoder's memory of one feature level (Mask2FormerTransformerModule.forward,
// modeling_mask2former.py:2095-2109): proj [B][C][HW] (the input projection's output) + level
// embedding e[c], then permuted to [HW][B][C] — written in that layout directly, in float32 (the
// promoted dtype of proj + e), so the decoder's key / value projections read contiguous rows.
// Tiles of 64 pixels x 64 channels of one image, transposed through LDS.  Backward: dproj[b][c][p]
// = g[p][b][c] in proj's dtype, and per (image, pixel tile) the channel sums of g (summed by
// k_level_embed_sum over the partials in a fixed order: d e).
constexpr int LM_T = 64;
template <typename T>
__global__ __launch_bounds__(256) void k_level_mem_fwd(const T* __restrict__ proj, const float* __restrict__ e, int B,
                                                       int C, int HW, float* __restrict__ out) {
  __shared__ float t[LM_T][LM_T + 1];
  const int p0 = blockIdx.x * LM_T, c0 = blockIdx.y * LM_T, b = blockIdx.z;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll 4
  for (int ci = ty; ci < LM_T; ci += 4) {  // coalesced along pixels
    const int c = c0 + ci, p = p0 + tx;
    t[ci][tx] = (c < C && p < HW) ? Num<T>::to_f(proj[((long long)b * C + c) * HW + p]) : 0.f;
  }
  __syncthreads();
  const float ev = c0 + tx < C ? e[c0 + tx] : 0.f;
#pragma unroll 4
  for (int pi = ty; pi < LM_T; pi += 4) {  // coalesced along channels
    const int p = p0 + pi, c = c0 + tx;
    if (p < HW && c < C) out[((long long)p * B + b) * C + c] = t[tx][pi] + ev;
  }
}
template <typename T>
__global__ __launch_bounds__(256) void k_level_mem_bwd(const float* __restrict__ g, int B, int C, int HW,
                                                       T* __restrict__ dproj, float* __restrict__ part) {
  __shared__ float t[LM_T][LM_T + 1];
  __shared__ float cs[4][LM_T];
  const int p0 = blockIdx.x * LM_T, c0 = blockIdx.y * LM_T, b = blockIdx.z;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  float acc = 0.f;
#pragma unroll 4
  for (int pi = ty; pi < LM_T; pi += 4) {  // coalesced along channels; channel sums in pixel order
    const int p = p0 + pi, c = c0 + tx;
    const float v = (p < HW && c < C) ? g[((long long)p * B + b) * C + c] : 0.f;
    t[tx][pi] = v;
    acc += v;
  }
  cs[ty][tx] = acc;
  __syncthreads();
  if (ty == 0 && c0 + tx < C)
    part[((long long)b * gridDim.x + blockIdx.x) * C + c0 + tx] = (cs[0][tx] + cs[1][tx]) + (cs[2][tx] + cs[3][tx]);
#pragma unroll 4
  for (int ci = ty; ci < LM_T; ci += 4) {  // coalesced along pixels
    const int c = c0 + ci, p = p0 + tx;
    if (c < C && p < HW) dproj[((long long)b * C + c) * HW + p] = Num<T>::from_f(t[ci][tx]);
  }
}
__global__ __launch_bounds__(256) void k_level_embed_sum(const float* __restrict__ part, int n, int C,
                                                         float* __restrict__ de) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int i = 0; i < n; ++i) s += part[(long long)i * C + c];
  de[c] = s;
}

}  // namespace
}  // namespace rgbd

using namespace rgbd;

extern "C" int rgbd_mask_logits(int dtype, const void* emb, const void* pix, int B, int Q, int C, int H, int W,
                                void* logits, void* stream) {
  RGBD_REQUIRE(emb && pix && logits && B > 0 && Q > 0 && C > 0 && H > 0 && W > 0, RGBD_E_ARG);
  RGBD_REQUIRE(C % 32 == 0, RGBD_E_SHAPE);
  // 16-byte loads of the query embeddings need 16-byte aligned rows
  RGBD_REQUIRE(((uintptr_t)emb & 15) == 0 && ((uintptr_t)pix & 15) == 0 && ((uintptr_t)logits & 15) == 0,
               RGBD_E_SHAPE);
  const long long P = (long long)H * W;
  RGBD_REQUIRE(P < (1ll << 31) / 4, RGBD_E_SHAPE);
  hipStream_t s = (hipStream_t)stream;
  // 64-pixel tiles: 2400 workgroups at the C2 shape (measured: the 128-pixel tile is no faster
  // in bf16 and 10 % slower in f32)
  constexpr int TP = 64;
  dim3 grid(ceil_div(P, TP), ceil_div(Q, ML_TQ), B);
  if (dtype == RGBD_F32)
    k_mask_logits<float, TP><<<grid, 256, 0, s>>>((const float*)emb, (const float*)pix, Q, C, (int)P, (float*)logits);
  else if (dtype == RGBD_BF16)
    k_mask_logits<bf16_t, TP><<<grid, 256, 0, s>>>((const bf16_t*)emb, (const bf16_t*)pix, Q, C, (int)P,
                                                   (bf16_t*)logits);
  else
    return RGBD_E_DTYPE;
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

extern "C" int rgbd_mask_attention(int dtype, const void* logits, int B, int Q, int H, int W, int th, int tw,
                                   int heads, uint8_t* attn, void* stream) {
  RGBD_REQUIRE(logits && attn && B > 0 && Q > 0 && H > 0 && W > 0 && th > 0 && tw > 0 && heads > 0, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  const float rh = (float)H / (float)th, rw = (float)W / (float)tw;
  const long long n = (long long)B * Q * th * tw;
  const int grid = (int)std::min<long long>(ceil_div(n, 256), 8192);
  if (dtype == RGBD_F32)
    k_mask_attention<float><<<grid, 256, 0, s>>>((const float*)logits, B * Q, Q, H, W, th, tw, heads, rh, rw, attn);
  else if (dtype == RGBD_BF16)
    k_mask_attention<bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)logits, B * Q, Q, H, W, th, tw, heads, rh, rw, attn);
  else
    return RGBD_E_DTYPE;
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

extern "C" size_t rgbd_level_memory_workspace_size(int B, int C, int HW) {
  return (size_t)B * ((HW + LM_T - 1) / LM_T) * C * sizeof(float);
}

extern "C" int rgbd_level_memory_fwd(int dtype, const void* proj, const float* embed, int B, int C, int HW, float* out,
                                     void* stream) {
  RGBD_REQUIRE(proj && embed && out && B > 0 && C > 0 && HW > 0, RGBD_E_ARG);
  RGBD_REQUIRE(dtype == RGBD_F32 || dtype == RGBD_BF16, RGBD_E_DTYPE);
  const dim3 grid((HW + LM_T - 1) / LM_T, (C + LM_T - 1) / LM_T, B);
  if (dtype == RGBD_F32)
    k_level_mem_fwd<float><<<grid, 256, 0, (hipStream_t)stream>>>((const float*)proj, embed, B, C, HW, out);
  else
    k_level_mem_fwd<bf16_t><<<grid, 256, 0, (hipStream_t)stream>>>((const bf16_t*)proj, embed, B, C, HW, out);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

extern "C" int rgbd_level_memory_bwd(int dtype, const float* g, int B, int C, int HW, void* dproj, float* dembed,
                                     void* ws, void* stream) {
  RGBD_REQUIRE(g && dproj && dembed && ws && B > 0 && C > 0 && HW > 0, RGBD_E_ARG);
  RGBD_REQUIRE(dtype == RGBD_F32 || dtype == RGBD_BF16, RGBD_E_DTYPE);
  const dim3 grid((HW + LM_T - 1) / LM_T, (C + LM_T - 1) / LM_T, B);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_F32)
    k_level_mem_bwd<float><<<grid, 256, 0, s>>>(g, B, C, HW, (float*)dproj, (float*)ws);
  else
    k_level_mem_bwd<bf16_t><<<grid, 256, 0, s>>>(g, B, C, HW, (bf16_t*)dproj, (float*)ws);
  k_level_embed_sum<<<(C + 255) / 256, 256, 0, s>>>((const float*)ws, B * (int)grid.x, C, dembed);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}
