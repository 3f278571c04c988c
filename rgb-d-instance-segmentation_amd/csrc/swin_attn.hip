// f2: Swin-T's (shifted-)window multi-head self-attention on gfx950, the core of
// every SwinLayer of the backbone the reference calls at custom_model.py:330
// (transformers 5.15 modeling_swin.py SwinLayer.forward :529-582, SwinAttention.forward
// :418-468, eager_attention_forward :373-398, get_attn_mask :591-610).
//
// HF pads the LayerNorm'ed map to multiples of the window (zeros), rolls it by -shift, cuts
// 7x7 windows, projects q/k/v, adds the relative-position bias (table[(2w-1)^2][heads] gathered
// by a fixed index) and the shift mask (-100 between tokens of different shift regions),
// softmax, P.V, and undoes window / roll / pad.  Projections are per token, so here q/k/v are
// projected on the ORIGINAL token layout (one GEMM) and this kernel does the rest by index
// arithmetic: a window token (i, j) of window (wy, wx) in the rolled padded map is padded-map
// position ((7wy + i + s) mod Hp, (7wx + j + s) mod Wp); inside the H x W map it is that token's
// projection, outside it is a zero row's projection, i.e. the projection biases.  The output
// goes straight back to the token's original row.
//
// One wave per (image, window, head), head_dim 32, the 49 tokens padded to 64:
//   S^T = K Q^T   (MFMA: A = key rows, B = query rows; q and k fragments loaded straight from
//                 global, 8 consecutive dims per lane = one K step of 32 = head_dim)
//   s = S * scale + bias[h][idx(q, k)] + shift mask, keys >= 49 excluded; softmax per query
//   column in float32 (keys sit on the lane's 4 registers, its lane group and the 4 key tiles)
//   O^T = V^T P^T (MFMA: A = V^T from a transposed LDS copy of V, B = P^T straight from the
//                 accumulators — the k order of each 32-key step is the accumulators' own,
//                 applied to both operands), normalised by the row sum, 4 consecutive dims per
//                 lane stored to the query token's row.
// bf16: v_mfma_f32_16x16x32_bf16 (P rounded to bf16 as HF's eager path rounds it); f32: exact
// f32 MFMA.  Bound: latency / L2 (per (window, head) 64 x 32 x 3 operands, 2 x 49^2 x 32 MACs).
#include "common.hpp"
#include "mfma.hpp"

namespace rgbd {
namespace {

constexpr int SW_WS = 7, SW_T = 49, SW_HD = 32;
constexpr int SW_TABLE = (2 * SW_WS - 1) * (2 * SW_WS - 1);  // 169
constexpr int SW_WAVES = 4;

struct SwinArgs {
  const void *q, *k, *v;
  long long ldq;  // row stride (elements) of q / k / v (3C when they share one GEMM output)
  const float *bq, *bk, *bv;  // projection biases (padded-map tokens), may be NULL
  const float* table;         // [169][heads]
  void* out;                  // [B*H*W][ldo]
  long long ldo;
  int B, H, W, heads, shift, Hp, Wp, nwy, nwx;
  float scale;
};

template <typename T> struct SwT;
template <> struct SwT<bf16_t> {
  static constexpr int VT_S = 64 + 8;  // Vt row (keys) stride, bf16 elements
};
template <> struct SwT<float> {
  static constexpr int VT_S = 64 + 4;
};

__device__ __forceinline__ int sw_region(int y, int Hp, int s) { return (y >= Hp - SW_WS) + (y >= Hp - s); }

template <typename T>
__global__ __launch_bounds__(64 * SW_WAVES) void k_swin_attn(SwinArgs a) {
  __shared__ __attribute__((aligned(16))) T vts[SW_WAVES][SW_HD][SwT<T>::VT_S];
  __shared__ float tab[SW_WAVES][SW_TABLE + 3];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long long item = (long long)blockIdx.x * SW_WAVES + wv;
  const long long total = (long long)a.B * a.nwy * a.nwx * a.heads;
  if (item >= total) return;  // wave-uniform; no workgroup barrier below
  const int h = (int)(item % a.heads);
  long long rest = item / a.heads;
  const int wx = (int)(rest % a.nwx);
  rest /= a.nwx;
  const int wy = (int)(rest % a.nwy);
  const int b = (int)(rest / a.nwy);
  const int r = lane & 15, g = lane >> 4;
  T* vt = &vts[wv][0][0];
  float* tb = tab[wv];
  for (int i = lane; i < SW_TABLE; i += 64) tb[i] = a.table[i * a.heads + h];

  // token t of the window -> original row (or -1: padded-map position, projection = bias)
  auto token_row = [&](int t, int* region) -> long long {
    const int ti = t / SW_WS, tj = t % SW_WS;
    const int ys = wy * SW_WS + ti, xs = wx * SW_WS + tj;  // rolled padded map
    if (region) *region = a.shift > 0 ? 3 * sw_region(ys, a.Hp, a.shift) + sw_region(xs, a.Wp, a.shift) : 0;
    const int py = a.shift > 0 ? (ys + a.shift) % a.Hp : ys, px = a.shift > 0 ? (xs + a.shift) % a.Wp : xs;
    if (py >= a.H || px >= a.W) return -1;
    return ((long long)b * a.H + py) * a.W + px;
  };
  // 8 consecutive head dims (8g..8g+7) of token t's q / k / v row
  // The row's load is unconditional (a clamped row) and only the rare lanes of padded tokens
  // overwrite it: with the load inside an if / else the compiler waited for it at the join, so
  // every call was a memory round trip.
  auto frag_of = [&](const void* base, const float* bias, int t) -> Frag<T> {
    Frag<T> f;
    const long long row = t < SW_T ? token_row(t, nullptr) : -1;
    const int d0 = h * SW_HD + 8 * g;
    f.load(reinterpret_cast<const T*>(base) + (row >= 0 ? row : 0) * a.ldq + d0);
    if (row < 0) {
      if (t >= SW_T) {
        f.zero();
      } else {
        float e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) e[j] = bias ? bias[d0 + j] : 0.f;
        f.from8(e);  // the GEMM output of a zero row: bias (rounded to the operand dtype)
      }
    }
    return f;
  };

  // V^T into LDS: lane = token, its 32 dims as four 8-dim fragments
  {
    const int t = lane;
    // the row's four fragments loaded first and unconditionally (a clamped row), then converted;
    // only the rare lanes of padded tokens overwrite them with the bias (as frag_of): inside an
    // if / else, or converted as they arrive, each load was a memory round trip of its own
    const long long row = t < SW_T ? token_row(t, nullptr) : -1;
    Frag<T> fv[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) fv[c].load(reinterpret_cast<const T*>(a.v) + (row >= 0 ? row : 0) * a.ldq + h * SW_HD + 8 * c);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int d0 = h * SW_HD + 8 * c;
      float e[8];
      fv[c].to8(e);
      if (row < 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          e[j] = t < SW_T && a.bv ? Num<T>::to_f(Num<T>::from_f(a.bv[d0 + j])) : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) vt[(8 * c + j) * SwT<T>::VT_S + t] = Num<T>::from_f(e[j]);
    }
  }
  Frag<T> kf[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) kf[j] = frag_of(a.k, a.bk, 16 * j + r);
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  for (int qi = 0; qi < 4; ++qi) {
    const int tq = 16 * qi + r;  // this lane's query (column of S^T)
    int qreg = 0;
    const long long qrow = tq < SW_T ? token_row(tq, &qreg) : -1;
    const Frag<T> qf = frag_of(a.q, a.bq, tq);
    const int qy = tq / SW_WS, qx = tq % SW_WS;
    f32x4 s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      mma(s[j], kf[j], qf);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int tk = 16 * j + 4 * g + e;
        float v = -INFINITY;
        if (tk < SW_T) {
          const int ky = tk / SW_WS, kx = tk % SW_WS;
          const int idx = (qy - ky + SW_WS - 1) * (2 * SW_WS - 1) + (qx - kx + SW_WS - 1);
          int kreg = 0;
          if (a.shift > 0) token_row(tk, &kreg);
          // HF: (q k^T) * scale + (bias + shift mask), the mask added to the bias first
          const float bm = tb[idx] + (a.shift > 0 && kreg != qreg ? -100.f : 0.f);
          v = s[j][e] * a.scale + bm;
        }
        s[j][e] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    float l = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float p = s[j][e] == -INFINITY ? 0.f : expf(s[j][e] - mx);
        s[j][e] = p;
        l += p;
      }
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    const float inv = 1.f / l;
    // P^T as the B operand: 32-key step kp covers key tiles 2kp, 2kp+1; element e of the first
    // half is key 16(2kp) + 4g + e, of the second half key 16(2kp+1) + 4g + e.  The softmax is
    // normalised before the rounding to the operand dtype, as HF's softmax(...).to(dtype).
    Frag<T> pf[2];
#pragma unroll
    for (int kp = 0; kp < 2; ++kp) {
      float e8[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        e8[e] = s[2 * kp][e] * inv;
        e8[4 + e] = s[2 * kp + 1][e] * inv;
      }
      pf[kp].from8(e8);
    }
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kp = 0; kp < 2; ++kp) {
        // V^T fragment in the same key order: dims 16 dt + r, keys 16(2kp) + 4g + 0..3 and
        // 16(2kp+1) + 4g + 0..3
        const T* row = vt + (16 * dt + r) * SwT<T>::VT_S;
        float e8[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          e8[e] = Num<T>::to_f(row[32 * kp + 4 * g + e]);
          e8[4 + e] = Num<T>::to_f(row[32 * kp + 16 + 4 * g + e]);
        }
        Frag<T> vf;
        vf.from8(e8);
        mma(o, vf, pf[kp]);
      }
      // o[e] = O^T[dim 16 dt + 4 g + e][query tq]
      if (qrow >= 0) {
        T* dst = reinterpret_cast<T*>(a.out) + qrow * a.ldo + h * SW_HD + 16 * dt + 4 * g;
        if constexpr (sizeof(T) == 2) {
          *reinterpret_cast<uint2*>(dst) = make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
        } else {
          *reinterpret_cast<float4*>(dst) = make_float4(o[0], o[1], o[2], o[3]);
        }
      }
    }
  }
}

}  // namespace
}  // namespace rgbd

using namespace rgbd;

extern "C" {

int rgbd_swin_window_attn(int dtype, const void* q, const void* k, const void* v, long long ldq, const float* bq,
                          const float* bk, const float* bv, const float* table, int B, int H, int W, int heads,
                          int window, int shift, float scale, void* out, long long ldo, void* stream) {
  RGBD_REQUIRE(q && k && v && table && out && B > 0 && H > 0 && W > 0 && heads > 0, RGBD_E_ARG);
  RGBD_REQUIRE(window == SW_WS && shift >= 0 && shift < SW_WS, RGBD_E_SHAPE);
  RGBD_REQUIRE(ldq >= (long long)heads * SW_HD && ldo >= (long long)heads * SW_HD, RGBD_E_SHAPE);
  const int esz = dtype == RGBD_BF16 ? 2 : 4;
  RGBD_REQUIRE((ldq * esz) % 16 == 0 && (ldo * esz) % 16 == 0, RGBD_E_SHAPE);
  RGBD_REQUIRE(((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)out) % 16 == 0, RGBD_E_SHAPE);
  SwinArgs a;
  a.q = q; a.k = k; a.v = v; a.ldq = ldq;
  a.bq = bq; a.bk = bk; a.bv = bv; a.table = table;
  a.out = out; a.ldo = ldo;
  a.B = B; a.H = H; a.W = W; a.heads = heads; a.shift = shift;
  a.Hp = (H + SW_WS - 1) / SW_WS * SW_WS;
  a.Wp = (W + SW_WS - 1) / SW_WS * SW_WS;
  a.nwy = a.Hp / SW_WS; a.nwx = a.Wp / SW_WS;
  a.scale = scale;
  const long long items = (long long)B * a.nwy * a.nwx * heads;
  const int blocks = (int)((items + SW_WAVES - 1) / SW_WAVES);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_BF16)
    hipLaunchKernelGGL(k_swin_attn<bf16_t>, dim3(blocks), dim3(64 * SW_WAVES), 0, s, a);
  else if (dtype == RGBD_F32)
    hipLaunchKernelGGL(k_swin_attn<float>, dim3(blocks), dim3(64 * SW_WAVES), 0, s, a);
  else
    return RGBD_E_DTYPE;
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
