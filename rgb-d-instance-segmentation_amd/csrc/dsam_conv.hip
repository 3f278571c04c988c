// K5: DSAM masked 3x3/stride-2 convolutions as MFMA implicit GEMMs (gfx950).
//
// Reference: DSAModule.forward (mask2former/utils/custom_model.py:682-699) evaluates, per
// sample, four Conv3x3s2 on rgb_features * pooled_mask_i plus a bias-free projection conv,
// i.e. five convolutions at batch 1 (and the Python loop of :339-352 repeats it per sample).
// Here one launch covers the whole batch and all five convolutions:
//
//   out[m, n] = sum_{seg<5} sum_{tap<9} sum_{c<Cin} Wseg[n, c, tap] * x[src(m, tap), c] * bit_seg
//
// with K = 5*9*Cin ordered (seg, tap, c): the A operand (im2col of the NHWC input) is loaded
// once per (tap, 32-channel chunk) and re-used by all five segments; segment `seg` < 4 keeps
// an element only where bit `seg` of the pooled region code of its SOURCE pixel is set
// (x * mask, :689).  A segment whose bit is absent from every pixel of a wave's 32 rows is
// skipped (its contribution is exactly zero), which removes most masked FLOPs on real scenes.
//
// dX (training) is the transposed convolution with the same packed structure: output pixels
// are split into the four stride-2 parity classes so only live taps are visited, and the
// mask bit is taken at the OUTPUT pixel (d(x*m)/dx = m).  dW contracts over pixels with an
// LDS-staged im2col tile.
#include "mfma.hpp"
#include "timing.hpp"

using namespace rgbd;

namespace {

enum { MASK_NONE = 0, MASK_SRC = 1, MASK_DST = 2 };

struct ConvArgs {
  const void* x;          // NHWC [B][Hi][Wi][C]
  const uint8_t* code;    // region codes: [B][Hi][Wi] (MASK_SRC) or [B][Ho][Wo] (MASK_DST)
  const void* w;          // packed B operand [N][nseg * KH*KW * C]
  int B, Hi, Wi, C;
  int Ho, Wo, N;
  int KH, KW, stride, pad;
  int nseg, mask_mode, transposed;
  const float* bias4;               // DSAM conv biases [4][N] (summed over i < n_masks[b])
  const rgbd_decomp_info* info;
  const void* residual;             // NCHW [B][N][Ho][Wo] added in the epilogue (optional)
  void* out_nchw;                   // optional
  void* out_nhwc;                   // optional
  int ksplit;                       // v2 only: K split over (tap, chunk) ranges (1 = none)
  float* partial;                   // v2 split-K slabs: f32 [ksplit][B][Ho][Wo][N]
  uint16_t* tile_codes;             // bf16: [nclass][M tiles][9] codes present per tap
};

constexpr int BM = 64, BN = 64;

template <typename T>
__global__ __launch_bounds__(256) void k_conv_igemm(ConvArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int wm = wave & 1, wn = wave >> 1;
  int py = 0, px = 0, Hc = a.Ho, Wc = a.Wo;
  if (a.transposed) {
    py = blockIdx.z >> 1;
    px = blockIdx.z & 1;
    Hc = (a.Ho - py + 1) >> 1;
    Wc = (a.Wo - px + 1) >> 1;
  }
  const long long HWc = (long long)Hc * Wc;
  const long long Mtot = (long long)a.B * HWc;
  const long long mbase = (long long)blockIdx.x * BM + wm * 32;
  const int nbase = blockIdx.y * BN + wn * 32;
  if (mbase >= Mtot) return;  // wave-uniform

  int rb[2], roy[2], rox[2];
  bool rvalid[2];
  uint32_t rcode[2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const long long m = mbase + 16 * mi + r;
    rvalid[mi] = m < Mtot;
    const long long mm = rvalid[mi] ? m : 0;
    rb[mi] = (int)(mm / HWc);
    const int rem = (int)(mm % HWc);
    const int i = rem / Wc, j = rem % Wc;
    roy[mi] = a.transposed ? 2 * i + py : i;
    rox[mi] = a.transposed ? 2 * j + px : j;
    rcode[mi] = (a.mask_mode == MASK_DST && rvalid[mi])
                    ? a.code[((long long)rb[mi] * a.Ho + roy[mi]) * a.Wo + rox[mi]]
                    : 0xffu;
  }
  const int ntap = a.KH * a.KW;
  const long long ktot = (long long)a.nseg * ntap * a.C;
  const T* wp = (const T*)a.w;
  const T* xp = (const T*)a.x;
  bool nvalid[2];
  const T* wrow[2];
#pragma unroll
  for (int nj = 0; nj < 2; ++nj) {
    const int n = nbase + 16 * nj + r;
    nvalid[nj] = n < a.N;
    wrow[nj] = wp + (long long)(nvalid[nj] ? n : 0) * ktot + 8 * g;
  }
  f32x4 acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj) acc[mi][nj] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int ky = 0; ky < a.KH; ++ky) {
    if (a.transposed && ((py + a.pad - ky) & 1)) continue;
    for (int kx = 0; kx < a.KW; ++kx) {
      if (a.transposed && ((px + a.pad - kx) & 1)) continue;
      const int tap = ky * a.KW + kx;
      const T* src[2];
      bool inb[2];
      uint32_t scode[2];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        int iy, ix;
        if (a.transposed) {
          iy = (roy[mi] + a.pad - ky) >> 1;
          ix = (rox[mi] + a.pad - kx) >> 1;
        } else {
          iy = roy[mi] * a.stride - a.pad + ky;
          ix = rox[mi] * a.stride - a.pad + kx;
        }
        inb[mi] = rvalid[mi] && iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi;
        const long long pix = inb[mi] ? ((long long)rb[mi] * a.Hi + iy) * a.Wi + ix : 0;
        src[mi] = xp + pix * a.C + 8 * g;
        scode[mi] = (a.mask_mode == MASK_SRC) ? (inb[mi] ? a.code[pix] : 0u) : rcode[mi];
      }
      for (int c0 = 0; c0 < a.C; c0 += 32) {
        const bool cok = c0 + 8 * g < a.C;  // C % 8 == 0: a lane's 8-chunk is all in or all out
        Frag<T> A[2];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          if (inb[mi] && cok)
            A[mi].load(src[mi] + c0);
          else
            A[mi].zero();
        }
        for (int seg = 0; seg < a.nseg; ++seg) {
          bool keep[2] = {true, true};
          if (a.mask_mode != MASK_NONE && seg < 4) {
            keep[0] = (scode[0] >> seg) & 1u;
            keep[1] = (scode[1] >> seg) & 1u;
            if (!__any(keep[0] || keep[1])) continue;  // all-zero segment for this wave
          }
          Frag<T> As[2] = {A[0], A[1]};
          As[0].select(keep[0]);
          As[1].select(keep[1]);
          const long long koff = ((long long)seg * ntap + tap) * a.C + c0;
#pragma unroll
          for (int nj = 0; nj < 2; ++nj) {
            Frag<T> Bf;
            if (nvalid[nj] && cok)
              Bf.load(wrow[nj] + koff);
            else
              Bf.zero();
            mma(acc[0][nj], As[0], Bf);
            mma(acc[1][nj], As[1], Bf);
          }
        }
      }
    }
  }

  // epilogue: D[m = row][n = col], row = 4g + reg, col = r
  const T* res = (const T*)a.residual;
  T* onchw = (T*)a.out_nchw;
  T* onhwc = (T*)a.out_nhwc;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const long long m = mbase + 16 * mi + 4 * g + reg;
      if (m >= Mtot) continue;
      const int b = (int)(m / HWc);
      const int rem = (int)(m % HWc);
      const int i = rem / Wc, j = rem % Wc;
      const int oy = a.transposed ? 2 * i + py : i;
      const int ox = a.transposed ? 2 * j + px : j;
      int nmask = 0;
      if (a.info) nmask = a.info[b].n_masks;
#pragma unroll
      for (int nj = 0; nj < 2; ++nj) {
        const int n = nbase + 16 * nj + r;
        if (n >= a.N) continue;
        float v = acc[mi][nj][reg];
        if (a.bias4) {
          float bs = 0.f;
          for (int s = 0; s < nmask; ++s) bs += a.bias4[s * a.N + n];
          v += bs;
        }
        const long long o_nchw = (((long long)b * a.N + n) * a.Ho + oy) * a.Wo + ox;
        if (res) v = Num<T>::to_f(res[o_nchw]) + v;
        const T tv = Num<T>::from_f(v);
        if (onchw) onchw[o_nchw] = tv;
        if (onhwc) onhwc[(((long long)b * a.Ho + oy) * a.Wo + ox) * a.N + n] = tv;
      }
    }
  }
}

template <typename T>
__global__ void k_pack_dsam(const float* __restrict__ conv_w, const float* __restrict__ proj_w, int Cin,
                            int Cout, T* __restrict__ wfwd, T* __restrict__ wbwd) {
  // element (seg, o, c, tap) of W_seg
  const long long total = 5ll * Cout * Cin * 9;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int tap = (int)(e % 9);
    const int c = (int)((e / 9) % Cin);
    const int o = (int)((e / (9ll * Cin)) % Cout);
    const int seg = (int)(e / (9ll * Cin * Cout));
    const float v = seg < 4 ? conv_w[(((long long)seg * Cout + o) * Cin + c) * 9 + tap]
                            : proj_w[((long long)o * Cin + c) * 9 + tap];
    const T tv = Num<T>::from_f(v);
    if (wfwd) wfwd[(long long)o * 45 * Cin + ((long long)seg * 9 + tap) * Cin + c] = tv;
    if (wbwd) wbwd[(long long)c * 45 * Cout + ((long long)seg * 9 + tap) * Cout + o] = tv;
  }
}

// bf16 code-merged filters: W_k = proj + sum_{i in k} conv_i for every 4-bit code k (fixed
// summation order: proj, then conv_0..conv_3, in f32, rounded once).  wfwd[k][o][tap*Cin + c],
// wbwd[k][c][tap*Cout + o].
__global__ void k_pack_dsam_codes(const float* __restrict__ conv_w, const float* __restrict__ proj_w, int Cin,
                                  int Cout, bf16_t* __restrict__ wfwd, bf16_t* __restrict__ wbwd) {
  const long long per = (long long)Cout * Cin * 9;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < per;
       e += (long long)gridDim.x * blockDim.x) {
    const int tap = (int)(e % 9);
    const int c = (int)((e / 9) % Cin);
    const int o = (int)(e / (9ll * Cin));
    float w4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w4[i] = conv_w[(((long long)i * Cout + o) * Cin + c) * 9 + tap];
    const float wp = proj_w[e];
#pragma unroll 1
    for (int k = 0; k < 16; ++k) {
      float v = wp;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if ((k >> i) & 1) v += w4[i];
      const bf16_t tv = f32_to_bf16(v);
      if (wfwd) wfwd[((long long)k * Cout + o) * 9 * Cin + (long long)tap * Cin + c] = tv;
      if (wbwd) wbwd[((long long)k * Cin + c) * 9 * Cout + (long long)tap * Cout + o] = tv;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_nchw_to_nhwc(const T* __restrict__ src, T* __restrict__ dst, int C,
                                                      int HW) {
  __shared__ T tile[32][33];
  const int b = blockIdx.z;
  const int p0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int k = ty; k < 32; k += 8) {
    const int c = c0 + k, p = p0 + tx;
    if (c < C && p < HW) tile[k][tx] = src[((long long)b * C + c) * HW + p];
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int p = p0 + k, c = c0 + tx;
    if (c < C && p < HW) dst[((long long)b * HW + p) * C + c] = tile[tx][k];
  }
}

// ----------------------------------------------------------------------- dW
// D[o][kk] = sum_m G[m][o] * X[m][kk],  kk = (seg*9 + tap)*Cin + c,  per split z (images).
template <typename T>
__global__ __launch_bounds__(256) void k_dsam_wgrad(const T* __restrict__ gout, const T* __restrict__ x,
                                                    const uint8_t* __restrict__ code, int B, int Cin,
                                                    int h, int w, int Cout, int splits,
                                                    float* __restrict__ partial) {
  __shared__ T Gs[64][32 + 8];   // [o][px]
  __shared__ T Xs[32][64 + 8];   // [px][kk]
  const int ho = (h + 1) / 2, wo = (w + 1) / 2;  // 3x3 s2 p1
  const int hwo = ho * wo;
  const int KK = 45 * Cin;
  const int kk0 = blockIdx.x * 64, o0 = blockIdx.y * 64, z = blockIdx.z;
  const int b0 = (int)((long long)z * B / splits), b1 = (int)((long long)(z + 1) * B / splits);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int wm = wave & 1, wn = wave >> 1;
  f32x4 acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj) acc[mi][nj] = f32x4{0.f, 0.f, 0.f, 0.f};
  // staging roles
  const int go = threadIdx.x >> 2, gp = (threadIdx.x & 3) * 8;     // G: o row, 8 px
  const int xpx = threadIdx.x >> 3, xk = (threadIdx.x & 7) * 8;     // X: px row, 8 kk
  const int kk = kk0 + xk;
  const bool kk_ok = kk < KK;
  const int seg = kk_ok ? kk / (9 * Cin) : 0;
  const int tap = kk_ok ? (kk / Cin) % 9 : 0;
  const int cc = kk_ok ? kk % Cin : 0;
  const int ky = tap / 3, kx = tap % 3;
  for (int b = b0; b < b1; ++b) {
    for (int p0 = 0; p0 < hwo; p0 += 32) {
      __syncthreads();
      {  // stage G^T tile
        const int o = o0 + go;
        for (int j = 0; j < 8; ++j) {
          const int p = p0 + gp + j;
          Gs[go][gp + j] = (o < Cout && p < hwo) ? gout[((long long)b * Cout + o) * hwo + p] : (T)0;
        }
      }
      {  // stage im2col tile
        const int p = p0 + xpx;
        bool ok = kk_ok && p < hwo;
        int iy = 0, ix = 0;
        if (ok) {
          iy = 2 * (p / wo) - 1 + ky;
          ix = 2 * (p % wo) - 1 + kx;
          ok = iy >= 0 && iy < h && ix >= 0 && ix < w;
        }
        const long long pix = ((long long)b * h + iy) * w + ix;
        if (ok && seg < 4) ok = (code[pix] >> seg) & 1u;
        for (int j = 0; j < 8; ++j) Xs[xpx][xk + j] = ok ? x[pix * Cin + cc + j] : (T)0;
      }
      __syncthreads();
      Frag<T> Af[2], Bf[2];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        const int o = wm * 32 + 16 * mi + r;
#pragma unroll
        for (int j = 0; j < 8; ++j) Af[mi].set(j, Num<T>::to_f(Gs[o][8 * g + j]));
      }
#pragma unroll
      for (int nj = 0; nj < 2; ++nj) {
        const int c = wn * 32 + 16 * nj + r;
#pragma unroll
        for (int j = 0; j < 8; ++j) Bf[nj].set(j, Num<T>::to_f(Xs[8 * g + j][c]));
      }
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int nj = 0; nj < 2; ++nj) mma(acc[mi][nj], Af[mi], Bf[nj]);
    }
  }
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int o = o0 + wm * 32 + 16 * mi + 4 * g + reg;
#pragma unroll
      for (int nj = 0; nj < 2; ++nj) {
        const int c = kk0 + wn * 32 + 16 * nj + r;
        if (o < Cout && c < KK) partial[((long long)z * Cout + o) * KK + c] = acc[mi][nj][reg];
      }
    }
}

// bf16 dW, code-merged (see k_conv_codes): the workgroup for code k accumulates
//   dW_k[o][tap][c] = sum over output px p with code(src(p, tap)) == k of G[p][o] X[src][c]
// over its batch split, skipping every 32-px chunk whose rows never meet code k (presence table
// from k_code_presence: no loads at all); k_dsam_wgrad_combine folds dW_k into the five filters
// (conv_i gets the codes with bit i, proj gets all).  Work ~ one dense dW instead of
// popcount + 1 of them.  X tile staged [px][kk] from NHWC with 16-byte loads, read back transposed
// with ds_read_b64_tr_b16 (gfx950) as the MFMA B operand; the A operand (G^T, 8 consecutive
// pixels of one channel, NCHW) is loaded one chunk ahead into registers.
constexpr int WG_KK = 128, WG_O = 64, PXC = 32, XPAD = 136;
typedef __attribute__((ext_vector_type(4))) short v4s;

__global__ void k_code_presence(const uint8_t* __restrict__ code, int B, int h, int w,
                                uint16_t* __restrict__ pres, uint32_t* __restrict__ gmask) {
  // one 32-lane group per (b, 32-px output chunk): OR of 1 << code over the chunk's 9-tap sources
  const int ho = (h + 1) / 2, wo = (w + 1) / 2, hwo = ho * wo, nchunk = (hwo + PXC - 1) / PXC;
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long grp = t >> 5;
  const int l = (int)(t & 31);
  uint32_t m = 0u;
  if (grp < (long long)B * nchunk) {
    const int b = (int)(grp / nchunk), p = (int)(grp % nchunk) * PXC + l;
    if (p < hwo) {
      const int oy = p / wo, ox = p % wo;
      for (int tap = 0; tap < 9; ++tap) {
        const int iy = 2 * oy - 1 + tap / 3, ix = 2 * ox - 1 + tap % 3;
        if (iy >= 0 && iy < h && ix >= 0 && ix < w) m |= 1u << code[((long long)b * h + iy) * w + ix];
      }
    }
  }
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) m |= (uint32_t)__shfl_xor((int)m, o);
  if (l == 0 && grp < (long long)B * nchunk) {
    pres[grp] = (uint16_t)m;
    if (m) atomicOr(gmask, m);
  }
}

__global__ __launch_bounds__(256) void k_dsam_wgrad_bf16(const bf16_t* __restrict__ gout, const bf16_t* __restrict__ x,
                                                         const uint8_t* __restrict__ code,
                                                         const uint16_t* __restrict__ pres,
                                                         const uint32_t* __restrict__ gmask, int B, int Cin, int h,
                                                         int w, int Cout, int splits, float* __restrict__ partial) {
  __shared__ __attribute__((aligned(16))) bf16_t Xs[2][PXC][XPAD];
  const int kcode = blockIdx.z & 15, split = blockIdx.z >> 4;
  if (!((*gmask >> kcode) & 1u)) return;  // code absent from the batch: no partial, combine skips it
  const int ho = (h + 1) / 2, wo = (w + 1) / 2;
  const int hwo = ho * wo;
  const int KK = 9 * Cin;
  const int kk0 = blockIdx.x * WG_KK, o0 = blockIdx.y * WG_O;
  const int b0 = (int)((long long)split * B / splits), b1 = (int)((long long)(split + 1) * B / splits);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  // staging role: pixel row spx, two 8-channel chunks at kk0 + 16*skg + 8*q
  const int spx = threadIdx.x >> 3, skg = threadIdx.x & 7;
  int s_ky[2], s_kx[2], s_c[2];
  bool s_ok[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int kk = kk0 + 16 * skg + 8 * q;
    s_ok[q] = kk < KK;
    const int k2 = s_ok[q] ? kk : 0;
    const int tap = k2 / Cin;
    s_ky[q] = tap / 3;
    s_kx[q] = tap % 3;
    s_c[q] = k2 % Cin;
  }
  const int nchunk = (hwo + PXC - 1) / PXC;
  const int total = (b1 - b0) * nchunk;
  auto chunk_live = [&](int it) {
    return (pres[(long long)(b0 + it / nchunk) * nchunk + it % nchunk] >> kcode) & 1u;
  };
  auto next_live = [&](int it) {
    while (it < total && !chunk_live(it)) ++it;
    return it;
  };
  int staged_any = 0;  // does the staged chunk hold any element of code k?
  auto stage = [&](int buf, int it) {
    const int b = b0 + it / nchunk, p = (it % nchunk) * PXC + spx;
    const int oy = p / wo, ox = p % wo;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int iy = 2 * oy - 1 + s_ky[q], ix = 2 * ox - 1 + s_kx[q];
      bool ok = s_ok[q] && p < hwo && iy >= 0 && iy < h && ix >= 0 && ix < w;
      const long long pix = ((long long)b * h + iy) * w + ix;
      if (ok) ok = code[pix] == kcode;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (ok) v = *reinterpret_cast<const uint4*>(x + pix * Cin + s_c[q]);
      staged_any |= ok ? 1 : 0;
      *reinterpret_cast<uint4*>(&Xs[buf][spx][16 * skg + 8 * q]) = v;
    }
  };
  // A: G^T rows o, 8 consecutive pixels of chunk it
  auto load_a = [&](Frag<bf16_t>* af, int it) {
    const int b = b0 + it / nchunk, pa = (it % nchunk) * PXC + 8 * g;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int o = o0 + 16 * mi + r;
      const bf16_t* src = gout + ((long long)b * Cout + (o < Cout ? o : 0)) * hwo + pa;
      if (o < Cout && pa + 8 <= hwo && (hwo & 3) == 0) {
        // 8-byte aligned (hwo % 4 == 0, pa % 8 == 0): two 8-byte loads
        const uint2 lo = *reinterpret_cast<const uint2*>(src);
        const uint2 hi = *reinterpret_cast<const uint2*>(src + 4);
        af[mi].v = make_uint4(lo.x, lo.y, hi.x, hi.y);
      } else {
        af[mi].zero();
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (o < Cout && pa + j < hwo) af[mi].set_raw(j, src[j]);
      }
    }
  };
  f32x4 acc[4][2];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj) acc[mi][nj] = f32x4{0.f, 0.f, 0.f, 0.f};
  Frag<bf16_t> af[4], afn[4];
  int cur = next_live(0), buf = 0;
  if (cur < total) {
    stage(0, cur);
    load_a(af, cur);
  }
  int live = __syncthreads_or(staged_any);
  while (cur < total) {
    const int nxt = next_live(cur + 1);
    staged_any = 0;
    if (nxt < total) {
      stage(buf ^ 1, nxt);
      load_a(afn, nxt);
    }
    if (live) {
      // B: transposed LDS reads, columns (kk) wave*32 + 16*nj + i, rows (px) 8g .. 8g+7
      const int q4 = (lane & 15) >> 2, p4 = lane & 3;
#pragma unroll
      for (int nj = 0; nj < 2; ++nj) {
        const int col = wave * 32 + 16 * nj + 4 * p4;
        v4s t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s*)(&Xs[buf][8 * g + q4][col]));
        v4s t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s*)(&Xs[buf][8 * g + 4 + q4][col]));
        Frag<bf16_t> bf;
        bf.v = make_uint4((uint32_t)(uint16_t)t0.x | ((uint32_t)(uint16_t)t0.y << 16),
                          (uint32_t)(uint16_t)t0.z | ((uint32_t)(uint16_t)t0.w << 16),
                          (uint32_t)(uint16_t)t1.x | ((uint32_t)(uint16_t)t1.y << 16),
                          (uint32_t)(uint16_t)t1.z | ((uint32_t)(uint16_t)t1.w << 16));
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) mma(acc[mi][nj], af[mi], bf);
      }
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) af[mi] = afn[mi];
    live = __syncthreads_or(staged_any);
    buf ^= 1;
    cur = nxt;
  }
  float* dst = partial + ((long long)(split * 16 + kcode) * Cout) * KK;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int o = o0 + 16 * mi + 4 * g + reg;
#pragma unroll
      for (int nj = 0; nj < 2; ++nj) {
        const int c = kk0 + wave * 32 + 16 * nj + r;
        if (o < Cout && c < KK) dst[(long long)o * KK + c] = acc[mi][nj][reg];
      }
    }
}

// dW_k (present codes, split partials) -> the reference filters, fixed summation order
__global__ void k_dsam_wgrad_combine(const float* __restrict__ partial, int splits,
                                     const uint32_t* __restrict__ gmask, int Cin, int Cout,
                                     float* __restrict__ dconv_w, float* __restrict__ dproj_w) {
  const long long KK = 9ll * Cin;
  const long long total = (long long)Cout * KK;
  const uint32_t m = *gmask;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    float seg[4] = {0.f, 0.f, 0.f, 0.f}, pr = 0.f;
    for (int k = 0; k < 16; ++k) {
      if (!((m >> k) & 1u)) continue;
      float v = 0.f;
      for (int sp = 0; sp < splits; ++sp) v += partial[(long long)(sp * 16 + k) * total + e];
      pr += v;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if ((k >> i) & 1) seg[i] += v;
    }
    const int o = (int)(e / KK);
    const int kk = (int)(e % KK);
    const int tap = kk / Cin, c = kk % Cin;
#pragma unroll
    for (int i = 0; i < 4; ++i) dconv_w[(((long long)i * Cout + o) * Cin + c) * 9 + tap] = seg[i];
    dproj_w[((long long)o * Cin + c) * 9 + tap] = pr;
  }
}

__global__ void k_dsam_wgrad_final(const float* __restrict__ partial, int splits, int Cin, int Cout,
                                   float* __restrict__ dconv_w, float* __restrict__ dproj_w) {
  const long long KK = 45ll * Cin;
  const long long total = (long long)Cout * KK;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int z = 0; z < splits; ++z) s += partial[(long long)z * total + e];  // fixed order
    const int o = (int)(e / KK);
    const int kk = (int)(e % KK);
    const int seg = kk / (9 * Cin), tap = (kk / Cin) % 9, c = kk % Cin;
    if (seg < 4)
      dconv_w[(((long long)seg * Cout + o) * Cin + c) * 9 + tap] = s;
    else
      dproj_w[((long long)o * Cin + c) * 9 + tap] = s;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_chan_sum(const T* __restrict__ g, int HW, float* __restrict__ out) {
  // out[b*C + c] = sum_p g[b][c][p]   (one block per (b, c))
  __shared__ float red[4];
  const long long base = (long long)blockIdx.x * HW;
  float s = 0.f;
  for (int p = threadIdx.x; p < HW; p += 256) s += Num<T>::to_f(g[base + p]);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ void k_dsam_bias_grad(const float* __restrict__ csum, const rgbd_decomp_info* info, int B,
                                 int Cout, float* __restrict__ dbias) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;  // (i, o)
  if (t >= 4 * Cout) return;
  const int i = t / Cout, o = t % Cout;
  float s = 0.f;
  for (int b = 0; b < B; ++b)
    if (i < info[b].n_masks) s += csum[b * Cout + o];  // conv_layers[i] used only if i < len(masks)
  dbias[t] = s;
}

// ----------------------------------------------------------------------- bf16: code-merged
// The masked sum  sum_i conv_i(x * m_i) + proj(x)  is regrouped by region CODE (the 4-bit
// pooled mask pattern of a source pixel, bit i = m_i): a source pixel with code k meets the
// merged filter  W_k = proj + sum_{i in k} conv_i  (packed per code by k_pack_dsam_codes), so
// each im2col row is multiplied by ONE filter instead of popcount(k) + 1 of them.
//
// Workgroup tile 128 output pixels (flattened over batch x grid, or over one stride-2 parity
// class for dX) x 128 output channels; 4 waves as 2x2, wave tile 64 px x 64 ch (4x4 MFMA).
// The K loop runs over (tap, code present among the tile's rows at that tap, 32-ch chunk);
// a row whose code differs from the step's contributes zero (register select).  A (im2col rows,
// 16 B per lane straight from NHWC) and B (W_k rows) of step s+1 are loaded while step s runs;
// B goes through a double-buffered LDS tile with 64-byte rows XOR-swizzled by row bit 2
// (conflict-free ds_read_b128 / ds_write_b128).
constexpr int V2M = 128, V2N = 128;
__device__ __forceinline__ int cm_slot(int row, int chunk) { return row * 32 + 8 * (chunk ^ ((row >> 1) & 2)); }

// Pre-pass of k_conv_codes: for each 128-row tile (and stride-2 parity class of dX), the set
// of region codes its rows meet at each tap (one thread per row; computed once per conv instead
// of once per (N tile, K split) workgroup).
__global__ __launch_bounds__(128) void k_conv_tile_codes(ConvArgs a) {
  __shared__ uint32_t sm[9];
  const int nclass = a.transposed ? 4 : 1;
  const int cls = blockIdx.z;
  int py = 0, px = 0, Hc = a.Ho, Wc = a.Wo;
  if (a.transposed) {
    py = cls >> 1;
    px = cls & 1;
    Hc = (a.Ho - py + 1) >> 1;
    Wc = (a.Wo - px + 1) >> 1;
  }
  if (threadIdx.x < 9) sm[threadIdx.x] = 0u;
  __syncthreads();
  const long long HWc = (long long)Hc * Wc, Mtot = (long long)a.B * HWc;
  const long long m = (long long)blockIdx.x * V2M + threadIdx.x;
  if (m < Mtot) {
    const int b = (int)(m / HWc), rem = (int)(m % HWc), i = rem / Wc, j = rem % Wc;
    const int oy = a.transposed ? 2 * i + py : i, ox = a.transposed ? 2 * j + px : j;
    const uint32_t rc = a.mask_mode == MASK_DST ? a.code[((long long)b * a.Ho + oy) * a.Wo + ox] : 0u;
    int t = 0;
    for (int ky = 0; ky < 3; ++ky)
      for (int kx = 0; kx < 3; ++kx) {
        if (a.transposed && (((py + 1 - ky) & 1) || ((px + 1 - kx) & 1))) continue;
        int iy, ix;
        if (a.transposed) {
          iy = (oy + 1 - ky) >> 1;
          ix = (ox + 1 - kx) >> 1;
        } else {
          iy = oy * 2 - 1 + ky;
          ix = ox * 2 - 1 + kx;
        }
        if (iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi) {
          const uint32_t c = a.mask_mode == MASK_SRC ? a.code[((long long)b * a.Hi + iy) * a.Wi + ix] : rc;
          atomicOr(&sm[t], 1u << c);
        }
        ++t;
      }
  }
  __syncthreads();
  if (threadIdx.x < 9) a.tile_codes[((long long)cls * gridDim.x + blockIdx.x) * 9 + threadIdx.x] = (uint16_t)sm[threadIdx.x];
  (void)nclass;
}

__global__ __launch_bounds__(256) void k_conv_codes(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t sB[2][V2N * 32];
  __shared__ uint8_t tcl[9 * 16], tcnt[9], tfirst[9];
  __shared__ int tbase[10], tdelta[9], ttap[9];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int wm = wave & 1, wn = wave >> 1;
  const int nclass = a.transposed ? 4 : 1;
  const int cls = blockIdx.z % nclass, split = blockIdx.z / nclass;
  int py = 0, px = 0, Hc = a.Ho, Wc = a.Wo;
  if (a.transposed) {
    py = cls >> 1;
    px = cls & 1;
    Hc = (a.Ho - py + 1) >> 1;
    Wc = (a.Wo - px + 1) >> 1;
  }
  const int HWc = Hc * Wc;
  const int Mtot = a.B * HWc;
  const int mblk = blockIdx.x * V2M;
  if (mblk >= Mtot) return;  // whole workgroup
  const int n0 = blockIdx.y * V2N;
  const bf16_t* xp = (const bf16_t*)a.x;
  const bf16_t* wp = (const bf16_t*)a.w;
  const int krow = 9 * a.C;  // one code's packed row (elements)
  // ---- tap table (uniform): origin-relative source offset of each tap, in pixels
  if (tid == 0) {
    int n = 0, base = 0, t = 0;
    const int nchunk = a.C / 32;
    for (int ky = 0; ky < 3; ++ky)
      for (int kx = 0; kx < 3; ++kx) {
        int dy = ky, dx = kx;  // forward: origin (2oy-1, 2ox-1)
        if (a.transposed) {
          if (((py + 1 - ky) & 1) || ((px + 1 - kx) & 1)) continue;
          dy = (py + 1 - ky) >> 1;  // dX: origin (i, j) of the parity-class grid
          dx = (px + 1 - kx) >> 1;
        }
        uint32_t msk = a.tile_codes[((long long)cls * gridDim.x + blockIdx.x) * 9 + t];
        ttap[t] = ky * 3 + kx;
        tdelta[t] = dy * a.Wi + dx;
        tfirst[t] = (uint8_t)n;
        tbase[t] = base;
        const int cnt = __popc(msk);
        tcnt[t] = (uint8_t)cnt;
        base += cnt * nchunk;
        while (msk) {
          const int k = __ffs(msk) - 1;
          msk &= msk - 1u;
          tcl[n++] = (uint8_t)k;
        }
        ++t;
      }
    for (int q = t; q < 9; ++q) tcnt[q] = 0;
    tbase[t] = base;
    for (int q = t + 1; q < 10; ++q) tbase[q] = base;
  }
  // ---- rows owned by this lane: m = mblk + wm*64 + 16*mi + r.  Per row: origin pixel index,
  // 9-bit mask of in-bounds taps and the 4-bit code each tap meets (SRC: source pixel's code;
  // DST: the row's own code).  Taps are indexed by position t in the tap table.
  int rorg[4];
  uint32_t rvalid[4], rc_lo[4], rc_hi[4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int m = mblk + wm * 64 + 16 * mi + r;
    rvalid[mi] = 0u;
    rc_lo[mi] = rc_hi[mi] = 0u;
    rorg[mi] = 0;
    if (m < Mtot) {
      const int b = m / HWc, rem = m % HWc, i = rem / Wc, j = rem % Wc;
      int t = 0;
      if (a.transposed) {
        const int oy = 2 * i + py, ox = 2 * j + px;
        const uint32_t rc = a.code[((long long)b * a.Ho + oy) * a.Wo + ox];
        rorg[mi] = (b * a.Hi + i) * a.Wi + j;
        for (int ky = 0; ky < 3; ++ky)
          for (int kx = 0; kx < 3; ++kx) {
            if (((py + 1 - ky) & 1) || ((px + 1 - kx) & 1)) continue;
            const int iy = i + ((py + 1 - ky) >> 1), ix = j + ((px + 1 - kx) >> 1);
            if (iy < a.Hi && ix < a.Wi) {
              rvalid[mi] |= 1u << t;
              if (t < 8) rc_lo[mi] |= rc << (4 * t); else rc_hi[mi] |= rc;
            }
            ++t;
          }
      } else {
        const int oy = i, ox = j;
        rorg[mi] = (b * a.Hi + 2 * oy - 1) * a.Wi + 2 * ox - 1;
        const uint8_t* cb = a.code + (long long)b * a.Hi * a.Wi;
        for (int ky = 0; ky < 3; ++ky)
          for (int kx = 0; kx < 3; ++kx) {
            const int iy = 2 * oy - 1 + ky, ix = 2 * ox - 1 + kx;
            if (iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi) {
              const uint32_t c = cb[iy * a.Wi + ix];
              rvalid[mi] |= 1u << t;
              if (t < 8) rc_lo[mi] |= c << (4 * t); else rc_hi[mi] |= c;
            }
            ++t;
          }
      }
    }
  }
  __syncthreads();
  const int nchunk = a.C / 32;
  const int T = tbase[9];
  const int s0 = (int)((long long)split * T / a.ksplit), s1 = (int)((long long)(split + 1) * T / a.ksplit);
  // B staging rows: thread -> pieces tid, tid + 256 (row id>>2, 16-byte chunk id&3)
  int boff[2];
  bool bok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = tid + 256 * i, n = n0 + (id >> 2);
    bok[i] = n < a.N;
    boff[i] = (bok[i] ? n : 0) * krow + 8 * (id & 3);
  }
  uint4 rbv[2];
  // step state (wave-uniform): tap position, chunk, code index within the tap
  int st_t = 0, st_ch = 0, st_ci = 0;
  auto seek = [&](int st) {
    int t = 0;
    while (st >= tbase[t + 1]) ++t;
    const int rel = st - tbase[t], cnt = tcnt[t];
    st_t = t;
    st_ch = rel / cnt;
    st_ci = rel - st_ch * cnt;
  };
  auto advance = [&]() {
    if (++st_ci == tcnt[st_t]) {
      st_ci = 0;
      if (++st_ch == nchunk) {
        st_ch = 0;
        do ++st_t; while (st_t < 9 && tcnt[st_t] == 0);
      }
    }
  };
  auto bload = [&](int t, int ch, int code) {
    const int koff = __builtin_amdgcn_readfirstlane(code * a.N * krow + ttap[t] * a.C + ch * 32);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      rbv[i] = bok[i] ? *reinterpret_cast<const uint4*>(wp + koff + boff[i]) : make_uint4(0u, 0u, 0u, 0u);
  };
  auto bstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + 256 * i;
      *reinterpret_cast<uint4*>(&sB[buf][cm_slot(id >> 2, id & 3)]) = rbv[i];
    }
  };
  auto aload = [&](int t, int ch, Frag<bf16_t>* af, uint32_t& rq) {
    const int d = __builtin_amdgcn_readfirstlane(tdelta[t]);
    const int coff = ch * 32 + 8 * g;
    rq = 0u;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const bool v = (rvalid[mi] >> t) & 1u;
      const int pix = v ? rorg[mi] + d : 0;
      af[mi].load(xp + (long long)pix * a.C + coff);
      const uint32_t c = v ? ((t < 8 ? rc_lo[mi] >> (4 * t) : rc_hi[mi]) & 15u) : 0xffu;
      rq |= c << (8 * mi);
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int nj = 0; nj < 4; ++nj) acc[mi][nj] = f32x4{0.f, 0.f, 0.f, 0.f};
  int ccode = 0;
  Frag<bf16_t> Ac[4], An[4];
  uint32_t rqc = 0u, rqn = 0u;  // byte mi: code met by row mi at the step's tap (0xff: none)
  if (s0 < s1) {
    seek(s0);
    ccode = tcl[tfirst[st_t] + st_ci];
    bload(st_t, st_ch, ccode);
    aload(st_t, st_ch, Ac, rqc);
    bstore(0);
  }
  lds_barrier();
  for (int st = s0; st < s1; ++st) {
    int ncode = 0;
    bool fresh = false;
    if (st + 1 < s1) {  // prefetch step st+1: B always, A rows when its (tap, chunk) is new
      advance();
      ncode = tcl[tfirst[st_t] + st_ci];
      bload(st_t, st_ch, ncode);
      fresh = st_ci == 0;
      if (fresh) aload(st_t, st_ch, An, rqn);
    }
    Frag<bf16_t> As[4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      As[mi] = Ac[mi];
      As[mi].select(((rqc >> (8 * mi)) & 0xffu) == (uint32_t)ccode);
    }
    const int buf = (st - s0) & 1;
#pragma unroll
    for (int nj = 0; nj < 4; ++nj) {
      Frag<bf16_t> bf;
      bf.v = *reinterpret_cast<const uint4*>(&sB[buf][cm_slot(wn * 64 + 16 * nj + r, g)]);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) mma(acc[mi][nj], As[mi], bf);
    }
    if (st + 1 < s1) bstore(buf ^ 1);
    if (fresh) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) Ac[mi] = An[mi];
      rqc = rqn;
    }
    ccode = ncode;
    lds_barrier();
  }
  if (a.ksplit > 1) {  // split-K: f32 slab [split][class][m][N], reduced by k_splitk_finish
    // slab rows: [split][class (in order)][m] = [split][B*Ho*Wo] in total
    long long coff = 0;
    for (int c = 0; c < cls; ++c)
      coff += (long long)a.B * ((a.Ho - (c >> 1) + 1) >> 1) * ((a.Wo - (c & 1) + 1) >> 1);
    float* slab = a.partial + ((long long)split * a.B * a.Ho * a.Wo + coff) * a.N;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int m = mblk + wm * 64 + 16 * mi + 4 * g + reg;
        if (m >= Mtot) continue;
#pragma unroll
        for (int nj = 0; nj < 4; ++nj) {
          const int n = n0 + wn * 64 + 16 * nj + r;
          if (n < a.N) slab[(long long)m * a.N + n] = acc[mi][nj][reg];
        }
      }
    return;
  }
  // ---- epilogue (same contract as k_conv_igemm)
  const bf16_t* res = (const bf16_t*)a.residual;
  bf16_t* onchw = (bf16_t*)a.out_nchw;
  bf16_t* onhwc = (bf16_t*)a.out_nhwc;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const long long m = mblk + wm * 64 + 16 * mi + 4 * g + reg;
      if (m >= Mtot) continue;
      const int b = (int)(m / HWc);
      const int rem = (int)(m % HWc);
      const int i = rem / Wc, j = rem % Wc;
      const int oy = a.transposed ? 2 * i + py : i;
      const int ox = a.transposed ? 2 * j + px : j;
      const int nmask = a.info ? a.info[b].n_masks : 0;
#pragma unroll
      for (int nj = 0; nj < 4; ++nj) {
        const int n = n0 + wn * 64 + 16 * nj + r;
        if (n >= a.N) continue;
        float v = acc[mi][nj][reg];
        if (a.bias4) {
          float bs = 0.f;
          for (int sb = 0; sb < nmask; ++sb) bs += a.bias4[sb * a.N + n];
          v += bs;
        }
        const long long o_nchw = (((long long)b * a.N + n) * a.Ho + oy) * a.Wo + ox;
        if (res) v = bf16_to_f32(res[o_nchw]) + v;
        const bf16_t tv = f32_to_bf16(v);
        if (onchw) onchw[o_nchw] = tv;
        if (onhwc) onhwc[(((long long)b * a.Ho + oy) * a.Wo + ox) * a.N + n] = tv;
      }
    }
  }
}

// split-K finish: sum the slabs in fixed order, add biases / residual, write NCHW (+NHWC) bf16.
// Slabs are [split][class][m][N] in k_conv_codes' row order (m over the batch x parity-class
// grid).  One block per 32 pixels x 32 channels, transposed through LDS so both stores coalesce.
__global__ __launch_bounds__(256) void k_splitk_finish(ConvArgs a) {
  __shared__ float tile[32][33];
  const long long P = (long long)a.B * a.Ho * a.Wo;
  const long long p0 = (long long)blockIdx.x * 32;
  const int n0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  const long long HW = (long long)a.Ho * a.Wo;
  for (int k = ty; k < 32; k += 8) {  // k: pixel within tile, tx: channel
    const long long p = p0 + k;
    const int n = n0 + tx;
    float v = 0.f;
    if (p < P && n < a.N) {
      const int b = (int)(p / HW), rem = (int)(p % HW), oy = rem / a.Wo, ox = rem % a.Wo;
      int cls = 0, Hc = a.Ho, Wc = a.Wo, i = oy, j = ox;
      if (a.transposed) {
        cls = (oy & 1) * 2 + (ox & 1);
        Hc = (a.Ho - (oy & 1) + 1) >> 1;
        Wc = (a.Wo - (ox & 1) + 1) >> 1;
        i = oy >> 1;
        j = ox >> 1;
      }
      const long long m = ((long long)b * Hc + i) * Wc + j;
      // class c's slab offset: sum of the row counts of classes < c
      long long coff = 0;
      for (int c = 0; c < cls; ++c) {
        const int hc = (a.Ho - (c >> 1) + 1) >> 1, wc = (a.Wo - (c & 1) + 1) >> 1;
        coff += (long long)a.B * hc * wc;
      }
      for (int sp = 0; sp < a.ksplit; ++sp) v += a.partial[((long long)sp * P + coff + m) * a.N + n];
      if (a.bias4) {
        const int nm = a.info[b].n_masks;
        float bs = 0.f;
        for (int q = 0; q < nm; ++q) bs += a.bias4[q * a.N + n];
        v += bs;
      }
      if (a.residual) v += bf16_to_f32(((const bf16_t*)a.residual)[((long long)b * a.N + n) * HW + rem]);
      if (a.out_nhwc) ((bf16_t*)a.out_nhwc)[p * a.N + n] = f32_to_bf16(v);
    }
    tile[k][tx] = v;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {  // k: channel within tile, tx: pixel
    const long long p = p0 + tx;
    const int n = n0 + k;
    if (p < P && n < a.N && a.out_nchw) {
      const int b = (int)(p / HW);
      ((bf16_t*)a.out_nchw)[((long long)b * a.N + n) * HW + (p % HW)] = f32_to_bf16(tile[tx][k]);
    }
  }
}

// split-K factor of the bf16 v2 path: enough workgroups to cover the chip ~3x
int v2_ksplit(long long Mmax, int N, int nclass, int C, int transposed) {
  const long long wgs = (long long)ceil_div(Mmax, V2M) * ceil_div(N, V2N) * nclass;
  const int tc_min = (transposed ? 1 : 9) * (C / 32);
  return (int)std::max<long long>(1, std::min<long long>(std::min(tc_min, 8), ceil_div(768, wgs)));
}
long long conv_mmax(const ConvArgs& a) {
  return a.transposed ? (long long)a.B * ((a.Ho + 1) / 2) * ((a.Wo + 1) / 2) : (long long)a.B * a.Ho * a.Wo;
}
size_t v2_partial_bytes(const ConvArgs& a) {
  const int ks = v2_ksplit(conv_mmax(a), a.N, a.transposed ? 4 : 1, a.C, a.transposed);
  return ks > 1 ? align256((size_t)ks * a.B * a.Ho * a.Wo * a.N * sizeof(float)) : 0;
}
size_t tile_codes_bytes(const ConvArgs& a) {
  return align256((size_t)(a.transposed ? 4 : 1) * ceil_div(conv_mmax(a), V2M) * 9 * sizeof(uint16_t));
}

template <typename T>
int launch_conv(const ConvArgs& a, hipStream_t s) {
  TimerScope ts(a.transposed ? "dsam_dx" : "dsam_fwd", s);
  int nclass = a.transposed ? 4 : 1;
  long long Mmax = (long long)a.B * a.Ho * a.Wo;
  if (a.transposed) Mmax = (long long)a.B * ((a.Ho + 1) / 2) * ((a.Wo + 1) / 2);
  if constexpr (sizeof(T) == 2) {
    RGBD_REQUIRE(a.C % 32 == 0 && a.N % 32 == 0, RGBD_E_SHAPE);  // code-merged bf16 path only
    {
      ConvArgs b = a;
      b.ksplit = v2_ksplit(Mmax, a.N, nclass, a.C, a.transposed);
      // workspace: [split-K slabs | tile code sets]
      b.tile_codes = (uint16_t*)((char*)a.partial + v2_partial_bytes(a));
      k_conv_tile_codes<<<dim3(ceil_div(Mmax, V2M), 1, nclass), V2M, 0, s>>>(b);
      dim3 grid2(ceil_div(Mmax, V2M), ceil_div(a.N, V2N), nclass * b.ksplit);
      k_conv_codes<<<grid2, 256, 0, s>>>(b);
      if (b.ksplit > 1) {
        dim3 g3(ceil_div((long long)a.B * a.Ho * a.Wo, 32), ceil_div(a.N, 32));
        k_splitk_finish<<<g3, 256, 0, s>>>(b);
      }
      RGBD_CHECK_LAUNCH();
      return RGBD_OK;
    }
  }
  dim3 grid(ceil_div(Mmax, BM), ceil_div(a.N, BN), nclass);
  k_conv_igemm<T><<<grid, 256, 0, s>>>(a);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int dsam_wgrad_splits_codes(int B, int Cin, int Cout) {
  // ~4 codes present per batch is typical; aim at ~3 live workgroups per CU
  const long long tiles = (long long)ceil_div(9ll * Cin, WG_KK) * ceil_div(Cout, WG_O) * 4;
  return (int)std::max<long long>(1, std::min<long long>(B, ceil_div(768, tiles)));
}
int dsam_wgrad_splits(int B, int Cin, int Cout) {
  const long long tiles = (long long)ceil_div(45ll * Cin, WG_KK) * ceil_div(Cout, WG_O);
  int sp = (int)std::min<long long>(B, std::max<long long>(1, ceil_div(1024, tiles)));
  return sp < 1 ? 1 : sp;
}

}  // namespace

extern "C" {

const char* rgbd_version(void) { return "rgbd_hip 0.1.0 (gfx950)"; }

int rgbd_nchw_to_nhwc(int dtype, const void* src, void* dst, int B, int C, int H, int W, void* stream) {
  RGBD_REQUIRE(src && dst && B > 0 && C > 0 && H > 0 && W > 0, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(ceil_div((long long)H * W, 32), ceil_div(C, 32), B);
  if (dtype == RGBD_F32)
    k_nchw_to_nhwc<float><<<grid, 256, 0, s>>>((const float*)src, (float*)dst, C, H * W);
  else if (dtype == RGBD_BF16)
    k_nchw_to_nhwc<bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)src, (bf16_t*)dst, C, H * W);
  else
    return RGBD_E_DTYPE;
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

long long rgbd_dsam_packed_elems(int dtype, int Cin, int Cout) {
  if (Cin <= 0 || Cout <= 0) return 0;
  if (dtype == RGBD_F32) return 45ll * Cin * Cout;
  if (dtype == RGBD_BF16) return 144ll * Cin * Cout;
  return 0;
}

int rgbd_dsam_pack_weights(int dtype, const float* conv_w, const float* proj_w, int Cin, int Cout,
                           void* wfwd, void* wbwd, void* stream) {
  RGBD_REQUIRE(conv_w && proj_w && (wfwd || wbwd) && Cin > 0 && Cout > 0, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_F32) {
    const int nb = (int)std::min<long long>(ceil_div(45ll * Cin * Cout, 256), 4096);
    k_pack_dsam<float><<<nb, 256, 0, s>>>(conv_w, proj_w, Cin, Cout, (float*)wfwd, (float*)wbwd);
  } else if (dtype == RGBD_BF16) {
    RGBD_REQUIRE(Cin % 32 == 0 && Cout % 32 == 0, RGBD_E_SHAPE);
    const int nb = (int)std::min<long long>(ceil_div(9ll * Cin * Cout, 256), 4096);
    k_pack_dsam_codes<<<nb, 256, 0, s>>>(conv_w, proj_w, Cin, Cout, (bf16_t*)wfwd, (bf16_t*)wbwd);
  } else {
    return RGBD_E_DTYPE;
  }
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

static ConvArgs fwd_args(int B, int Cin, int h, int w, int Cout) {
  ConvArgs a = {};
  a.B = B; a.Hi = h; a.Wi = w; a.C = Cin;
  a.Ho = (h + 1) / 2; a.Wo = (w + 1) / 2; a.N = Cout;
  a.KH = 3; a.KW = 3; a.stride = 2; a.pad = 1;
  a.nseg = 5; a.mask_mode = MASK_SRC; a.transposed = 0; a.ksplit = 1;
  return a;
}
static ConvArgs dx_args(int B, int Cin, int h, int w, int Cout) {
  ConvArgs a = {};
  a.B = B; a.Hi = (h + 1) / 2; a.Wi = (w + 1) / 2; a.C = Cout;
  a.Ho = h; a.Wo = w; a.N = Cin;
  a.KH = 3; a.KW = 3; a.stride = 2; a.pad = 1;
  a.nseg = 5; a.mask_mode = MASK_DST; a.transposed = 1; a.ksplit = 1;
  return a;
}

size_t rgbd_dsam_conv_workspace_size(int dtype, int B, int Cin, int h, int w, int Cout) {
  if (dtype != RGBD_BF16 || B <= 0 || h <= 0 || w <= 0) return 256;
  const ConvArgs f = fwd_args(B, Cin, h, w, Cout), d = dx_args(B, Cin, h, w, Cout);
  return std::max<size_t>(256, std::max(v2_partial_bytes(f) + tile_codes_bytes(f),
                                        v2_partial_bytes(d) + tile_codes_bytes(d)));
}

int rgbd_dsam_fwd(int dtype, const void* x_nhwc, const uint8_t* code, const rgbd_decomp_info* info,
                  int B, int Cin, int h, int w, int Cout, const void* wfwd, const float* bias,
                  const void* residual, void* out_nchw, void* out_nhwc, void* ws, void* stream) {
  RGBD_REQUIRE(x_nhwc && code && info && wfwd && bias && (out_nchw || out_nhwc), RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && h > 0 && w > 0 && Cout > 0 && Cin > 0, RGBD_E_ARG);
  RGBD_REQUIRE(Cin % 8 == 0, RGBD_E_SHAPE);
  ConvArgs a = fwd_args(B, Cin, h, w, Cout);
  a.x = x_nhwc; a.code = code; a.w = wfwd;
  a.bias4 = bias; a.info = info; a.residual = residual; a.out_nchw = out_nchw; a.out_nhwc = out_nhwc;
  a.partial = (float*)ws;
  RGBD_REQUIRE(ws || dtype != RGBD_BF16, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_F32) return launch_conv<float>(a, s);
  if (dtype == RGBD_BF16) return launch_conv<bf16_t>(a, s);
  return RGBD_E_DTYPE;
}

int rgbd_dsam_bwd_data(int dtype, const void* gout_nhwc, const uint8_t* code, int B, int Cin, int h,
                       int w, int Cout, const void* wbwd, const void* gin_nchw, void* dx_nchw,
                       void* dx_nhwc, void* ws, void* stream) {
  RGBD_REQUIRE(gout_nhwc && code && wbwd && (dx_nchw || dx_nhwc), RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && h > 0 && w > 0 && Cout > 0 && Cin > 0, RGBD_E_ARG);
  RGBD_REQUIRE(Cout % 8 == 0, RGBD_E_SHAPE);
  ConvArgs a = dx_args(B, Cin, h, w, Cout);
  a.x = gout_nhwc; a.code = code; a.w = wbwd;
  a.residual = gin_nchw; a.out_nchw = dx_nchw; a.out_nhwc = dx_nhwc;
  a.partial = (float*)ws;
  RGBD_REQUIRE(ws || dtype != RGBD_BF16, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_F32) return launch_conv<float>(a, s);
  if (dtype == RGBD_BF16) return launch_conv<bf16_t>(a, s);
  return RGBD_E_DTYPE;
}

// bf16 workspace: [splits][16 codes][Cout][9 Cin] f32 partials | [B] f32 x Cout channel sums |
// presence table [B][chunks] u16 | global code mask u32
struct WgradWs {
  size_t partial, csum, pres, gmask, total;
};
static WgradWs wgrad_ws(int dtype, int B, int Cin, int h, int w, int Cout) {
  WgradWs o;
  size_t off = 0;
  const int hwo = ((h + 1) / 2) * ((w + 1) / 2);
  const size_t part = dtype == RGBD_BF16 ? (size_t)dsam_wgrad_splits_codes(B, Cin, Cout) * 16 * Cout * 9 * Cin
                                         : (size_t)dsam_wgrad_splits(B, Cin, Cout) * Cout * 45 * Cin;
  o.partial = off;
  off += align256(sizeof(float) * part);
  o.csum = off;
  off += align256(sizeof(float) * (size_t)B * Cout);
  o.pres = off;
  off += align256(sizeof(uint16_t) * (size_t)B * ((hwo + PXC - 1) / PXC));
  o.gmask = off;
  off += 256;
  o.total = off;
  return o;
}

size_t rgbd_dsam_bwd_weight_workspace_size(int dtype, int B, int Cin, int h, int w, int Cout) {
  if (B <= 0 || h <= 0 || w <= 0 || Cin <= 0 || Cout <= 0) return 256;
  return wgrad_ws(dtype, B, Cin, h, w, Cout).total;
}

int rgbd_dsam_bwd_weight(int dtype, const void* gout_nchw, const void* x_nhwc, const uint8_t* code,
                         const rgbd_decomp_info* info, int B, int Cin, int h, int w, int Cout,
                         float* dconv_w, float* dproj_w, float* dbias, void* ws, void* stream) {
  RGBD_REQUIRE(gout_nchw && x_nhwc && code && info && dconv_w && dproj_w && dbias && ws, RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && h > 0 && w > 0 && Cout > 0 && Cin > 0, RGBD_E_ARG);
  RGBD_REQUIRE(Cin % 8 == 0, RGBD_E_SHAPE);
  hipStream_t s = (hipStream_t)stream;
  const WgradWs L = wgrad_ws(dtype, B, Cin, h, w, Cout);
  float* partial = (float*)((char*)ws + L.partial);
  float* csum = (float*)((char*)ws + L.csum);
  TimerScope ts("dsam_wgrad", s);
  const int hwo = ((h + 1) / 2) * ((w + 1) / 2);
  if (dtype == RGBD_F32) {
    const int sp = dsam_wgrad_splits(B, Cin, Cout);
    dim3 grid(ceil_div(45ll * Cin, 64), ceil_div(Cout, 64), sp);
    k_dsam_wgrad<float><<<grid, 256, 0, s>>>((const float*)gout_nchw, (const float*)x_nhwc, code, B, Cin, h, w,
                                             Cout, sp, partial);
    k_chan_sum<float><<<B * Cout, 256, 0, s>>>((const float*)gout_nchw, hwo, csum);
    const long long total = 45ll * Cin * Cout;
    k_dsam_wgrad_final<<<(int)std::min<long long>(ceil_div(total, 256), 4096), 256, 0, s>>>(
        partial, sp, Cin, Cout, dconv_w, dproj_w);
  } else if (dtype == RGBD_BF16) {
    RGBD_REQUIRE(Cin % 32 == 0 && Cout % 32 == 0, RGBD_E_SHAPE);
    const int spc = dsam_wgrad_splits_codes(B, Cin, Cout);
    uint16_t* pres = (uint16_t*)((char*)ws + L.pres);
    uint32_t* gmask = (uint32_t*)((char*)ws + L.gmask);
    const hipError_t me = hipMemsetAsync(gmask, 0, sizeof(uint32_t), s);
    if (me != hipSuccess) return (int)me;
    const long long nthr = (long long)B * ((hwo + PXC - 1) / PXC) * 32;
    k_code_presence<<<(int)ceil_div(nthr, 256), 256, 0, s>>>(code, B, h, w, pres, gmask);
    dim3 g2(ceil_div(9ll * Cin, WG_KK), ceil_div(Cout, WG_O), spc * 16);
    k_dsam_wgrad_bf16<<<g2, 256, 0, s>>>((const bf16_t*)gout_nchw, (const bf16_t*)x_nhwc, code, pres, gmask, B,
                                         Cin, h, w, Cout, spc, partial);
    k_chan_sum<bf16_t><<<B * Cout, 256, 0, s>>>((const bf16_t*)gout_nchw, hwo, csum);
    const long long total = 9ll * Cin * Cout;
    k_dsam_wgrad_combine<<<(int)std::min<long long>(ceil_div(total, 256), 4096), 256, 0, s>>>(
        partial, spc, gmask, Cin, Cout, dconv_w, dproj_w);
  } else {
    return RGBD_E_DTYPE;
  }
  k_dsam_bias_grad<<<ceil_div(4 * Cout, 256), 256, 0, s>>>(csum, info, B, Cout, dbias);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
