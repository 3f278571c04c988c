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

// bf16 dW: X tile staged [px][kk] from NHWC with 16-byte loads, read back transposed with
// ds_read_b64_tr_b16 (gfx950) as the MFMA B operand (8 consecutive pixels per lane); the A
// operand (G^T, 8 consecutive pixels of one channel) is a direct 16-byte load from NCHW.
constexpr int WG_KK = 128, WG_O = 64, PXC = 32, XPAD = 136;
typedef __attribute__((ext_vector_type(4))) short v4s;

__global__ __launch_bounds__(256) void k_dsam_wgrad_bf16(const bf16_t* __restrict__ gout, const bf16_t* __restrict__ x,
                                                         const uint8_t* __restrict__ code, int B, int Cin, int h,
                                                         int w, int Cout, int splits, float* __restrict__ partial) {
  __shared__ __attribute__((aligned(16))) bf16_t Xs[2][PXC][XPAD];
  const int ho = (h + 1) / 2, wo = (w + 1) / 2;
  const int hwo = ho * wo;
  const int KK = 45 * Cin;
  const int kk0 = blockIdx.x * WG_KK, o0 = blockIdx.y * WG_O, z = blockIdx.z;
  const int b0 = (int)((long long)z * B / splits), b1 = (int)((long long)(z + 1) * B / splits);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  // staging role: pixel row spx, two 8-channel chunks at kk0 + 16*skg + 8*q
  const int spx = threadIdx.x >> 3, skg = threadIdx.x & 7;
  int s_seg[2], s_ky[2], s_kx[2], s_c[2];
  bool s_ok[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int kk = kk0 + 16 * skg + 8 * q;
    s_ok[q] = kk < KK;
    const int k2 = s_ok[q] ? kk : 0;
    s_seg[q] = k2 / (9 * Cin);
    const int tap = (k2 / Cin) % 9;
    s_ky[q] = tap / 3;
    s_kx[q] = tap % 3;
    s_c[q] = k2 % Cin;
  }
  int staged_any = 0;  // does the staged chunk hold any unmasked element?
  auto stage = [&](int buf, int b, int p0) {
    const int p = p0 + spx;
    const int oy = p / wo, ox = p % wo;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int iy = 2 * oy - 1 + s_ky[q], ix = 2 * ox - 1 + s_kx[q];
      bool ok = s_ok[q] && p < hwo && iy >= 0 && iy < h && ix >= 0 && ix < w;
      const long long pix = ((long long)b * h + iy) * w + ix;
      if (ok && s_seg[q] < 4) ok = (code[pix] >> s_seg[q]) & 1u;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (ok) v = *reinterpret_cast<const uint4*>(x + pix * Cin + s_c[q]);
      staged_any |= ok ? 1 : 0;
      *reinterpret_cast<uint4*>(&Xs[buf][spx][16 * skg + 8 * q]) = v;
    }
  };
  f32x4 acc[4][2];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj) acc[mi][nj] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nchunk = (hwo + PXC - 1) / PXC;
  const int total = (b1 - b0) * nchunk;
  if (total > 0) stage(0, b0, 0);
  int live = __syncthreads_or(staged_any);
  for (int it = 0; it < total; ++it) {
    const int buf = it & 1;
    const int b = b0 + it / nchunk, p0 = (it % nchunk) * PXC;
    staged_any = 0;
    if (it + 1 < total) stage(buf ^ 1, b0 + (it + 1) / nchunk, ((it + 1) % nchunk) * PXC);
    if (!live) {  // every im2col element of this chunk is masked out: contribution is zero
      live = __syncthreads_or(staged_any);
      continue;
    }
    // A: G^T rows o, 8 consecutive pixels
    Frag<bf16_t> af[4];
    const int pa = p0 + 8 * g;
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
    live = __syncthreads_or(staged_any);
  }
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int o = o0 + 16 * mi + 4 * g + reg;
#pragma unroll
      for (int nj = 0; nj < 2; ++nj) {
        const int c = kk0 + wave * 32 + 16 * nj + r;
        if (o < Cout && c < KK) partial[((long long)z * Cout + o) * KK + c] = acc[mi][nj][reg];
      }
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

// ----------------------------------------------------------------------- bf16 v2
// Workgroup tile 128 output pixels (flattened over batch x grid, or over one stride-2 parity
// class for dX) x 128 output channels; 4 waves as 2x2, wave tile 64 px x 64 ch (4x4 MFMA).
// A (im2col rows) is gathered straight from NHWC global memory, 8 channels (16 B) per lane,
// once per (tap, 32-ch chunk) and re-used by every live segment; B (packed weights) is staged
// per (tap, chunk, segment) step through a double-buffered LDS tile shared by the 4 waves.
// A segment whose mask bit is absent from every pixel the workgroup reads is skipped for
// the whole K loop (exact: its contribution is zero).
constexpr int V2M = 128, V2N = 128, V2BROW = 40;  // 80-byte LDS rows (conflict-free b128 reads)

__global__ __launch_bounds__(256) void k_conv_igemm_v2(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t sB[2][V2N][V2BROW];
  __shared__ uint32_t seg_or;
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
  const long long HWc = (long long)Hc * Wc;
  const long long Mtot = (long long)a.B * HWc;
  const long long mblk = (long long)blockIdx.x * V2M;
  if (mblk >= Mtot) return;  // whole workgroup
  const int n0 = blockIdx.y * V2N;
  const bf16_t* xp = (const bf16_t*)a.x;
  const bf16_t* wp = (const bf16_t*)a.w;
  const long long ktot = 5ll * 9 * a.C;
  // rows owned by this lane: m = mblk + wm*64 + 16*mi + r
  int rb[4], roy[4], rox[4];
  bool rvalid[4];
  uint32_t rcode[4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const long long m = mblk + wm * 64 + 16 * mi + r;
    rvalid[mi] = m < Mtot;
    const long long mm = rvalid[mi] ? m : 0;
    rb[mi] = (int)(mm / HWc);
    const int rem = (int)(mm % HWc);
    const int i = rem / Wc, j = rem % Wc;
    roy[mi] = a.transposed ? 2 * i + py : i;
    rox[mi] = a.transposed ? 2 * j + px : j;
    rcode[mi] = (a.mask_mode == MASK_DST && rvalid[mi])
                    ? a.code[((long long)rb[mi] * a.Ho + roy[mi]) * a.Wo + rox[mi]]
                    : 0u;
  }
  // ---- live segments of the workgroup (OR of every code any of its rows reads)
  if (tid == 0) seg_or = 0u;
  __syncthreads();
  {
    uint32_t o = 0u;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      if (!rvalid[mi]) continue;
      if (a.mask_mode == MASK_DST) {
        o |= rcode[mi];
      } else {
        for (int t = 0; t < 9; ++t) {
          const int iy = roy[mi] * 2 - 1 + t / 3, ix = rox[mi] * 2 - 1 + t % 3;
          if (iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi)
            o |= a.code[((long long)rb[mi] * a.Hi + iy) * a.Wi + ix];
        }
      }
    }
    if (o) atomicOr(&seg_or, o);
  }
  __syncthreads();
  const uint32_t live = (seg_or & 0xfu) | 0x10u;  // segment 4 (projection) always live
  int segs[5], nseg = 0;
  for (int sgi = 0; sgi < 5; ++sgi)
    if ((live >> sgi) & 1u) segs[nseg++] = sgi;
  // ---- K steps = (tap, chunk) x live segments
  int taps[9], ntap = 0;
  for (int ky = 0; ky < 3; ++ky)
    for (int kx = 0; kx < 3; ++kx) {
      if (a.transposed && (((py + 1 - ky) & 1) || ((px + 1 - kx) & 1))) continue;
      taps[ntap++] = ky * 3 + kx;
    }
  const int nchunk = a.C / 32;
  // this split's (tap, chunk) range
  const int tc_total = ntap * nchunk;
  const int tc0 = (int)((long long)split * tc_total / a.ksplit), tc1 = (int)((long long)(split + 1) * tc_total / a.ksplit);
  const int nsteps = (tc1 - tc0) * nseg;
  // B staging: 128 rows (n) x 4 pieces of 8 channels; thread -> pieces tid, tid + 256
  uint4 rbv[2];
#define V2_BLOAD(STEP)                                                                            \
  {                                                                                               \
    const int st_ = (STEP);                                                                       \
    const int sg_ = segs[st_ % nseg], tc_ = tc0 + st_ / nseg;                                     \
    const int tap_ = taps[tc_ / nchunk], ch_ = tc_ % nchunk;                                      \
    const long long koff_ = ((long long)sg_ * 9 + tap_) * a.C + ch_ * 32;                         \
    _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                               \
      const int id = tid + 256 * i, n = n0 + (id >> 2);                                          \
      rbv[i] = n < a.N ? *reinterpret_cast<const uint4*>(wp + (long long)n * ktot + koff_ + 8 * (id & 3)) \
                       : make_uint4(0u, 0u, 0u, 0u);                                              \
    }                                                                                             \
  }
#define V2_BSTORE(BUF)                                                                    \
  _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                         \
    const int id = tid + 256 * i;                                                         \
    *reinterpret_cast<uint4*>(&sB[BUF][id >> 2][8 * (id & 3)]) = rbv[i];                  \
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int nj = 0; nj < 4; ++nj) acc[mi][nj] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nsteps > 0) {
    V2_BLOAD(0);
    V2_BSTORE(0);
  }
  lds_barrier();
  Frag<bf16_t> A[4];
  uint32_t scode[4];
  for (int st = 0; st < nsteps; ++st) {
    const int sgi = st % nseg, tc = tc0 + st / nseg;
    const int seg = segs[sgi];
    if (st + 1 < nsteps) V2_BLOAD(st + 1);
    if (sgi == 0) {  // new (tap, chunk): gather the A rows
      const int tap = taps[tc / nchunk], ch = tc % nchunk;
      const int ky = tap / 3, kx = tap % 3;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        int iy, ix;
        if (a.transposed) {
          iy = (roy[mi] + 1 - ky) >> 1;
          ix = (rox[mi] + 1 - kx) >> 1;
        } else {
          iy = roy[mi] * 2 - 1 + ky;
          ix = rox[mi] * 2 - 1 + kx;
        }
        const bool inb = rvalid[mi] && iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi;
        const long long pix = inb ? ((long long)rb[mi] * a.Hi + iy) * a.Wi + ix : 0;
        if (inb)
          A[mi].load(xp + pix * a.C + ch * 32 + 8 * g);
        else
          A[mi].zero();
        scode[mi] = a.mask_mode == MASK_SRC ? (inb ? a.code[pix] : 0u) : rcode[mi];
      }
    }
    Frag<bf16_t> As[4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      As[mi] = A[mi];
      if (seg < 4) As[mi].select((scode[mi] >> seg) & 1u);
    }
#pragma unroll
    for (int nj = 0; nj < 4; ++nj) {
      Frag<bf16_t> bf;
      bf.v = *reinterpret_cast<const uint4*>(&sB[st & 1][wn * 64 + 16 * nj + r][8 * g]);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) mma(acc[mi][nj], As[mi], bf);
    }
    if (st + 1 < nsteps) V2_BSTORE((st + 1) & 1);
    lds_barrier();
  }
#undef V2_BLOAD
#undef V2_BSTORE
  if (a.ksplit > 1) {  // split-K: f32 slab, reduced + finished by k_splitk_finish
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const long long m = mblk + wm * 64 + 16 * mi + 4 * g + reg;
        if (m >= Mtot) continue;
        const int b = (int)(m / HWc);
        const int rem = (int)(m % HWc);
        const int i = rem / Wc, j = rem % Wc;
        const int oy = a.transposed ? 2 * i + py : i;
        const int ox = a.transposed ? 2 * j + px : j;
        float* dst = a.partial + ((((long long)split * a.B + b) * a.Ho + oy) * a.Wo + ox) * a.N;
#pragma unroll
        for (int nj = 0; nj < 4; ++nj) {
          const int n = n0 + wn * 64 + 16 * nj + r;
          if (n < a.N) dst[n] = acc[mi][nj][reg];
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
// One block per 32 pixels x 32 channels, transposed through LDS so both stores coalesce.
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
      for (int sp = 0; sp < a.ksplit; ++sp) v += a.partial[((long long)sp * P + p) * a.N + n];
      const int b = (int)(p / HW);
      if (a.bias4) {
        const int nm = a.info[b].n_masks;
        float bs = 0.f;
        for (int i = 0; i < nm; ++i) bs += a.bias4[i * a.N + n];
        v += bs;
      }
      if (a.out_nhwc) {
        // NHWC store wants the residual too: read it (NCHW, strided) here
        if (a.residual) v += bf16_to_f32(((const bf16_t*)a.residual)[((long long)b * a.N + n) * HW + (p % HW)]);
        ((bf16_t*)a.out_nhwc)[p * a.N + n] = f32_to_bf16(v);
      } else if (a.residual) {
        v += bf16_to_f32(((const bf16_t*)a.residual)[((long long)b * a.N + n) * HW + (p % HW)]);
      }
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

template <typename T>
int launch_conv(const ConvArgs& a, hipStream_t s) {
  TimerScope ts(a.transposed ? "dsam_dx" : "dsam_fwd", s);
  int nclass = a.transposed ? 4 : 1;
  long long Mmax = (long long)a.B * a.Ho * a.Wo;
  if (a.transposed) Mmax = (long long)a.B * ((a.Ho + 1) / 2) * ((a.Wo + 1) / 2);
  if constexpr (sizeof(T) == 2) {
    if (a.C % 32 == 0 && a.nseg == 5) {
      ConvArgs b = a;
      b.ksplit = v2_ksplit(Mmax, a.N, nclass, a.C, a.transposed);
      dim3 grid2(ceil_div(Mmax, V2M), ceil_div(a.N, V2N), nclass * b.ksplit);
      k_conv_igemm_v2<<<grid2, 256, 0, s>>>(b);
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

int rgbd_dsam_pack_weights(int dtype, const float* conv_w, const float* proj_w, int Cin, int Cout,
                           void* wfwd, void* wbwd, void* stream) {
  RGBD_REQUIRE(conv_w && proj_w && (wfwd || wbwd) && Cin > 0 && Cout > 0, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  const long long total = 45ll * Cin * Cout;
  const int nb = (int)std::min<long long>(ceil_div(total, 256), 4096);
  if (dtype == RGBD_F32)
    k_pack_dsam<float><<<nb, 256, 0, s>>>(conv_w, proj_w, Cin, Cout, (float*)wfwd, (float*)wbwd);
  else if (dtype == RGBD_BF16)
    k_pack_dsam<bf16_t><<<nb, 256, 0, s>>>(conv_w, proj_w, Cin, Cout, (bf16_t*)wfwd, (bf16_t*)wbwd);
  else
    return RGBD_E_DTYPE;
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
  return std::max<size_t>(256, std::max(v2_partial_bytes(fwd_args(B, Cin, h, w, Cout)),
                                        v2_partial_bytes(dx_args(B, Cin, h, w, Cout))));
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
  RGBD_REQUIRE(ws || dtype != RGBD_BF16 || v2_partial_bytes(a) == 0, RGBD_E_ARG);
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
  RGBD_REQUIRE(ws || dtype != RGBD_BF16 || v2_partial_bytes(a) == 0, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_F32) return launch_conv<float>(a, s);
  if (dtype == RGBD_BF16) return launch_conv<bf16_t>(a, s);
  return RGBD_E_DTYPE;
}

size_t rgbd_dsam_bwd_weight_workspace_size(int dtype, int B, int Cin, int h, int w, int Cout) {
  (void)dtype; (void)h; (void)w;
  const int sp = dsam_wgrad_splits(B, Cin, Cout);
  return align256(sizeof(float) * (size_t)sp * Cout * 45 * Cin) + align256(sizeof(float) * (size_t)B * Cout);
}

int rgbd_dsam_bwd_weight(int dtype, const void* gout_nchw, const void* x_nhwc, const uint8_t* code,
                         const rgbd_decomp_info* info, int B, int Cin, int h, int w, int Cout,
                         float* dconv_w, float* dproj_w, float* dbias, void* ws, void* stream) {
  RGBD_REQUIRE(gout_nchw && x_nhwc && code && info && dconv_w && dproj_w && dbias && ws, RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && h > 0 && w > 0 && Cout > 0 && Cin > 0, RGBD_E_ARG);
  RGBD_REQUIRE(Cin % 8 == 0, RGBD_E_SHAPE);
  hipStream_t s = (hipStream_t)stream;
  const int sp = dsam_wgrad_splits(B, Cin, Cout);
  float* partial = (float*)ws;
  float* csum = (float*)((char*)ws + align256(sizeof(float) * (size_t)sp * Cout * 45 * Cin));
  TimerScope ts("dsam_wgrad", s);
  dim3 grid(ceil_div(45ll * Cin, 64), ceil_div(Cout, 64), sp);
  const int hwo = ((h + 1) / 2) * ((w + 1) / 2);
  if (dtype == RGBD_F32) {
    k_dsam_wgrad<float><<<grid, 256, 0, s>>>((const float*)gout_nchw, (const float*)x_nhwc, code, B, Cin, h, w,
                                             Cout, sp, partial);
    k_chan_sum<float><<<B * Cout, 256, 0, s>>>((const float*)gout_nchw, hwo, csum);
  } else if (dtype == RGBD_BF16) {
    dim3 g2(ceil_div(45ll * Cin, WG_KK), ceil_div(Cout, WG_O), sp);
    k_dsam_wgrad_bf16<<<g2, 256, 0, s>>>((const bf16_t*)gout_nchw, (const bf16_t*)x_nhwc, code, B, Cin, h, w,
                                         Cout, sp, partial);
    k_chan_sum<bf16_t><<<B * Cout, 256, 0, s>>>((const bf16_t*)gout_nchw, hwo, csum);
  } else {
    return RGBD_E_DTYPE;
  }
  const long long total = 45ll * Cin * Cout;
  k_dsam_wgrad_final<<<(int)std::min<long long>(ceil_div(total, 256), 4096), 256, 0, s>>>(
      partial, sp, Cin, Cout, dconv_w, dproj_w);
  k_dsam_bias_grad<<<ceil_div(4 * Cout, 256), 256, 0, s>>>(csum, info, B, Cout, dbias);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
