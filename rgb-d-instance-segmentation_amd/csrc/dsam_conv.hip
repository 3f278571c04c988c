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
#include <cstdlib>

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
  const void* residual_nhwc;        // bf16 only: NHWC residual, used when out_nchw is null
  void* out_nchw;                   // optional
  void* out_nhwc;                   // optional
  int ksplit;                       // unused (1)
  uint16_t* tmasks;                 // bf16: [class][tile][16] per-tap code sets (k_dsam_plan)
  int* items;                       // bf16: work list of k_dsam_lds (k_dsam_items)
  int* nitems;
  int* tickets;                     // bf16: per (class, tile, N tile) chunk counter, zeroed by k_dsam_plan
  int* work;                        // bf16: per N tile next-item counter of k_dsam_lds, zeroed by k_dsam_plan
  int ntiles0;                      // bf16: tiles of the largest class
  int chunk_len;                    // bf16: steps per workgroup chunk of a tile
  int ncg;                          // bf16: K chunk groups per tap (C / (32 * KC))
  int linear;                       // bf16: tile rows = 128 consecutive pixels of the (class) grid
                                    // over the batch instead of 8 x 16 blocks (small grids)
  float* partial;                   // bf16: partial tiles of multi-chunk tiles (reduced by their last chunk)
  const bf16_t* zero;               // bf16: LD_ZERO_BYTES of zeros (zeroed by k_dsam_plan)
  unsigned long long* stamps;       // diagnostics only (rgbd_debug_dsam_stamps); null otherwise
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

// bf16 code-merged filters W_k = proj + sum_{i in k} conv_i (fixed summation order: proj, then
// conv_0..conv_3, in f32, rounded once), packed for the codes present in the batch only (bit k of
// *code_mask; all 16 when code_mask is NULL), as the B tiles of k_dsam_lds:
//   wfwd [16 code][9 tap][Cin/32 chunk][Cout n][32 c]   (forward: rows n = output channels)
//   wbwd [16 code][9 tap][Cout/32 chunk][Cin n][32 o]   (dX: rows n = input channels)
// so the tile of one (code, tap, chunk) is contiguous (one linear LDS-DMA stream), with the four
// 16-byte chunks of each 64-byte row stored XOR-swizzled by lds_swz(n) (the LDS image the MFMA
// fragment reads want).  A one-tile tail pad keeps an over-reading last N tile in bounds.
//
// lds_swz: 16-byte chunk g of 64-byte row n sits at slot g ^ lds_swz(n).  A fragment read has
// lane (r, g) take chunk g of row base+r (base a multiple of 16); the slot is 4*(n%4) + chunk, and
// with the XOR by 2 on rows 8..15 of every 16 the 16 lanes of each ds_read_b128 lane group
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...; MI355X_MICROARCH.md LDS table) hit 16 distinct
// 4-bank slots: conflict-free.  (The earlier (n >> 2) & 3 was conflict-free only for 16
// consecutive lanes, not for the hardware groups.)
__host__ __device__ __forceinline__ int lds_swz(int n) { return ((n >> 3) & 1) << 1; }

// Both packings from one pass over the f32 weights.  Workgroup = a block of PK_OB output x PK_CB
// input channels: its 5 x PK_OB rows of (32 c x 9 taps) f32 (conv_0..3, proj; 1152 contiguous
// bytes each in OIHW) are staged in LDS by 16-byte loads, all in flight together.  A unit is 8
// consecutive channels of one (row, tap): wfwd units (o, tap, 8 c) and wbwd units (c, tap, 8 o);
// each reads its 5 x 8 segment values once and writes one 16-byte chunk per present code.  Rows
// are padded to 289 floats so the unit reads of a wave fall on distinct banks.
constexpr int PK_OB = 16, PK_CB = 32, PK_LD = PK_CB * 9 + 1;
constexpr size_t PK_SMEM = 5 * PK_OB * PK_LD * sizeof(float);
__global__ __launch_bounds__(256) void k_pack_codes(const float* __restrict__ conv_w, const float* __restrict__ proj_w,
                                                    int Cin, int Cout, const uint32_t* __restrict__ code_mask,
                                                    bf16_t* __restrict__ wfwd, bf16_t* __restrict__ wbwd) {
  extern __shared__ float sw[];  // [5 seg][PK_OB o][PK_LD]: element (o, c, tap) at c * 9 + tap
  const int c0 = blockIdx.x * PK_CB, o0 = blockIdx.y * PK_OB, tid = threadIdx.x;
  const int nci = Cin / 32, nco = Cout / 32;
  if (blockIdx.x == 0 && blockIdx.y == 0)  // tail pads (read only by an over-reaching last N tile)
    for (int i = tid; i < 192 * 32; i += 256) {
      wfwd[144ll * Cin * Cout + i] = 0;
      if (wbwd) wbwd[144ll * Cin * Cout + i] = 0;
    }
  constexpr int NQ = 5 * PK_OB * (PK_CB * 9 / 4);  // float4 pieces of the block
  constexpr int PER = (NQ + 255) / 256;
  float4 v[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = tid + 256 * j;
    if (i < NQ) {
      const int row = i / (PK_CB * 9 / 4), q = i - row * (PK_CB * 9 / 4), seg = row / PK_OB, o = o0 + row % PK_OB;
      const float* src = seg < 4 ? conv_w + (((long long)seg * Cout + o) * Cin + c0) * 9 : proj_w + ((long long)o * Cin + c0) * 9;
      v[j] = reinterpret_cast<const float4*>(src)[q];
    }
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = tid + 256 * j;
    if (i < NQ) {
      const int row = i / (PK_CB * 9 / 4), q = i - row * (PK_CB * 9 / 4);
      float* d = sw + row * PK_LD + 4 * q;
      d[0] = v[j].x;
      d[1] = v[j].y;
      d[2] = v[j].z;
      d[3] = v[j].w;
    }
  }
  __syncthreads();
  const uint32_t m = code_mask ? *code_mask : 0xffffu;
  // units 0..575: wfwd (tap, o, 8-c chunk q); 576..1151: wbwd (tap, c, 8-o chunk q)
  const int nunits = wbwd ? 2 * 9 * PK_OB * 4 : 9 * PK_OB * 4;
  for (int u = tid; u < nunits; u += 256) {
    const bool bwd = u >= 9 * PK_OB * 4;
    const int w = bwd ? u - 9 * PK_OB * 4 : u;
    const int tap = w / (PK_OB * 4);
    int base, step;  // LDS offset of value e: base + e * step (+ seg * PK_OB * PK_LD)
    long long dst0;  // element offset of the unit's 16-byte chunk for code 0
    long long kstride;
    if (!bwd) {
      const int ol = (w >> 2) & (PK_OB - 1), q = w & 3, n = o0 + ol;
      base = ol * PK_LD + 8 * q * 9 + tap;
      step = 9;
      dst0 = (((long long)tap * nci + blockIdx.x) * Cout + n) * 32 + 8 * ((q ^ lds_swz(n)) & 3);
      kstride = 9ll * nci * Cout * 32;
    } else {
      const int cl = (w >> 1) & (PK_CB - 1), q = w & 1, n = c0 + cl, qo = (o0 & 31) / 8 + q;
      base = 8 * q * PK_LD + cl * 9 + tap;
      step = PK_LD;
      dst0 = (((long long)tap * nco + (o0 >> 5)) * Cin + n) * 32 + 8 * ((qo ^ lds_swz(n)) & 3);
      kstride = 9ll * nco * Cin * 32;
    }
    float s[5][8];
#pragma unroll
    for (int sg = 0; sg < 5; ++sg)
#pragma unroll
      for (int e = 0; e < 8; ++e) s[sg][e] = sw[sg * PK_OB * PK_LD + base + e * step];
    bf16_t* out = bwd ? wbwd : wfwd;
    for (int k = 0; k < 16; ++k) {
      if (!((m >> k) & 1u)) continue;
      float r[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t = s[4][e];  // proj, then conv_0..conv_3 of the code's bits, in f32, rounded once
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if ((k >> i) & 1) t += s[i][e];
        r[e] = t;
      }
      *reinterpret_cast<uint4*>(out + dst0 + k * kstride) =
          make_uint4(pack_bf16x2(r[0], r[1]), pack_bf16x2(r[2], r[3]), pack_bf16x2(r[4], r[5]), pack_bf16x2(r[6], r[7]));
    }
  }
}

// OR of (1 << code) over each code map (codes present per DSAM input resolution).
struct CodeMaps {
  const uint8_t* p[8];
  long long n[8];
};
__global__ __launch_bounds__(256) void k_code_masks(CodeMaps cm, uint32_t* __restrict__ masks) {
  const int y = blockIdx.y;
  const uint8_t* p = cm.p[y];
  const long long n = cm.n[y];
  uint32_t m = 0u;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) m |= 1u << (p[i] & 15);
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) m |= (uint32_t)__shfl_xor((int)m, o);
  if ((threadIdx.x & 63) == 0 && m) atomicOr(masks + y, m);
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

// bf16 NCHW -> NHWC with 16-byte global accesses (HW % 8 == 0, C % 8 == 0): a workgroup moves a
// 64-channel x 64-pixel tile; loads take 8 pixels of one channel, stores 8 channels of one pixel,
// the transpose happens in the LDS writes ([pixel][channel] rows padded to 72 elements).
__global__ __launch_bounds__(256) void k_nchw_to_nhwc_v8(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst,
                                                         int C, int HW) {
  __shared__ __attribute__((aligned(16))) bf16_t tile[64][72];
  const int b = blockIdx.z, p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int v = threadIdx.x + 256 * k, cl = v >> 3, pl = (v & 7) * 8;  // channel, 8-pixel group
    const int c = c0 + cl, p = p0 + pl;
    uint4 u = make_uint4(0u, 0u, 0u, 0u);
    if (c < C && p < HW) u = *reinterpret_cast<const uint4*>(src + ((long long)b * C + c) * HW + p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      tile[pl + 2 * e][cl] = (bf16_t)(w[e] & 0xffffu);
      tile[pl + 2 * e + 1][cl] = (bf16_t)(w[e] >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int v = threadIdx.x + 256 * k, pl = v >> 3, cl = (v & 7) * 8;  // pixel, 8-channel group
    const int p = p0 + pl, c = c0 + cl;
    if (p < HW && c < C)
      *reinterpret_cast<uint4*>(dst + ((long long)b * HW + p) * C + c) = *reinterpret_cast<const uint4*>(&tile[pl][cl]);
  }
}

// Several bf16 NCHW -> NHWC conversions in one launch (the hot path's four colour maps in the
// forward, its three upstream gradients in the backward): a 1-D grid of 64 x 64 tiles over all
// jobs; a job whose HW is not a multiple of 8 loads its pixels one by one (same tile, same stores).
constexpr int NHWC_MAXJOB = 4;
struct NhwcJobs {
  const bf16_t* src[NHWC_MAXJOB];
  bf16_t* dst[NHWC_MAXJOB];
  int C[NHWC_MAXJOB], HW[NHWC_MAXJOB], tp[NHWC_MAXJOB], tc[NHWC_MAXJOB];
  int block0[NHWC_MAXJOB + 1];  // first block of each job; block0[n] = grid
  int n;
};
__global__ __launch_bounds__(256) void k_nchw_to_nhwc_multi(const NhwcJobs J) {
  __shared__ __attribute__((aligned(16))) bf16_t tile[64][72];
  int j = 0;
#pragma unroll
  for (int i = 1; i < NHWC_MAXJOB; ++i)
    if (i < J.n && (int)blockIdx.x >= J.block0[i]) j = i;
  const bf16_t* src = J.src[j];
  bf16_t* dst = J.dst[j];
  const int C = J.C[j], HW = J.HW[j], per = J.tp[j] * J.tc[j];
  const int idx = blockIdx.x - J.block0[j], b = idx / per, t = idx - b * per;
  const int p0 = (t % J.tp[j]) * 64, c0 = (t / J.tp[j]) * 64;
  const bool vec = (HW & 7) == 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int v = threadIdx.x + 256 * k, cl = v >> 3, pl = (v & 7) * 8;  // channel, 8-pixel group
    const int c = c0 + cl, p = p0 + pl;
    const bf16_t* row = src + ((long long)b * C + c) * HW;
    bf16_t e8[8];
    if (vec) {
      uint4 u = make_uint4(0u, 0u, 0u, 0u);
      if (c < C && p < HW) u = *reinterpret_cast<const uint4*>(row + p);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        e8[2 * e] = (bf16_t)(w[e] & 0xffffu);
        e8[2 * e + 1] = (bf16_t)(w[e] >> 16);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) e8[e] = (c < C && p + e < HW) ? row[p + e] : (bf16_t)0;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) tile[pl + e][cl] = e8[e];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int v = threadIdx.x + 256 * k, pl = v >> 3, cl = (v & 7) * 8;  // pixel, 8-channel group
    const int p = p0 + pl, c = c0 + cl;
    if (p < HW && c < C)
      *reinterpret_cast<uint4*>(dst + ((long long)b * HW + p) * C + c) = *reinterpret_cast<const uint4*>(&tile[pl][cl]);
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

// bf16 dW, code-merged:
//   dW_k[o][tap][c] = sum over output px p with code(src(p, tap)) == k of G[p][o] X[src][c]
// for every region code k present, folded by k_dsam_wgrad_fold into the five filters (conv_i
// gets the codes with bit i, proj gets all): work ~ one dense dW instead of popcount + 1 of them.
// A unit is 64 raster-consecutive output pixels of one image.  Load balance: one code (the
// remainder region) typically meets every unit while the others meet a few percent, so
// wg_plan_body builds per-code lists of live units (code_presence_body) and cuts them into items of
// about equal length; wg_masks_body precomputes, per list entry and tap, the 64-bit mask of the
// unit's pixels whose source meets code k; k_dsam_wgrad_mm runs persistently over
// (item, output tile) work.
//
// Output tile: 32*FM channels (o) x 128 kk (kk = tap*Cin + c: four 32-wide blocks, each inside
// one tap), 4 waves as 2x2 (wave tile 16*FM x 64); one unit (64 px = two MFMA k-blocks) per
// step, operands by LDS-DMA in an S-deep ring, S-1 steps ahead:
//   G  [64 px][32*FM o] from the NHWC upstream gradient (FM blocks of 64-byte rows),
//   X  [64 px][4 x 32 c] im2col rows from the NHWC input; every row copies a valid (clamped)
//      pixel and the rows outside the input, past the image or of another code are zeroed in
//      registers from the entry's tap masks (staged in LDS with the item's unit ids).
// Both MFMA operands are read with ds_read_b64_tr_b16 ([px][col] -> k-major fragments); rows are
// XOR-swizzled by row bit 3 so the 32-lane halves of a transposed read fall on disjoint banks.
constexpr int LD_ZERO_BYTES = 512;  // zeroed global row the DMA reads for masked-out operand rows
constexpr int WPX = 64;        // output pixels per unit / step
constexpr int WITEM_MAX = 64;  // units per item (LDS staging of ids + masks)
typedef __attribute__((ext_vector_type(4))) short v4s;

template <int FM>
struct WgCfg {
  static constexpr int S = FM == 6 ? 3 : 4;
  static constexpr int NBLK = FM + 4;            // 4 KB blocks per stage: FM of G, 4 of X
  static constexpr int STAGE = NBLK * WPX * 64;
  static constexpr int PER = NBLK;               // DMA pieces per wave per step
  static constexpr int OFF_UNITS = S * STAGE;    // [WITEM_MAX] int unit ids
  static constexpr int OFF_MASKS = OFF_UNITS + WITEM_MAX * 4;  // [WITEM_MAX][9] u64 tap masks
  static constexpr size_t SMEM = (size_t)OFF_MASKS + WITEM_MAX * 9 * 8;
  static_assert(SMEM <= 163840, "dW LDS budget");
};

__device__ __forceinline__ int wg_swz(int row) { return ((row >> 3) & 1) << 1; }

struct WgArgs {
  const bf16_t* gout;     // NHWC [B][ho][wo][Cout]
  const bf16_t* x;        // NHWC [B][h][w][Cin]
  const uint8_t* code;    // [B][h][w]
  const uint16_t* pres;   // [B * nunit] bit k: code k met by the unit's sources
  int* list;              // [<= 16 * B * nunit] live entries: unit | code << 24, by code then unit
  unsigned long long* masks;  // [entry][9] tap masks of the entry's unit for its code
  int4* items;            // [<= 16 * B * nunit] (code, first entry, end entry, -)
  int* counts;            // [0] live entries, [1] items
  int B, Cin, h, w, Cout, ho, wo, nunit, ntile_kk, ntile_o, target;
  float inv_wo;
  const bf16_t* zero;     // LD_ZERO_BYTES of zeros (rows the im2col gather masks out)
  float* partial;         // [item][Cout][9*Cin] f32
};

__device__ __forceinline__ void code_presence_body(const uint8_t* __restrict__ code, int B, int h, int w,
                                                   uint16_t* __restrict__ pres, int block) {
  // one wave per 64-px unit: OR of 1 << code over its 9-tap sources
  const int ho = (h + 1) / 2, wo = (w + 1) / 2, hwo = ho * wo, nunit = (hwo + WPX - 1) / WPX;
  const long long u = (block * (long long)blockDim.x + threadIdx.x) >> 6;
  const int l = threadIdx.x & 63;
  uint32_t m = 0u;
  if (u < (long long)B * nunit) {
    const int b = (int)(u / nunit), p = (int)(u % nunit) * WPX + l;
    if (p < hwo) {
      const int oy = p / wo, ox = p % wo;
      uint32_t cv[9];
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int iy = 2 * oy - 1 + tap / 3, ix = 2 * ox - 1 + tap % 3;
        const bool ok = iy >= 0 && iy < h && ix >= 0 && ix < w;
        cv[tap] = code[((long long)b * h + (ok ? iy : 0)) * w + (ok ? ix : 0)];  // unconditional: one round trip
        cv[tap] = ok ? 1u << cv[tap] : 0u;
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) m |= cv[tap];
    }
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) m |= (uint32_t)__shfl_xor((int)m, o);
  if (l == 0 && u < (long long)B * nunit) {
    pres[u] = (uint16_t)m;
  }
}

// Plan (one 1024-thread workgroup): per code the ordered list of live units, then items of
// about equal length L = ceil(entries / (target / output tiles)), capped at WITEM_MAX.
constexpr int WG_PRES_LDS = 8192;  // presence entries k_wg_plan keeps in LDS
__device__ __forceinline__ void wg_plan_body(const WgArgs& a) {
  __shared__ int cnt_s[16], off_s[17];
  if (threadIdx.x < LD_ZERO_BYTES / 16)
    reinterpret_cast<uint4*>(const_cast<bf16_t*>(a.zero))[threadIdx.x] = make_uint4(0u, 0u, 0u, 0u);
  __shared__ uint16_t spres[WG_PRES_LDS];  // the compaction pass re-reads presence from LDS
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int U = a.B * a.nunit;
  const bool in_lds = U <= WG_PRES_LDS;
  if (tid < 16) cnt_s[tid] = 0;
  __syncthreads();
  // counts per code
  uint32_t c16[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) c16[k] = 0u;
  for (int u = tid; u < U; u += 1024) {
    const uint32_t m = a.pres[u];
    if (in_lds) spres[u] = (uint16_t)m;
#pragma unroll
    for (int k = 0; k < 16; ++k) c16[k] += (m >> k) & 1u;
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    uint32_t v = c16[k];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v += (uint32_t)__shfl_xor((int)v, o);
    if (lane == 0 && v) atomicAdd(&cnt_s[k], (int)v);
  }
  __syncthreads();
  if (tid == 0) {
    int o = 0;
    for (int k = 0; k < 16; ++k) {
      off_s[k] = o;
      o += cnt_s[k];
    }
    off_s[16] = o;
  }
  __syncthreads();
  // ordered compaction, all 16 codes per pass: wave ballots -> per-(code, wave) counts ->
  // exclusive offsets; units keep their order within each code
  __shared__ int wc[16][16], wpre[16][16], cbase[16], ctot[16];
  if (tid < 16) cbase[tid] = off_s[tid];
  for (int u0 = 0; u0 < U; u0 += 1024) {
    const int u = u0 + tid;
    const uint32_t m = u < U ? (in_lds ? (uint32_t)spres[u] : (uint32_t)a.pres[u]) : 0u;
    unsigned long long bal[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      bal[k] = __ballot((m >> k) & 1u);
      if (lane == 0) wc[k][w] = __popcll(bal[k]);
    }
    __syncthreads();
    if (tid < 256) {
      const int k = tid >> 4, q = tid & 15;
      int pre = 0;
      for (int i = 0; i < q; ++i) pre += wc[k][i];
      wpre[k][q] = pre;
      if (q == 15) ctot[k] = pre + wc[k][15];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if ((m >> k) & 1u)
        a.list[cbase[k] + wpre[k][w] + __popcll(bal[k] & ((1ull << lane) - 1ull))] = u | (k << 24);
    __syncthreads();
    if (tid < 16) cbase[tid] += ctot[tid];
    __syncthreads();
  }
  // items: code k's c live units cut into n_k = ceil(c / L) near-equal runs, emitted in parallel
  __shared__ int ibase[17];
  const int total = off_s[16];
  const int want = max(1, a.target / max(1, a.ntile_kk * a.ntile_o));
  const int L = min(max(1, (total + want - 1) / want), WITEM_MAX);
  if (tid == 0) {
    int ni = 0;
    for (int k = 0; k < 16; ++k) {
      ibase[k] = ni;
      ni += (cnt_s[k] + L - 1) / L;
    }
    ibase[16] = ni;
    a.counts[0] = total;
    a.counts[1] = ni;
    a.counts[2] = 0;  // k_dsam_wgrad_mm's next-work counter
    a.counts[3] = 0;  // ... and its next channel-sum unit (fold)
  }
  __syncthreads();
  for (int it = tid; it < ibase[16]; it += 1024) {
    int k = 0;
    while (it >= ibase[k + 1]) ++k;
    const int c = cnt_s[k], n = ibase[k + 1] - ibase[k], j = it - ibase[k];
    a.items[it] = make_int4(k, off_s[k] + (int)((long long)c * j / n), off_s[k] + (int)((long long)c * (j + 1) / n), 0);
  }
}

// Tap masks of every live entry: one wave per entry, lane = pixel of the unit.
__device__ __forceinline__ void wg_masks_body(const WgArgs& a, int block) {
  const int e = (block * 256 + threadIdx.x) >> 6, l = threadIdx.x & 63;
  if (e >= a.counts[0]) return;  // wave-uniform
  const int v = a.list[e], u = v & 0xffffff, k = v >> 24;
  const int hwo = a.ho * a.wo, b = u / a.nunit, p = (u % a.nunit) * WPX + l;
  const bool pv = p < hwo;
  const int oy = pv ? p / a.wo : 0, ox = pv ? p % a.wo : 0;
  uint32_t cv[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int iy = 2 * oy - 1 + tap / 3, ix = 2 * ox - 1 + tap % 3;
    const bool ok = pv && iy >= 0 && iy < a.h && ix >= 0 && ix < a.w;
    cv[tap] = a.code[((long long)b * a.h + (ok ? iy : 0)) * a.w + (ok ? ix : 0)];  // unconditional: one round trip
    cv[tap] = ok ? cv[tap] : 0xffu;
  }
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const unsigned long long m = __ballot(cv[tap] == (uint32_t)k);
    if (l == 0) a.masks[(long long)e * 9 + tap] = m;
  }
}

// The dW planning of up to WG_MAXLEG legs in three launches (blockIdx.z = leg; blocks past a
// leg's own count exit): unit presence, the per-code lists and items, the tap masks.
constexpr int WG_MAXLEG = 4;
struct WgLegs {
  WgArgs a[WG_MAXLEG];
  int max_entries[WG_MAXLEG];
  int n;
};
__global__ __launch_bounds__(256) void k_code_presence_legs(const WgLegs L) {
  const WgArgs& a = L.a[blockIdx.z];
  if ((long long)blockIdx.x * 256 >= (long long)a.B * a.nunit * 64) return;  // block-uniform
  code_presence_body(a.code, a.B, a.h, a.w, const_cast<uint16_t*>(a.pres), blockIdx.x);
}
__global__ __launch_bounds__(1024) void k_wg_plan_legs(const WgLegs L) { wg_plan_body(L.a[blockIdx.z]); }
__global__ __launch_bounds__(256) void k_wg_masks_legs(const WgLegs L) {
  const WgArgs& a = L.a[blockIdx.z];
  if ((long long)blockIdx.x * 4 >= L.max_entries[blockIdx.z]) return;  // block-uniform
  wg_masks_body(a, blockIdx.x);
}

// out[(split*B + b)*C + c] = sum over pixel range `split` of g[b][p][c], NHWC bf16 g: workgroup
// (b, 64 channels, split), thread = channel pair x one of 8 pixel strides, fixed-order combine.
constexpr int CS_SPLIT_MAX = 16;
__host__ __device__ inline int chan_sum_splits(int HW) {
  const int sp = HW / 256;
  return sp < 1 ? 1 : (sp > CS_SPLIT_MAX ? CS_SPLIT_MAX : sp);
}
// one workgroup's share: image b, channels [64 cb, 64 cb + 64), pixel range sp of nsp
__device__ __forceinline__ void chan_sum_body(const bf16_t* __restrict__ g, int HW, int C, int B, int b, int cb,
                                              int sp, int nsp, float* __restrict__ out, float2 (*red)[32]) {
  const int cp = threadIdx.x & 31, sub = threadIdx.x >> 5;
  const int c = cb * 64 + 2 * cp;
  const int p0 = (int)((long long)sp * HW / nsp), p1 = (int)((long long)(sp + 1) * HW / nsp);
  float2 acc = make_float2(0.f, 0.f);
  if (c < C) {
    const bf16_t* base = g + (long long)b * HW * C + c;
#pragma unroll 4
    for (int p = p0 + sub; p < p1; p += 8) {
      const uint32_t u = *reinterpret_cast<const uint32_t*>(base + (long long)p * C);
      acc.x += __uint_as_float(u << 16);
      acc.y += __uint_as_float(u & 0xffff0000u);
    }
  }
  red[sub][cp] = acc;
  __syncthreads();
  if (sub == 0 && c < C) {
    float2 t = red[0][cp];
    for (int q = 1; q < 8; ++q) {
      t.x += red[q][cp].x;
      t.y += red[q][cp].y;
    }
    float* o = out + ((long long)sp * B + b) * C + c;
    o[0] = t.x;
    if (c + 1 < C) o[1] = t.y;
  }
}
// NL legs of one output tile shape in one persistent launch: every workgroup drains leg 0's work
// counter, then leg 1's, ..., so legs that are ready together share the CUs instead of queueing
// whole-chip launches behind each other (the loop body is instantiated per leg: each leg's
// arguments stay scalar kernel arguments).
//
// With fold set, the workgroups then drain the legs' bias channel sums (chan_sum_body units of the
// upstream gradient, counter counts[3]) — work that would otherwise be one more launch after the
// GEMM's drain tail.
template <int NL>
struct WgMulti {
  WgArgs a[NL];
  float* csum[NL];  // [nsplit][B][Cout] channel sums (fold)
  int n;            // legs in use, 1..NL
  int fold;
};

template <int FM, int NL>
__global__ __launch_bounds__(256) void k_dsam_wgrad_mm(const WgMulti<NL> L) {
  using Cfg = WgCfg<FM>;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  int* sunits = (int*)(smem + Cfg::OFF_UNITS);
  unsigned long long* smasks = (unsigned long long*)(smem + Cfg::OFF_MASKS);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int wm = wave & 1, wn = wave >> 1;
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  // per-lane copy roles: pixel row pr of every block, 16-byte chunk q
  const int pr = 16 * wave + (lane >> 2);
  const int qch = 8 * ((lane & 3) ^ wg_swz(pr));
  // transposed fragment [k = 8g + j][col = c0 + r] of a [64 px][32 col] block (64-byte rows): the
  // XOR swizzle term depends on row bit 3 = g & 1 only, so every read of a lane is its base
  // address plus a compile-time offset
  const int q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int trow = 8 * g + q4;
  const int tbase0 = trow * 64 + 16 * ((p4 >> 1) ^ wg_swz(trow)) + (4 * p4 & 7) * 2;        // c0 = 0
  const int tbase16 = trow * 64 + 16 * ((2 | (p4 >> 1)) ^ wg_swz(trow)) + (4 * p4 & 7) * 2;  // c0 = 16
  typedef __attribute__((address_space(3))) char lds_char;
  typedef __attribute__((address_space(3))) v4s lds_v4s;
  lds_char* const lsm = (lds_char*)smem;  // one generic -> LDS conversion, not one per read
  lds_char* b0 = lsm;   // this step's slot + the lane's base, per c0
  lds_char* b16 = lsm;
  auto trfrag = [&](int blk, int kb, int c0) {  // blk: block byte offset in the slot; c0 in {0, 16}
    lds_char* p = (c0 ? b16 : b0) + blk + kb * 32 * 64;
    const v4s t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)p);
    const v4s t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p + 4 * 64));
    Frag<bf16_t> f;
    const uint2 u0 = __builtin_bit_cast(uint2, t0), u1 = __builtin_bit_cast(uint2, t1);
    f.v = make_uint4(u0.x, u0.y, u1.x, u1.y);
    return f;
  };
  int* next_s = (int*)(smem + Cfg::OFF_UNITS) + WITEM_MAX - 1;  // unit ids are staged after the read
  auto run_leg = [&](const WgArgs& a) {
    const int KK = 9 * a.Cin, hwo = a.ho * a.wo, ntile = a.ntile_kk * a.ntile_o;
    const int nwork = a.counts[1] * ntile;
    for (;;) {
      // dynamic assignment of (item, tile) work: items differ in live units per code
      __syncthreads();
      if (tid == 0) *next_s = __hip_atomic_fetch_add(a.counts + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int wi = *next_s;
      __syncthreads();  // every thread has it before the unit ids overwrite the slot
      if (wi >= nwork) break;
      const int4 item = a.items[wi / ntile];
      const int tile = wi % ntile, e0 = item.y, nst = item.z - item.y;
      const int kk0 = (tile % a.ntile_kk) * 128, o0 = (tile / a.ntile_kk) * 32 * FM;
      // stage the item's unit ids and tap masks
      for (int i = tid; i < nst; i += 256) sunits[i] = a.list[e0 + i] & 0xffffff;
      for (int i = tid; i < nst * 9; i += 256) smasks[i] = a.masks[(long long)e0 * 9 + i];
      __syncthreads();
      // X block j: (tap, channel offset) uniform; source offset dy*w + dx from the row's origin
      int xtap[4], xoff[4], xc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kk = kk0 + 32 * j;
        const bool ok = kk < KK;
        xtap[j] = ok ? kk / a.Cin : -1;
        const int tp = ok ? xtap[j] : 0;
        xoff[j] = (tp / 3) * a.w + tp % 3;
        xc[j] = ok ? kk % a.Cin : 0;
      }
      const bf16_t* zrow = a.zero + qch;
      // One step = one unit: G rows (its 64 output pixels) and X rows (their im2col sources).  A
      // row of X whose source is outside the input, past the image, or of another code than the
      // item's reads the zero row: it contributes exactly zero, no masking in registers.
      auto issue = [&](int slot, int it) {
        const int u = __builtin_amdgcn_readfirstlane(sunits[it]);
        const int b = u / a.nunit;
        const int p = (u - b * a.nunit) * WPX + pr;
        const int pc = p < hwo ? p : hwo - 1;
        const int oy = (int)(((float)pc + 0.5f) * a.inv_wo), ox = pc - oy * a.wo;
        const uint32_t sb = lds0 + slot * Cfg::STAGE + wave * 1024;
        const bf16_t* gsrc = a.gout + ((long long)b * hwo + pc) * a.Cout + qch;
#pragma unroll
        for (int ob = 0; ob < FM; ++ob) dma_lds16(gsrc + min(o0 + 32 * ob, a.Cout - 32), sb + ob * 4096);
        const int org = (b * a.h + 2 * oy - 1) * a.w + 2 * ox - 1;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const unsigned long long m = xtap[j] >= 0 ? smasks[it * 9 + xtap[j]] : 0ull;
          const bool live = (m >> pr) & 1ull;
          const bf16_t* src = live ? a.x + (long long)(org + xoff[j]) * a.Cin + xc[j] + qch : zrow;
          dma_lds16(src, sb + (FM + j) * 4096);
        }
      };
      f32x4 acc[FM][4];
#pragma unroll
      for (int mi = 0; mi < FM; ++mi)
#pragma unroll
        for (int nj = 0; nj < 4; ++nj) acc[mi][nj] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int npro = nst < Cfg::S - 1 ? nst : Cfg::S - 1;
      for (int i = 0; i < npro; ++i) issue(i, i);
      if (npro >= 3) vm_wait_barrier<2 * Cfg::PER>();
      else if (npro == 2) vm_wait_barrier<Cfg::PER>();
      else vm_wait_barrier<0>();
#pragma unroll 1
      for (int s = 0; s < nst; ++s) {
        if (s + Cfg::S - 1 < nst) issue((s + Cfg::S - 1) % Cfg::S, s + Cfg::S - 1);
        int st = (s % Cfg::S) * Cfg::STAGE;
        asm volatile("" : "+s"(st));  // no strength reduction of the slot offset into per-read registers
        b0 = lsm + st + tbase0;
        b16 = lsm + st + tbase16;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          Frag<bf16_t> fa[FM], fb[4];
#pragma unroll
          for (int mi = 0; mi < FM; ++mi) {
            const int ol = wm * 16 * FM + 16 * mi;
            fa[mi] = trfrag((ol >> 5) * 4096, kb, ol & 31);
          }
#pragma unroll
          for (int nj = 0; nj < 4; ++nj) {
            const int kl = wn * 64 + 16 * nj;
            fb[nj] = trfrag((FM + (kl >> 5)) * 4096, kb, kl & 31);
          }
#pragma unroll
          for (int mi = 0; mi < FM; ++mi)
#pragma unroll
            for (int nj = 0; nj < 4; ++nj) mma(acc[mi][nj], fa[mi], fb[nj]);
        }
        const int ahead = (nst - 1 < s + Cfg::S - 1 ? nst - 1 : s + Cfg::S - 1) - (s + 1);
        if (ahead >= 2) vm_wait_barrier<2 * Cfg::PER>();
        else if (ahead == 1) vm_wait_barrier<Cfg::PER>();
        else vm_wait_barrier<0>();
      }
      float* dst = a.partial + ((long long)(wi / ntile) * a.Cout) * KK;
#pragma unroll
      for (int mi = 0; mi < FM; ++mi)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int o = o0 + wm * 16 * FM + 16 * mi + 4 * g + reg;
#pragma unroll
          for (int nj = 0; nj < 4; ++nj) {
            const int c = kk0 + wn * 64 + 16 * nj + r;
            if (o < a.Cout && c < KK) dst[(long long)o * KK + c] = acc[mi][nj][reg];
          }
        }
      __syncthreads();  // staged ids / masks and the ring are free for the next work unit
    }
  };
#pragma unroll
  for (int l = 0; l < NL; ++l)
    if (l < L.n) run_leg(L.a[l]);
  if (!L.fold) return;
  float2(*red)[32] = reinterpret_cast<float2(*)[32]>(smem);  // the ring is free: every wave left the loop
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    if (l >= L.n) break;
    const WgArgs& a = L.a[l];
    const int hwo = a.ho * a.wo, nsp = chan_sum_splits(hwo), ncb = (a.Cout + 63) / 64;
    const int nunit = a.B * ncb * nsp;
    for (;;) {
      __syncthreads();
      if (tid == 0) *next_s = __hip_atomic_fetch_add(a.counts + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int u = *next_s;
      if (u >= nunit) break;  // uniform: every thread read the same slot
      const int b = u % a.B, cb = (u / a.B) % ncb, sp = u / (a.B * ncb);
      chan_sum_body(a.gout, hwo, a.Cout, a.B, b, cb, sp, nsp, L.csum[l], red);
    }
  }
}

// dW_k (per item partials) -> the reference filters, fixed summation order (items in list
// order: codes ascending, units ascending).
struct CombArgs {
  const float* partial;
  const int4* items;
  const int* counts;
  int Cin, Cout;
  float* dconv_w;
  float* dproj_w;
  const float* csum;
  const rgbd_decomp_info* info;
  int B, nsplit;
  float* dbias;
};
// One block per (output channel o, 32-channel chunk of the input): 72 threads each own four
// consecutive kk of one tap and walk the items in list order (the summation order of the former
// one-block-per-row combine, so the same bits), the chunk's five [9 tap][32 c] rows are parked in LDS (5.6 KB) and written back as five
// contiguous (c, tap) runs of 288 floats.  A block is small, so many are resident per CU and the
// partial reads stream at HBM speed (the per-row form needs 5 x 9 Cin floats of LDS per block:
// two blocks per CU).  Blocks of chunk 0 also write o's bias gradients.  grid (Cin / 32, Cout, legs).
constexpr int FOLD_C = 32, FOLD_T = 128;
__device__ __forceinline__ void fold_body(const CombArgs& A, int o, int c0, float (*srow)[9 * FOLD_C]) {
  const float* __restrict__ partial = A.partial;
  const int4* __restrict__ items = A.items;
  const int Cin = A.Cin, Cout = A.Cout, KK = 9 * Cin, ni = A.counts[1];
  const int t = threadIdx.x;
  if (t < 9 * FOLD_C / 4) {
    const int tap = t / (FOLD_C / 4), q = t % (FOLD_C / 4);
    const long long kk = (long long)tap * Cin + c0 + 4 * q;
    const float* src = partial + (long long)o * KK + kk;
    const long long istr = (long long)Cout * KK;
    float4 seg[4], pr = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < 4; ++i) seg[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    auto acc = [&](const float4 v, int k) {
      pr.x += v.x; pr.y += v.y; pr.z += v.z; pr.w += v.w;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if ((k >> i) & 1) {
          seg[i].x += v.x; seg[i].y += v.y; seg[i].z += v.z; seg[i].w += v.w;
        }
    };
    int it = 0;
    for (; it + 8 <= ni; it += 8) {
      float4 v[8];
      int k[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[j] = *reinterpret_cast<const float4*>(src + (it + j) * istr);
        k[j] = items[it + j].x;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc(v[j], k[j]);
    }
    for (; it < ni; ++it) acc(*reinterpret_cast<const float4*>(src + it * istr), items[it].x);
    const int r = tap * FOLD_C + 4 * q;
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<float4*>(&srow[i][r]) = seg[i];
    *reinterpret_cast<float4*>(&srow[4][r]) = pr;
  }
  __syncthreads();
  // OIHW: element (o, c0 + c, tap) at o * KK + (c0 + c) * 9 + tap — a contiguous run per filter
  for (int e = t; e < 5 * 9 * FOLD_C; e += FOLD_T) {
    const int i = e / (9 * FOLD_C), f = e % (9 * FOLD_C), c = f / 9, tap = f % 9;
    const float v = srow[i][tap * FOLD_C + c];
    if (i < 4)
      A.dconv_w[((long long)i * Cout + o) * KK + (long long)c0 * 9 + f] = v;
    else
      A.dproj_w[(long long)o * KK + (long long)c0 * 9 + f] = v;
  }
  // o's bias gradients (csum [nsplit][B][Cout]; conv_layers[i] only where i < len(masks)): the
  // former combine's wave sums, waves 0 / 1 taking i = 0, 2 / 1, 3
  if (c0 == 0 && A.dbias) {
    const int wv = t >> 6, lane = t & 63;
    for (int i = wv; i < 4; i += FOLD_T / 64) {
      float sb = 0.f;
      for (int q = lane; q < A.nsplit * A.B; q += 64) {
        const int b = q % A.B;
        if (i < A.info[b].n_masks) sb += A.csum[(long long)q * Cout + o];
      }
      sb = wave_sum(sb);
      if (lane == 0) A.dbias[i * Cout + o] = sb;
    }
  }
}
__global__ __launch_bounds__(FOLD_T) void k_dsam_wgrad_fold(const CombArgs A0, const CombArgs A1) {
  __shared__ __attribute__((aligned(16))) float srow[5][9 * FOLD_C];
  const CombArgs& A = blockIdx.z == 0 ? A0 : A1;
  if ((int)blockIdx.y >= A.Cout || (int)blockIdx.x * FOLD_C >= A.Cin) return;  // block-uniform
  fold_body(A, blockIdx.y, blockIdx.x * FOLD_C, srow);
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

__global__ __launch_bounds__(256) void k_chan_sum_nhwc(const bf16_t* __restrict__ g, int HW, int C,
                                                       float* __restrict__ out) {
  __shared__ float2 red[8][32];
  chan_sum_body(g, HW, C, gridDim.x, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.z, out, red);
}

__global__ __launch_bounds__(256) void k_dsam_bias_grad(const float* __restrict__ csum, const rgbd_decomp_info* info,
                                                        int B, int Cout, int nsplit, float* __restrict__ dbias) {
  // csum [nsplit][B][Cout] channel sums (per-pixel-range partials).  One wave per (i, o): lanes
  // over (split, b) pairs, fixed-order wave tree: deterministic.
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;  // t = (i, o)
  if (t >= 4 * Cout) return;
  const int i = t / Cout, o = t % Cout;
  float s = 0.f;
  for (int q = lane; q < nsplit * B; q += 64) {
    const int b = q % B;
    if (i < info[b].n_masks) s += csum[(long long)q * Cout + o];  // conv_layers[i] used only if i < len(masks)
  }
  s = wave_sum(s);
  if (lane == 0) dbias[t] = s;
}

// ----------------------------------------------------------------------- bf16: code-merged
// The masked sum  sum_i conv_i(x * m_i) + proj(x)  is regrouped by region CODE (the 4-bit
// pooled mask pattern of a source pixel, bit i = m_i): a source pixel with code k meets the
// merged filter  W_k = proj + sum_{i in k} conv_i  (packed per code by k_pack_fwd_codes), so
// each im2col row is multiplied by ONE filter instead of popcount(k) + 1 of them.  Rows are
// output pixels flattened over batch x grid (forward) or over one stride-2 parity class of the
// input grid (dX, where only the taps of that class are live).

// Code-merged masked conv, bf16 (fwd and dX).  Workgroup = 8 waves (2 along M x 4 along N),
// tile 8 x 16 output pixels (128 rows) x 192 columns, wave tile 64 x 48 (4 x 3 MFMA 16x16x32).
// Steps run over (tap, group of KC 32-channel chunks, region code present among the tile's
// rows at that tap); each step's operands arrive by LDS-DMA in an S-stage ring, S-1 steps ahead:
//   A  the 128 im2col rows x KC*64 B (a row whose tap falls outside the input re-reads an
//      in-bounds pixel of its own row; rows whose code differs from the step's code, or whose
//      tap is outside, are zeroed in registers after the fragment read);
//   B  the KC contiguous 192-row x 64-B tiles of the packed W_code (k_pack_fwd_codes /
//      k_pack_bwd_codes layout): linear copies.
// Load balance: a tile's step count is 9 x (codes per tap) x chunk groups, 1x..5x a dense tile
// on real scenes (region boundaries), so k_dsam_plan records each tile's per-tap code sets
// and the tile's steps are cut into nc = ceil(steps / chunk_len) equal chunks, one workgroup
// each; the last chunk of a multi-chunk tile to finish sums the f32 partials in chunk order.
constexpr int LD_BM = 128, LD_BN = 192, LD_CH = 8;  // tile rows, tile columns, max chunks per tile
constexpr int LD_MAXSTEP = 2048;    // steps of one tile (9 taps x 16 codes x chunk groups)
constexpr int LD_A1 = LD_BM * 64;   // 8 KB per chunk
constexpr int LD_B1 = LD_BN * 64;   // 12 KB per chunk
template <int KC>
struct LdCfg {
  static constexpr int S = KC == 3 ? 2 : (KC == 2 ? 3 : 6);  // ring depth the LDS admits
  static constexpr int A = KC * LD_A1;
  static constexpr int STAGE = KC * (LD_A1 + LD_B1);
  static constexpr int ROWTAB = S * STAGE;                // [128] int4 row table
  static constexpr int ROWOUT = ROWTAB + LD_BM * 16;      // [128] int4 NCHW base, NHWC pixel, n_masks
  static constexpr int TMASK = ROWOUT + LD_BM * 16;       // [9] u32 code set per tap, [9][16] u8 code list
  static constexpr int BSUM = TMASK + 64 + 160;           // [5][192] f32 bias prefix sums
  static constexpr int STEPTAB = BSUM + 5 * LD_BN * 4;    // [LD_MAXSTEP] int: tap | cg << 4 | code << 12
  static constexpr size_t SMEM = STEPTAB + LD_MAXSTEP * 4;
  static_assert(SMEM <= 163840, "LDS budget");
};
constexpr int LD_EPI_LD = LD_BM + 4;  // epilogue LDS tile [96 n][132] f32 (two halves)

struct LdGeom {
  int py, px, Hc, Wc, nyl, nxl, ntap, tiles_x, tiles_y, ntiles;
};
__device__ __forceinline__ LdGeom ld_geom(const ConvArgs& a, int cls) {
  LdGeom G;
  G.py = G.px = 0;
  G.Hc = a.Ho;
  G.Wc = a.Wo;
  if (a.transposed) {
    G.py = cls >> 1;
    G.px = cls & 1;
    G.Hc = (a.Ho - G.py + 1) >> 1;
    G.Wc = (a.Wo - G.px + 1) >> 1;
  }
  G.nyl = a.transposed ? (G.py ? 2 : 1) : 3;
  G.nxl = a.transposed ? (G.px ? 2 : 1) : 3;
  G.ntap = G.nyl * G.nxl;
  G.tiles_x = (G.Wc + 15) >> 4;
  G.tiles_y = (G.Hc + 7) >> 3;
  G.ntiles = a.linear ? (int)(((long long)a.B * G.Hc * G.Wc + LD_BM - 1) / LD_BM) : a.B * G.tiles_x * G.tiles_y;
  return G;
}
// live tap t of the class -> kernel tap (ky, kx) and source offset (dy, dx) from the row origin
__device__ __forceinline__ void ld_tap(const ConvArgs& a, const LdGeom& G, int t, int& ky, int& kx, int& dy,
                                       int& dx) {
  const int iy = t / G.nxl, ix = t - iy * G.nxl;
  if (a.transposed) {
    ky = G.py ? 2 * iy : 1;
    kx = G.px ? 2 * ix : 1;
    dy = (G.py + 1 - ky) >> 1;
    dx = (G.px + 1 - kx) >> 1;
  } else {
    ky = dy = iy;
    kx = dx = ix;
  }
}
// Row ml of tile `tile`: pixel (ty*8 + ml/16, tx*16 + ml%16) of the class grid.  Returns whether
// the row exists; org = origin pixel of its taps, rv = in-bounds taps, lo/hi = 4-bit code per tap.
__device__ __forceinline__ bool ld_row(const ConvArgs& a, const LdGeom& G, int tile, int ml, int& b, int& i,
                                       int& j, int& org, uint32_t& rv, uint32_t& lo, uint32_t& hi) {
  int iq, jq;
  if (a.linear) {  // row ml = pixel tile * 128 + ml of the batch's (class) grid
    const int hw = G.Hc * G.Wc, m = tile * LD_BM + ml;
    b = m / hw;
    const int rem = m - b * hw;
    iq = rem / G.Wc;
    jq = rem - iq * G.Wc;
  } else {
    b = tile / (G.tiles_x * G.tiles_y);
    const int trem = tile - b * G.tiles_x * G.tiles_y;
    iq = (trem / G.tiles_x) * 8 + (ml >> 4);
    jq = (trem % G.tiles_x) * 16 + (ml & 15);
  }
  const bool mv = b < a.B && iq < G.Hc && jq < G.Wc;
  b = mv ? b : 0;
  i = mv ? iq : 0;
  j = mv ? jq : 0;
  rv = lo = hi = 0u;
  uint32_t cv[9];
  if (a.transposed) {
    const uint32_t rc = a.code[((long long)b * a.Ho + 2 * i + G.py) * a.Wo + 2 * j + G.px];
    org = mv ? (b * a.Hi + i) * a.Wi + j : 0;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      int ky, kx, dy, dx;
      ld_tap(a, G, t < G.ntap ? t : 0, ky, kx, dy, dx);
      if (mv && t < G.ntap && i + dy < a.Hi && j + dx < a.Wi) rv |= 1u << t;
      cv[t] = rc;
    }
  } else {
    org = mv ? (b * a.Hi + 2 * i - 1) * a.Wi + 2 * j - 1 : 0;
    int off[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = 2 * i - 1 + t / 3, ix = 2 * j - 1 + t % 3;
      const bool inb = mv && iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi;
      if (inb) rv |= 1u << t;
      off[t] = inb ? org + (t / 3) * a.Wi + t % 3 : 0;
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) cv[t] = a.code[off[t]];
  }
#pragma unroll
  for (int t = 0; t < 9; ++t)
    if ((rv >> t) & 1u) {
      const uint32_t c = cv[t] & 15u;
      if (t < 8) lo |= c << (4 * t); else hi |= c;
    }
  return mv;
}
__device__ __forceinline__ int ld_steps(const uint16_t* tm, int ntap, int ncg) {
  int s = 0;
  for (int t = 0; t < ntap; ++t) s += __popc((uint32_t)tm[t]) * ncg;
  return s;
}
__device__ __forceinline__ int ld_nchunks(int steps, int len) {
  const int n = (steps + len - 1) / len;
  return n < 1 ? 1 : (n > LD_CH ? LD_CH : n);
}

// Plan: per (class, tile) the set of region codes the tile's rows meet at each live tap,
// tmasks[(cls * ntiles0 + tile) * 16 + t] (u16).  One 128-thread workgroup per tile.
__device__ __forceinline__ void plan_tile(const ConvArgs& a, int cls, int tile, int ntn) {
  __shared__ uint32_t tm_s[9];
  const int ntiles0 = a.ntiles0, tid = threadIdx.x;
  const LdGeom G = ld_geom(a, cls);
  if (tile >= G.ntiles) return;
  if (tid < 9) tm_s[tid] = 0u;
  __syncthreads();
  int b, i, j, org;
  uint32_t rv, lo, hi;
  ld_row(a, G, tile, tid, b, i, j, org, rv, lo, hi);
  uint32_t tm[5] = {0u, 0u, 0u, 0u, 0u};
#pragma unroll
  for (int t = 0; t < 9; ++t)
    if ((rv >> t) & 1u) {
      const uint32_t c = (t < 8 ? lo >> (4 * t) : hi) & 15u;
      tm[t >> 1] |= (1u << c) << (16 * (t & 1));
    }
#pragma unroll
  for (int q = 0; q < 5; ++q)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) tm[q] |= (uint32_t)__shfl_xor((int)tm[q], o);
  if ((tid & 63) == 0)
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const uint32_t v = (tm[t >> 1] >> (16 * (t & 1))) & 0xffffu;
      if (v) atomicOr(&tm_s[t], v);
    }
  __syncthreads();
  if (tid < 16) a.tmasks[((long long)cls * ntiles0 + tile) * 16 + tid] = tid < 9 ? (uint16_t)tm_s[tid] : 0;
  if (cls == 0 && tile == 0 && tid < LD_ZERO_BYTES / 16)
    reinterpret_cast<uint4*>(const_cast<bf16_t*>(a.zero))[tid] = make_uint4(0u, 0u, 0u, 0u);
  for (int q = tid; q < ntn; q += 128) a.tickets[((long long)cls * ntiles0 + tile) * ntn + q] = 0;
  if (cls == 0 && tile == 0 && tid < ntn) a.work[tid] = 0;
}

// Several conv legs planned by one launch (the forward cascade's three DSAMs and the two dX
// legs, right after the decomposition): blockIdx.z runs over (leg, class), blockIdx.x over tiles.
constexpr int PLAN_MAXLEG = 8;
struct PlanLegs {
  ConvArgs a[PLAN_MAXLEG];
  int zb[PLAN_MAXLEG + 1];  // first z of each leg
  int ntn[PLAN_MAXLEG];
  int n;
};
__global__ __launch_bounds__(128) void k_dsam_plan(const PlanLegs L) {
  const int z = blockIdx.z;
  int leg = 0;
  while (leg + 1 < L.n && z >= L.zb[leg + 1]) ++leg;
  plan_tile(L.a[leg], z - L.zb[leg], blockIdx.x, L.ntn[leg]);
}

// Work list: per (class, tile) the chunk count, compacted into items (cls | chunk << 2 |
// tile << 5) in (class, tile, chunk) order by one workgroup; a[*nitems] = count.  dX lists the
// parity classes by decreasing live-tap count (3: 4 taps, 1 and 2: 2, 0: 1), so the longest
// items are taken first under the dynamic assignment.
__device__ __forceinline__ void items_body(const ConvArgs& a) {
  __shared__ int wsum[16];
  __shared__ int base_s;
  const int ntiles0 = a.ntiles0, ncg = a.ncg;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nclass = a.transposed ? 4 : 1, total = nclass * ntiles0;
  if (tid == 0) base_s = 0;
  __syncthreads();
  for (int e0 = 0; e0 < total; e0 += 1024) {
    const int e = e0 + tid;
    int nc = 0;
    if (e < total) {
      const int ce = e / ntiles0, tile = e - ce * ntiles0;
      const int cls = a.transposed ? (0x0213 >> (4 * ce)) & 15 : ce;  // class order 3, 1, 2, 0
      const LdGeom G = ld_geom(a, cls);
      if (tile < G.ntiles)
        nc = ld_nchunks(ld_steps(a.tmasks + ((long long)cls * ntiles0 + tile) * 16, G.ntap, ncg), a.chunk_len);
    }
    // block exclusive scan of nc
    int x = nc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int before = base_s;
    for (int q = 0; q < w; ++q) before += wsum[q];
    const int off = before + x - nc;
    if (e < total) {
      const int ce = e / ntiles0, tile = e - ce * ntiles0;
      const int cls = a.transposed ? (0x0213 >> (4 * ce)) & 15 : ce;  // class order 3, 1, 2, 0
      for (int c = 0; c < nc; ++c) a.items[off + c] = cls | (c << 2) | (tile << 5);
    }
    __syncthreads();
    if (tid == 1023) base_s = off + nc;
    __syncthreads();
  }
  if (tid == 0) *a.nitems = base_s;
}
__global__ __launch_bounds__(1024) void k_dsam_items(const PlanLegs L) { items_body(L.a[blockIdx.x]); }

// Diagnostics (rgbd_debug_dsam_stamps): the STAMPS instantiation of k_dsam_lds has wave 0 of every
// workgroup record, for its first LD_STAMP_ITEMS items, s_memtime at: item taken, prologue tables
// built, first DMA landed, K loop done, partial hand-off done (or the early return of a non-last
// chunk), epilogue done; then the item's steps | chunks << 16 | chunk << 24 and the item word:
// stamps[(wg * LD_STAMP_ITEMS + k) * 8 + field].  The production instantiation has none of it.
constexpr int LD_STAMP_ITEMS = 4;
__device__ __forceinline__ void ld_stamp(unsigned long long* st, int f) {
  if (!st) return;
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) st[f] = t;
  __builtin_amdgcn_sched_barrier(0);
}

// NODMA (diagnostic build only, rgbd_debug_dsam_mode; timing only, the results are garbage):
// bit 0 drops the in-loop B copies, bit 1 the in-loop A copies, bit 2 the per-step barrier (each
// wave still waits for its own copies), bit 3 the fragment reads (constant MFMA operands); bit 5
// copies every step's weights from its code's first filter tile and bit 6 every step's input rows from
// one fixed pixel block (the copies stay, their sources become L2-resident: the ceiling of
// locality work).
// One (tile, chunk) item of k_dsam_lds for N tile ntile (of ntn).
template <int KC, int NODMA = 0>
__device__ __forceinline__ void ld_item(const ConvArgs& a, int cls, int tile, int chunk, int ntile, int ntn,
                                        int* next_s, int nitems, unsigned long long* st = nullptr) {
  using Cfg = LdCfg<KC>;
  constexpr int S = Cfg::S;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  int4* rowtab = (int4*)(smem + Cfg::ROWTAB);
  int4* rowout = (int4*)(smem + Cfg::ROWOUT);
  float* bsum = (float*)(smem + Cfg::BSUM);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int wm = wave & 1, wn = wave >> 1;
  const LdGeom G = ld_geom(a, cls);
  const int ncg = a.C / (32 * KC);  // chunk groups
  const uint16_t* tmg = a.tmasks + ((long long)cls * a.ntiles0 + tile) * 16;
  // the tile's 16 u16 code sets in two 16-byte loads (one round trip; per-element loads behind
  // `t < ntap` were nine serialized ones, most of the item's table time)
  uint32_t tmask[9];
  {
    const uint4 q0 = reinterpret_cast<const uint4*>(tmg)[0], q1 = reinterpret_cast<const uint4*>(tmg)[1];
    const uint32_t w[5] = {q0.x, q0.y, q0.z, q0.w, q1.x};
#pragma unroll
    for (int t = 0; t < 9; ++t) tmask[t] = t < G.ntap ? (w[t >> 1] >> (16 * (t & 1))) & 0xffffu : 0u;
  }
  int tb[10];
  tb[0] = 0;
#pragma unroll
  for (int t = 0; t < 9; ++t) tb[t + 1] = tb[t] + __popc(tmask[t]) * ncg;
  const int total = tb[9];
  const int nc = ld_nchunks(total, a.chunk_len);
  const int n0 = ntile * LD_BN;
  const bf16_t* xp = (const bf16_t*)a.x;
  const bf16_t* wp = (const bf16_t*)a.w;
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  // ---- prologue: row table (threads 0..127), code lists per tap (the N tile's bias prefix sums
  // were built once per workgroup by k_dsam_lds)
  // step table, tap major, then chunk group, then code (ascending): one thread per (tap, chunk
  // group) writes its run from registers (no LDS round trips)
  for (int q = tid; q < G.ntap * ncg; q += 512) {
    const int t = q / ncg, cg = q - t * ncg;
    uint32_t msk = 0u;
    int e = 0;
#pragma unroll
    for (int u = 0; u < 9; ++u) {
      if (u == t) msk = tmask[u];
      if (u < t) e += __popc(tmask[u]) * ncg;
    }
    e += cg * __popc(msk);
    int* steptab = (int*)(smem + Cfg::STEPTAB);
    while (msk) {
      steptab[e++] = t | (cg << 4) | ((__ffs(msk) - 1) << 12);
      msk &= msk - 1u;
    }
  }
  if (tid < LD_BM) {
    int b, i, j, org;
    uint32_t rv, lo, hi;
    const bool mv = ld_row(a, G, tile, tid, b, i, j, org, rv, lo, hi);
    rowtab[tid] = make_int4(org, (int)rv, (int)lo, (int)hi);
    int obase = -1, opix = 0, nmk = 0;
    if (mv) {
      const int oy = a.transposed ? 2 * i + G.py : i, ox = a.transposed ? 2 * j + G.px : j;
      opix = (b * a.Ho + oy) * a.Wo + ox;
      obase = (b * a.N * a.Ho + oy) * a.Wo + ox;
      nmk = a.info ? a.info[b].n_masks : 0;
    }
    rowout[tid] = make_int4(obase, opix, nmk, 0);
  }
  __syncthreads();
  ld_stamp(st, 1);
  // DMA role: A rows 16*wave + lane/4 of every chunk, slot lane%4.  A row that is outside the
  // input at the step's tap, or whose source code is not the step's code, is read from the zero
  // row instead: it contributes exactly zero, with no masking of fragments in registers.
  const int R = 16 * wave + (lane >> 2);
  int aorg, achk;
  uint32_t aval, alo, ahi;
  {
    const int4 e = rowtab[R];
    aorg = e.x;
    aval = (uint32_t)e.y;
    alo = (uint32_t)e.z;
    ahi = (uint32_t)e.w;
    achk = 8 * ((lane & 3) ^ lds_swz(R));
  }
  const int* steptab = (const int*)(smem + Cfg::STEPTAB);
  const bf16_t* zrow = a.zero + achk;
  const int s0 = (int)((long long)chunk * total / nc), s1 = (int)((long long)(chunk + 1) * total / nc);
  const int nst = s1 - s0;
  if (st && threadIdx.x == 0) st[6] = (unsigned long long)(nst | (nc << 16) | (chunk << 24));
  auto issue = [&](int slot, int s, bool inloop = false) {  // step s (absolute)
    const int e = __builtin_amdgcn_readfirstlane(steptab[s]);
    const int t = e & 15, cg = (e >> 4) & 255, code = e >> 12;
    int ky, kx, dy, dx;
    ld_tap(a, G, t, ky, kx, dy, dx);
    const int delta = dy * a.Wi + dx, tap = ky * 3 + kx;
    const uint32_t sb = lds0 + slot * Cfg::STAGE;
    const uint32_t rc = (t < 8 ? alo >> (4 * t) : ahi) & 15u;
    const bool live = ((aval >> t) & 1u) && rc == (uint32_t)code;
    const bf16_t* asrc = live ? xp + (long long)(aorg + delta) * a.C + cg * 32 * KC + achk : zrow;
    if constexpr ((NODMA & 64) != 0)  // timing only: every step's rows from one fixed 128-pixel block
      if (inloop) asrc = xp + (long long)R * a.C + achk;
    if (!((NODMA & 2) && inloop))
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) dma_lds16(live ? asrc + kc * 32 : zrow, sb + kc * LD_A1 + wave * 1024);
    if ((NODMA & 1) && inloop) return;
    const long long tstride = (long long)a.N * 32;  // one (code, tap, chunk) tile, elements
    const bf16_t* bsrc = wp + ((long long)(code * 9 + tap) * (a.C / 32) + cg * KC) * tstride + (long long)n0 * 32 + lane * 8;
    if constexpr ((NODMA & 32) != 0)  // timing only: every step's weights from its code's first tile
      if (inloop) bsrc = wp + (long long)(code * 9) * (a.C / 32) * tstride + (long long)n0 * 32 + lane * 8;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const bf16_t* tbk = bsrc + kc * tstride;
      const uint32_t db = sb + Cfg::A + kc * LD_B1;
      dma_lds16(tbk + wave * 512, db + wave * 1024);
      if (wave < 4) dma_lds16(tbk + (wave + 8) * 512, db + (wave + 8) * 1024);
    }
  };
  const int cnt = KC * (wave < 4 ? 3 : 2);  // DMA instructions of this wave per step
  f32x4 acc[4][3];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int nj = 0; nj < 3; ++nj) acc[mi][nj] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int npro = nst < S - 1 ? nst : S - 1;
  for (int i = 0; i < npro; ++i) issue(i, s0 + i);
  if (npro >= 2) vm_wait_barrier_dyn((npro - 1) * cnt);  // step 0 landed, later ones may fly
  else vm_wait_barrier<0>();
  ld_stamp(st, 2);
#pragma unroll 1
  for (int s = 0; s < nst; ++s) {
    if (s + S - 1 < nst) issue((s + S - 1) % S, s0 + s + S - 1, true);
    const char* sa = smem + (s % S) * Cfg::STAGE;
    // fragments of chunk kc+1 are read while chunk kc's 12 MFMAs run
    Frag<bf16_t> fa[2][4], fb[2][3];
    auto rd = [&](int kc, int q) {
      if constexpr (NODMA & 8) {
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) fa[q][mi].v = make_uint4(lane, kc, s, mi);
#pragma unroll
        for (int nj = 0; nj < 3; ++nj) fb[q][nj].v = make_uint4(nj, lane, kc, s);
        return;
      }
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int row = wm * 64 + 16 * mi + r;
        fa[q][mi].v = *reinterpret_cast<const uint4*>(sa + kc * LD_A1 + row * 64 + 16 * (g ^ lds_swz(row)));
      }
#pragma unroll
      for (int nj = 0; nj < 3; ++nj) {
        const int row = wn * 48 + 16 * nj + r;
        fb[q][nj].v = *reinterpret_cast<const uint4*>(sa + Cfg::A + kc * LD_B1 + row * 64 + 16 * (g ^ lds_swz(row)));
      }
    };
    rd(0, 0);
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      if (kc + 1 < KC) rd(kc + 1, (kc + 1) & 1);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < 3; ++nj) mma(acc[mi][nj], fa[kc & 1][mi], fb[kc & 1][nj]);
    }
    // own DMA of step s+1 landed (only later steps' may stay in flight), LDS reads done, barrier
    const int ahead = (nst - 1 < s + S - 1 ? nst - 1 : s + S - 1) - (s + 1);
    if constexpr (NODMA & 4) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else if (ahead <= 0) vm_wait_barrier<0>();
    else vm_wait_barrier_dyn(ahead * cnt);
  }
  ld_stamp(st, 3);
  // the workgroup's next item, taken now so the counter and work-list reads overlap the hand-off
  // and the epilogue; published in LDS at every exit (k_dsam_lds's barrier orders it)
  int nxt = 0, nxv = 0;
  bool have = false;
  if (tid == 0) nxt = __hip_atomic_fetch_add(a.work + ntile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  auto fetch_word = [&] {  // the next item's work-list word (waits for the counter)
    if (tid == 0 && !have) {
      nxv = nxt < nitems ? a.items[nxt] : 0;
      have = true;
    }
  };
  auto publish = [&] {
    fetch_word();
    if (tid == 0) {
      next_s[0] = nxt;
      next_s[1] = nxv;
    }
  };
  if (nc > 1) {
    // Multi-chunk tile: publish this chunk's fragment-native partial ([wave][mi][nj][lane][4] f32),
    // take a ticket; the chunk that draws nc-1 sums all partials in chunk order (deterministic)
    // and runs the epilogue.  The hand-off is write-through: every partial byte is stored and
    // loaded sc1 (16 B per lane, through one wave-uniform buffer descriptor), every storing wave
    // drains, one lane per workgroup adds to the tile's ticket after the barrier, and only the
    // workgroup whose add returned nc-1 loads (MI355X_MICROARCH.md, visibility table row 1;
    // cdna_hip_programming.md Guideline 16).  No agent-scope release (an XCD-wide L2 write-back)
    // or acquire is needed, and the result is correct for any placement of the chunks.
    const long long tslab = (((long long)cls * a.ntiles0 + tile) * ntn + ntile) * LD_CH;
    const __amdgpu_buffer_rsrc_t prs = wt_rsrc(a.partial + tslab * (LD_BN * LD_BM), LD_CH * LD_BN * LD_BM * 4);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int nj = 0; nj < 3; ++nj)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[mi][nj]), prs,
                                               (chunk * (LD_BN * LD_BM) + (((wave * 4 + mi) * 3 + nj) * 64 + lane) * 4) * 4,
                                               0, WT_SC1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* last_s = (int*)(smem + Cfg::TMASK);
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(a.tickets + tslab / LD_CH, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last_s = old == nc - 1;
    }
    __syncthreads();
    if (!*last_s) {
      ld_stamp(st, 4);
      publish();
      return;
    }
    // every partial of the tile in flight at once, then summed in chunk order
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int nj = 0; nj < 3; ++nj) acc[mi][nj] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < nc; ++c) {
      u32x4 pv[4][3];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < 3; ++nj)
          pv[mi][nj] = __builtin_amdgcn_raw_buffer_load_b128(
              prs, (c * (LD_BN * LD_BM) + (((wave * 4 + mi) * 3 + nj) * 64 + lane) * 4) * 4, 0, WT_SC1);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < 3; ++nj) acc[mi][nj] += __builtin_bit_cast(f32x4, pv[mi][nj]);
    }
  }
  ld_stamp(st, 4);
  // ---- epilogue (same contract as k_conv_igemm), staged through LDS in two 96-column halves:
  // pass 1 runs along pixels (NCHW residual loads and stores), pass 2 along channels (NHWC);
  // every thread's loads of a pass are independent and issued together.
  if (!a.out_nchw) {
    // NHWC-only epilogue (the hot path's forward cascade and dX): one pass.  The accumulators go
    // to an LDS image [128 rows][196] f32 (rows = tile pixels; the 4-float pad makes the 4 rows
    // a wave writes per register land on disjoint banks), then each thread owns 6 (row, 8-channel)
    // items: all six 16-byte NHWC residual loads in flight together, two 16-byte LDS reads, the
    // bias sum of the row's image, res + (acc + bias) rounded once, one 16-byte store.
    constexpr int LDE = LD_BN + 4;
    constexpr int NCH = LD_BN / 8;
    constexpr int NIT = LD_BM * NCH / 512;
    static_assert(LD_BM * LDE * 4 <= Cfg::ROWTAB, "epilogue image must not overlap the row tables");
    float* et = (float*)smem;
    const bf16_t* rnhwc = (const bf16_t*)a.residual_nhwc;
    bf16_t* onhwc = (bf16_t*)a.out_nhwc;
    uint4 rv[NIT];  // residual loads first: in flight while the accumulators go through LDS
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int it = tid + 512 * i, ml = it / NCH, n = n0 + 8 * (it % NCH);
      const int4 ro = rowout[ml];
      rv[i] = make_uint4(0u, 0u, 0u, 0u);
      if (rnhwc && ro.x >= 0 && n < a.N) rv[i] = *reinterpret_cast<const uint4*>(rnhwc + (long long)ro.y * a.N + n);
    }
    __syncthreads();  // ring reads done
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int nj = 0; nj < 3; ++nj)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg)
          et[(wm * 64 + 16 * mi + 4 * g + reg) * LDE + wn * 48 + 16 * nj + r] = acc[mi][nj][reg];
    __syncthreads();
    fetch_word();
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int it = tid + 512 * i, ml = it / NCH, nl = 8 * (it % NCH), n = n0 + nl;
      const int4 ro = rowout[ml];
      if (ro.x < 0 || n >= a.N) continue;
      const float4 e0 = *reinterpret_cast<const float4*>(et + ml * LDE + nl);
      const float4 e1 = *reinterpret_cast<const float4*>(et + ml * LDE + nl + 4);
      float v[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
      const uint32_t uw[4] = {rv[i].x, rv[i].y, rv[i].z, rv[i].w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bsum[ro.z * LD_BN + nl + e];
      if (rnhwc)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] = __uint_as_float(uw[e] << 16) + v[2 * e];
          v[2 * e + 1] = __uint_as_float(uw[e] & 0xffff0000u) + v[2 * e + 1];
        }
      *reinterpret_cast<uint4*>(onhwc + (long long)ro.y * a.N + n) =
          make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
    }
    ld_stamp(st, 5);
    publish();
    return;
  }
  float* et = (float*)smem;  // [96 n][LD_EPI_LD] f32
  const bf16_t* res = (const bf16_t*)a.residual;
  bf16_t* onchw = (bf16_t*)a.out_nchw;
  bf16_t* onhwc = (bf16_t*)a.out_nhwc;
  const long long HoWo = (long long)a.Ho * a.Wo;
  constexpr int HN = LD_BN / 2;
  for (int half = 0; half < 2; ++half) {
    __syncthreads();  // ring reads / previous half done
    if ((wn >> 1) == half)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < 3; ++nj)
#pragma unroll
          for (int reg = 0; reg < 4; ++reg)
            et[((wn & 1) * 48 + 16 * nj + r) * LD_EPI_LD + wm * 64 + 16 * mi + 4 * g + reg] = acc[mi][nj][reg];
    __syncthreads();
    const int nh = n0 + half * HN;
    if (onchw) {
    // pass 1: items (channel, 4 consecutive tile rows = 4 consecutive pixels of one tile row);
    // forward rows are contiguous in NCHW (8-byte residual loads / stores), dX rows are not
    constexpr int NQ = HN * LD_BM / 4 / 512;  // 6 items per thread
    float4 rq[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {  // residual loads, all in flight
      const int it = tid + 512 * q, nl = it / (LD_BM / 4), ml = (it % (LD_BM / 4)) * 4, n = nh + nl;
      rq[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!res || n >= a.N) continue;
      const int4 r0 = rowout[ml], r3 = rowout[ml + 3];
      const long long o = r0.x + (long long)n * HoWo;
      if (!a.transposed && r0.x >= 0 && r3.x == r0.x + 3) {
        const uint2 u = *reinterpret_cast<const uint2*>(res + o);
        rq[q] = make_float4(bf16_to_f32((bf16_t)u.x), bf16_to_f32((bf16_t)(u.x >> 16)), bf16_to_f32((bf16_t)u.y),
                            bf16_to_f32((bf16_t)(u.y >> 16)));
      } else {
        float t4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int4 re = rowout[ml + e];
          t4[e] = re.x >= 0 ? bf16_to_f32(res[re.x + (long long)n * HoWo]) : 0.f;
        }
        rq[q] = make_float4(t4[0], t4[1], t4[2], t4[3]);
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int it = tid + 512 * q, nl = it / (LD_BM / 4), ml = (it % (LD_BM / 4)) * 4, n = nh + nl;
      if (n >= a.N) continue;
      const float rr[4] = {rq[q].x, rq[q].y, rq[q].z, rq[q].w};
      bf16_t tv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int4 re = rowout[ml + e];
        float v = et[nl * LD_EPI_LD + ml + e] + bsum[re.z * LD_BN + half * HN + nl];
        if (res) v = rr[e] + v;
        tv[e] = f32_to_bf16(v);
        et[nl * LD_EPI_LD + ml + e] = bf16_to_f32(tv[e]);
      }
      if (onchw) {
        const int4 r0 = rowout[ml], r3 = rowout[ml + 3];
        if (!a.transposed && r0.x >= 0 && r3.x == r0.x + 3) {
          *reinterpret_cast<uint2*>(onchw + r0.x + (long long)n * HoWo) =
              make_uint2((uint32_t)tv[0] | ((uint32_t)tv[1] << 16), (uint32_t)tv[2] | ((uint32_t)tv[3] << 16));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int4 re = rowout[ml + e];
            if (re.x >= 0) onchw[re.x + (long long)n * HoWo] = tv[e];
          }
        }
      }
    }
    }  // pass 1
    if (onhwc) {
      // pass 2: items (tile row, 8 consecutive channels) -> one 16-byte store.  Consecutive lanes
      // take consecutive tile rows of the same 8 channels, so the LDS column reads are
      // conflict-free.  Without pass 1 (no NCHW output: the bf16 dX of the hot path) the bias
      // and the NHWC residual are added here, in pass 1's order: res + (acc + bias), rounded once.
      __syncthreads();
      const bool fused = !onchw;
      const bf16_t* rnhwc = (const bf16_t*)a.residual_nhwc;
      for (int it = tid; it < LD_BM * (HN / 8); it += 512) {
        const int ml = it % LD_BM, nl = (it / LD_BM) * 8, n = nh + nl;
        const int4 ro = rowout[ml];
        if (ro.x < 0 || n >= a.N) continue;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = et[(nl + e) * LD_EPI_LD + ml];
        if (fused) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += bsum[ro.z * LD_BN + half * HN + nl + e];
          if (rnhwc) {
            const uint4 u = *reinterpret_cast<const uint4*>(rnhwc + (long long)ro.y * a.N + n);
            const uint32_t uw[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[2 * e] = __uint_as_float(uw[e] << 16) + v[2 * e];
              v[2 * e + 1] = __uint_as_float(uw[e] & 0xffff0000u) + v[2 * e + 1];
            }
          }
        }
        *reinterpret_cast<uint4*>(onhwc + (long long)ro.y * a.N + n) =
            make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
      }
    }
  }
  ld_stamp(st, 5);
  publish();
}

// Persistent: grid (workgroups, N tiles); each workgroup takes the next item of its N tile's list
// from a counter (items differ up to ~5x in steps: dynamic assignment balances the tail; the
// multi-chunk reductions stay in chunk order, so results do not depend on who ran what).
template <int KC, bool STAMPS = false, int NODMA = 0>
__global__ __launch_bounds__(512, 1) void k_dsam_lds(ConvArgs a) {
  using Cfg = LdCfg<KC>;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  if constexpr (NODMA != 0) {  // the ring starts zeroed: slots the modes never fill hold finite values
    for (int e = threadIdx.x; e < Cfg::S * Cfg::STAGE / 16; e += 512)
      reinterpret_cast<uint4*>(smem)[e] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
  }
  int* next_s = (int*)(smem + Cfg::TMASK + 216);  // free bytes behind the per-tap code lists: item, word
  const int nitems = *a.nitems;
  const int ntile = blockIdx.y;
  {  // the N tile's bias prefix sums over the four conv biases, kept for every item
    float* bsum = (float*)(smem + Cfg::BSUM);
    const int n0 = ntile * LD_BN;
    for (int e = threadIdx.x; e < 5 * LD_BN; e += 512) {
      const int k = e / LD_BN, nl = e - k * LD_BN, n = n0 + nl;
      float s = 0.f;
      if (a.bias4 && n < a.N)
        for (int sb = 0; sb < k; ++sb) s += a.bias4[sb * a.N + n];
      bsum[e] = s;
    }
  }
  if (threadIdx.x == 0) {
    const int it = __hip_atomic_fetch_add(a.work + ntile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    next_s[0] = it;
    next_s[1] = it < nitems ? a.items[it] : 0;
  }
  int done = 0;
  for (;;) {
    unsigned long long* st = nullptr;
    if constexpr (STAMPS) {
      if (done < LD_STAMP_ITEMS)
        st = a.stamps + ((long long)(blockIdx.x + blockIdx.y * gridDim.x) * LD_STAMP_ITEMS + done) * 8;
      ++done;
    }
    __syncthreads();  // next_s published (first item: above; later: by the previous item)
    const int it = next_s[0], v = next_s[1];
    if (it >= nitems) break;  // workgroup-uniform
    ld_stamp(st, 0);
    if (st && threadIdx.x == 0) st[7] = (unsigned long long)v;
    // next_s is rewritten only after the item's K loop, behind its prologue barrier
    ld_item<KC, NODMA>(a, v & 3, v >> 5, (v >> 2) & 7, ntile, gridDim.y, next_s, nitems, st);
  }
}


long long conv_mmax(const ConvArgs& a) {
  return a.transposed ? (long long)a.B * ((a.Ho + 1) / 2) * ((a.Wo + 1) / 2) : (long long)a.B * a.Ho * a.Wo;
}
// chunks per step: three where C allows (two-stage ring).  Two (three-stage ring) measured slower
// (round 4: 2 300 cycles per 64-channel step vs 2 840 per 96-channel step; K5 0.707 vs 0.676 ms):
// the step is bound by LDS traffic (fragment reads + DMA writes), not by the DMA latency
int ld_kc(int C) { return C % 96 == 0 ? 3 : (C % 64 == 0 ? 2 : 1); }
// k_dsam_lds tiling of a conv: tiles of the largest parity class, N tiles
// Linear tiles when 8 x 16 blocks would leave more than 15 % of the rows dead (the small grids:
// dsam1 / dsam2 outputs, their dX parity classes)
int ld_linear(int Hc, int Wc) {
  const long long blk = (long long)((Hc + 7) / 8 * 8) * ((Wc + 15) / 16 * 16);
  return (long long)Hc * Wc * 100 < 85 * blk;
}
struct LdPlan {
  int ntiles0, ntn, kc, chunk_len, linear;
  size_t tmask_bytes, items_bytes, ticket_bytes, partial_bytes;
};
LdPlan ld_plan(const ConvArgs& a) {
  LdPlan p;
  const int Hc0 = a.transposed ? (a.Ho + 1) / 2 : a.Ho, Wc0 = a.transposed ? (a.Wo + 1) / 2 : a.Wo;
  const int nclass = a.transposed ? 4 : 1;
  p.linear = ld_linear(Hc0, Wc0);
  p.ntiles0 = p.linear ? (int)(((long long)a.B * Hc0 * Wc0 + LD_BM - 1) / LD_BM) : a.B * ((Hc0 + 7) / 8) * ((Wc0 + 15) / 16);
  p.ntn = ceil_div(a.N, LD_BN);
  p.kc = ld_kc(a.C);
  // chunk length in steps: one dense tile (one code per tap); 60 % and 150 % measured slower
  // (K5 0.74 / 0.78 vs 0.71 ms per step, round 3)
  const int ntap = a.transposed ? 4 : 9;  // class 3 of dX has 4 live taps
  p.chunk_len = std::max(1, ntap * (a.C / (32 * p.kc)));
  p.tmask_bytes = align256((size_t)nclass * p.ntiles0 * 16 * sizeof(uint16_t));
  p.items_bytes = align256(((size_t)nclass * p.ntiles0 * LD_CH + 1) * sizeof(int));
  p.ticket_bytes = align256((size_t)(nclass * p.ntiles0 * p.ntn + 64) * sizeof(int)) + LD_ZERO_BYTES;  // + work counters
  p.partial_bytes = align256((size_t)nclass * p.ntiles0 * p.ntn * LD_CH * LD_BN * LD_BM * sizeof(float));
  return p;
}
size_t ld_plan_bytes(const LdPlan& p) { return p.tmask_bytes + p.items_bytes + p.ticket_bytes; }
size_t v2_partial_bytes(const ConvArgs& a) {
  const LdPlan p = ld_plan(a);
  return ld_plan_bytes(p) + p.partial_bytes;
}
// The bf16 launch arguments of a conv leg over its plan buffer [code sets | work list | tickets,
// counters, zero row] (ld_plan_bytes) and its partial-tile buffer (P.partial_bytes).
ConvArgs conv_carve(const ConvArgs& a, const LdPlan& P, char* plan, float* partial) {
  ConvArgs b = a;
  const int nclass = a.transposed ? 4 : 1;
  b.tmasks = (uint16_t*)plan;
  b.items = (int*)(plan + P.tmask_bytes);
  b.nitems = b.items + (size_t)nclass * P.ntiles0 * LD_CH;
  b.tickets = (int*)(plan + P.tmask_bytes + P.items_bytes);
  b.work = b.tickets + (size_t)nclass * P.ntiles0 * P.ntn;
  b.zero = (const bf16_t*)(plan + ld_plan_bytes(P) - LD_ZERO_BYTES);  // the ticket region's tail
  b.partial = partial;
  b.ntiles0 = P.ntiles0;
  b.chunk_len = P.chunk_len;
  b.ncg = a.C / (32 * P.kc);
  b.linear = P.linear;
  return b;
}
bool conv_shape_ok(const ConvArgs& a, const LdPlan& P) {
  return a.C % 32 == 0 && a.N % 32 == 0 && (long long)a.B * a.Hi * a.Wi < (1ll << 31) && conv_mmax(a) < (1ll << 31) &&
         P.ntn <= 64 && 9 * 16 * (a.C / (32 * P.kc)) <= LD_MAXSTEP;
}
// plan + work list of n conv legs (two launches)
hipError_t plan_convs(int n, const ConvArgs* legs, hipStream_t s) {
  PlanLegs L = {};
  L.n = n;
  int z = 0, mt = 1;
  for (int i = 0; i < n; ++i) {
    L.a[i] = legs[i];
    L.zb[i] = z;
    L.ntn[i] = ceil_div(legs[i].N, LD_BN);
    z += legs[i].transposed ? 4 : 1;
    mt = std::max(mt, legs[i].ntiles0);
  }
  L.zb[n] = z;
  k_dsam_plan<<<dim3(mt, 1, z), 128, 0, s>>>(L);
  k_dsam_items<<<n, 1024, 0, s>>>(L);
  return hipGetLastError();
}

#ifdef RGBD_DIAG
// rgbd_debug_dsam_stamps (diagnostic build only): buffer, its capacity in launches, launches
// stamped so far
unsigned long long* g_ld_stamps = nullptr;
int g_ld_stamp_cap = 0, g_ld_stamp_n = 0;
int g_ld_mode = 0;  // rgbd_debug_dsam_mode: NODMA bits of the stamped KC = 3 instantiation
template <int KC, int M>
hipError_t launch_ld_stamped(const ConvArgs& c, dim3 grid, hipStream_t s) {
  static const hipError_t sattr = hipFuncSetAttribute((const void*)k_dsam_lds<KC, true, M>,
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)LdCfg<KC>::SMEM);
  if (sattr != hipSuccess) return sattr;
  k_dsam_lds<KC, true, M><<<grid, 512, LdCfg<KC>::SMEM, s>>>(c);
  return hipSuccess;
}
#endif
template <int KC>
hipError_t launch_ld(const ConvArgs& b, dim3 grid, hipStream_t s) {
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)k_dsam_lds<KC>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LdCfg<KC>::SMEM);
  if (attr != hipSuccess) return attr;
#ifdef RGBD_DIAG
  if (g_ld_stamps && g_ld_stamp_n < g_ld_stamp_cap && grid.x * grid.y <= 256) {
    ConvArgs c = b;
    c.stamps = g_ld_stamps + (size_t)g_ld_stamp_n++ * 256 * LD_STAMP_ITEMS * 8;
    if constexpr (KC == 3) {
      switch (g_ld_mode) {
        case 1: return launch_ld_stamped<KC, 1>(c, grid, s);
        case 2: return launch_ld_stamped<KC, 2>(c, grid, s);
        case 3: return launch_ld_stamped<KC, 3>(c, grid, s);
        case 7: return launch_ld_stamped<KC, 7>(c, grid, s);
        case 15: return launch_ld_stamped<KC, 15>(c, grid, s);
        case 32: return launch_ld_stamped<KC, 32>(c, grid, s);
        case 64: return launch_ld_stamped<KC, 64>(c, grid, s);
        case 96: return launch_ld_stamped<KC, 96>(c, grid, s);
        case 8: return launch_ld_stamped<KC, 8>(c, grid, s);
        default: break;
      }
    }
    return launch_ld_stamped<KC, 0>(c, grid, s);
  }
#endif
  k_dsam_lds<KC><<<grid, 512, LdCfg<KC>::SMEM, s>>>(b);
  return hipSuccess;
}

template <typename T>
int launch_conv(const ConvArgs& a, hipStream_t s, const void* planned = nullptr) {
  TimerScope ts(a.transposed ? "dsam_dx" : "dsam_fwd", s);
  int nclass = a.transposed ? 4 : 1;
  const long long Mmax = conv_mmax(a);
  if constexpr (sizeof(T) == 2) {
    // code-merged bf16 path: the plan (unless the caller planned this leg ahead with
    // rgbd_dsam_plan) into the head of the workspace, then the persistent kernel
    const LdPlan P = ld_plan(a);
    RGBD_REQUIRE(conv_shape_ok(a, P), RGBD_E_SHAPE);
    char* plan = planned ? (char*)planned : (char*)a.partial;
    float* partial = planned ? a.partial : (float*)((char*)a.partial + ld_plan_bytes(P));
    const ConvArgs b = conv_carve(a, P, plan, partial);
    if (!planned) {
      const hipError_t pe = plan_convs(1, &b, s);
      if (pe != hipSuccess) return (int)pe;
    }
    // persistent: about one workgroup per CU (LDS-bound) over all N tiles
    constexpr int pers = 256;  // persistent: one LDS-bound workgroup per CU
    dim3 grid2(std::max(1, pers / P.ntn), P.ntn, 1);
    const hipError_t e = P.kc == 3 ? launch_ld<3>(b, grid2, s) : P.kc == 2 ? launch_ld<2>(b, grid2, s) : launch_ld<1>(b, grid2, s);
    if (e != hipSuccess) return (int)e;
    RGBD_CHECK_LAUNCH();
    return RGBD_OK;
  }
  dim3 grid(ceil_div(Mmax, BM), ceil_div(a.N, BN), nclass);
  k_conv_igemm<T><<<grid, 256, 0, s>>>(a);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

// ---- bf16 dW: output tile (FM); items and their partials are sized by the device plan, the
// workspace by the worst case (every code live in every unit)
struct WgPlan {
  int fm, nunit, ntile_kk, ntile_o, max_entries;
};
int wg_fm(int Cout) { return Cout % 192 == 0 ? 6 : (Cout % 128 == 0 ? 4 : 2); }
static WgPlan wg_plan(int B, int Cin, int h, int w, int Cout) {
  WgPlan p;
  p.fm = wg_fm(Cout);
  const int hwo = ((h + 1) / 2) * ((w + 1) / 2);
  p.nunit = (hwo + WPX - 1) / WPX;
  p.ntile_kk = ceil_div(9ll * Cin, 128);
  p.ntile_o = ceil_div(Cout, 32 * p.fm);
  p.max_entries = 16 * B * p.nunit;
  return p;
}
// items are at most max_entries; the plan targets about one work unit per CU (every unit writes an
// f32 partial tile the combine re-reads, so more units cost more than the balance they buy): 256,
// 384 for layers with many output tiles (dsam2's 108: units of ~3 items balance better under the
// dynamic assignment), 192 for layers with few (dsam0's 7) — measured per layer at 640x480
static int wg_target(const WgPlan& p) {
  const int tiles = p.ntile_kk * p.ntile_o;
  return tiles >= 64 ? 384 : (tiles <= 8 ? 192 : 256);
}
// partial buffer bound: items <= entries / L + 16 with L >= entries / (target / tiles)
static size_t wg_max_items(const WgPlan& p) {
  const long long want = std::max(1, wg_target(p) / std::max(1, p.ntile_kk * p.ntile_o));
  return (size_t)std::min<long long>(p.max_entries, want + 16 + p.max_entries / WITEM_MAX);
}

template <int FM, int NL>
hipError_t launch_wg(const WgMulti<NL>& m, int grid, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute((const void*)k_dsam_wgrad_mm<FM, NL>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)WgCfg<FM>::SMEM);
  if (attr != hipSuccess) return attr;
  k_dsam_wgrad_mm<FM, NL><<<grid, 256, WgCfg<FM>::SMEM, s>>>(m);
  return hipSuccess;
}
template <int NL>
hipError_t launch_wg_fm(int fm, const WgMulti<NL>& m, hipStream_t s) {
  const int grid = 256;  // persistent: one LDS-bound workgroup per CU
  return fm == 6 ? launch_wg<6, NL>(m, grid, s) : fm == 4 ? launch_wg<4, NL>(m, grid, s) : launch_wg<2, NL>(m, grid, s);
}

int dsam_wgrad_splits(int B, int Cin, int Cout) {
  const long long tiles = (long long)ceil_div(45ll * Cin, 64) * ceil_div(Cout, 64);
  int sp = (int)std::min<long long>(B, std::max<long long>(1, ceil_div(1024, tiles)));
  return sp < 1 ? 1 : sp;
}


}  // namespace

extern "C" {

const char* rgbd_version(void) { return "rgbd_hip 0.1.0 (gfx950)"; }

int rgbd_nchw_to_nhwc(int dtype, const void* src, void* dst, int B, int C, int H, int W, void* stream) {
  RGBD_REQUIRE(src && dst && B > 0 && C > 0 && H > 0 && W > 0, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_BF16 && ((long long)H * W) % 8 == 0 && C % 8 == 0) {
    k_nchw_to_nhwc_v8<<<dim3(ceil_div((long long)H * W, 64), ceil_div(C, 64), B), 256, 0, s>>>(
        (const bf16_t*)src, (bf16_t*)dst, C, H * W);
    RGBD_CHECK_LAUNCH();
    return RGBD_OK;
  }
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

int rgbd_nchw_to_nhwc_multi(int n, const rgbd_nhwc_job* jobs, void* stream) {
  RGBD_REQUIRE(n >= 1 && n <= NHWC_MAXJOB && jobs, RGBD_E_ARG);
  NhwcJobs J;
  long long blocks = 0;
  for (int i = 0; i < n; ++i) {
    const rgbd_nhwc_job& q = jobs[i];
    RGBD_REQUIRE(q.src && q.dst && q.B > 0 && q.C > 0 && q.H > 0 && q.W > 0, RGBD_E_ARG);
    RGBD_REQUIRE(q.C % 8 == 0, RGBD_E_SHAPE);  // 16-byte NHWC stores
    J.src[i] = (const bf16_t*)q.src;
    J.dst[i] = (bf16_t*)q.dst;
    J.C[i] = q.C;
    J.HW[i] = q.H * q.W;
    J.tp[i] = ceil_div((long long)q.H * q.W, 64);
    J.tc[i] = ceil_div(q.C, 64);
    J.block0[i] = (int)blocks;
    blocks += (long long)q.B * J.tp[i] * J.tc[i];
  }
  RGBD_REQUIRE(blocks < (1ll << 31), RGBD_E_SHAPE);
  J.block0[n] = (int)blocks;
  J.n = n;
  k_nchw_to_nhwc_multi<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(J);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

long long rgbd_dsam_packed_elems(int dtype, int Cin, int Cout) {
  if (Cin <= 0 || Cout <= 0) return 0;
  if (dtype == RGBD_F32) return 45ll * Cin * Cout;
  if (dtype == RGBD_BF16) return 144ll * Cin * Cout + 192 * 32;  // + one-tile tail pad
  return 0;
}

int rgbd_dsam_code_masks(int n, const uint8_t* const* codes_host, const long long* nbytes_host, uint32_t* masks,
                         void* stream) {
  RGBD_REQUIRE(n > 0 && n <= 8 && codes_host && nbytes_host && masks, RGBD_E_ARG);
  CodeMaps cm = {};
  long long most = 1;
  for (int i = 0; i < n; ++i) {
    RGBD_REQUIRE(codes_host[i] && nbytes_host[i] > 0, RGBD_E_ARG);
    cm.p[i] = codes_host[i];
    cm.n[i] = nbytes_host[i];
    most = std::max(most, nbytes_host[i]);
  }
  hipStream_t s = (hipStream_t)stream;
  const hipError_t me = hipMemsetAsync(masks, 0, sizeof(uint32_t) * n, s);
  if (me != hipSuccess) return (int)me;
  k_code_masks<<<dim3((unsigned)std::min<long long>(ceil_div(most, 256 * 8), 256), n), 256, 0, s>>>(cm, masks);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_dsam_pack_weights(int dtype, const float* conv_w, const float* proj_w, int Cin, int Cout,
                           const uint32_t* code_mask, void* wfwd, void* wbwd, void* stream) {
  RGBD_REQUIRE(conv_w && proj_w && (wfwd || wbwd) && Cin > 0 && Cout > 0, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_F32) {
    const int nb = (int)std::min<long long>(ceil_div(45ll * Cin * Cout, 256), 4096);
    k_pack_dsam<float><<<nb, 256, 0, s>>>(conv_w, proj_w, Cin, Cout, (float*)wfwd, (float*)wbwd);
  } else if (dtype == RGBD_BF16) {
    RGBD_REQUIRE(wfwd, RGBD_E_ARG);  // wbwd is the transpose of wfwd
    RGBD_REQUIRE(Cin % PK_CB == 0 && Cout % 32 == 0, RGBD_E_SHAPE);
    static const hipError_t attr = hipFuncSetAttribute((const void*)k_pack_codes,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)PK_SMEM);
    if (attr != hipSuccess) return (int)attr;
    k_pack_codes<<<dim3(Cin / PK_CB, Cout / PK_OB), 256, PK_SMEM, s>>>(conv_w, proj_w, Cin, Cout, code_mask,
                                                                       (bf16_t*)wfwd, (bf16_t*)wbwd);
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
  return std::max<size_t>(256, std::max(v2_partial_bytes(f), v2_partial_bytes(d)));
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

static int fwd_nhwc(int dtype, const void* x_nhwc, const uint8_t* code, const rgbd_decomp_info* info, int B,
                    int Cin, int h, int w, int Cout, const void* wfwd, const float* bias, const void* residual_nhwc,
                    void* out_nhwc, const void* planned, void* ws, void* stream) {
  RGBD_REQUIRE(dtype == RGBD_BF16, RGBD_E_DTYPE);
  RGBD_REQUIRE(x_nhwc && code && info && wfwd && bias && out_nhwc && ws, RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && h > 0 && w > 0 && Cout > 0 && Cin > 0, RGBD_E_ARG);
  ConvArgs a = fwd_args(B, Cin, h, w, Cout);
  a.x = x_nhwc; a.code = code; a.w = wfwd;
  a.bias4 = bias; a.info = info; a.residual_nhwc = residual_nhwc; a.out_nhwc = out_nhwc;
  a.partial = (float*)ws;
  return launch_conv<bf16_t>(a, (hipStream_t)stream, planned);
}
int rgbd_dsam_fwd_nhwc(int dtype, const void* x_nhwc, const uint8_t* code, const rgbd_decomp_info* info,
                       int B, int Cin, int h, int w, int Cout, const void* wfwd, const float* bias,
                       const void* residual_nhwc, void* out_nhwc, void* ws, void* stream) {
  return fwd_nhwc(dtype, x_nhwc, code, info, B, Cin, h, w, Cout, wfwd, bias, residual_nhwc, out_nhwc, nullptr, ws,
                  stream);
}
int rgbd_dsam_fwd_nhwc_planned(int dtype, const void* x_nhwc, const uint8_t* code, const rgbd_decomp_info* info,
                               int B, int Cin, int h, int w, int Cout, const void* wfwd, const float* bias,
                               const void* residual_nhwc, void* out_nhwc, const void* plan, void* ws, void* stream) {
  RGBD_REQUIRE(plan, RGBD_E_ARG);
  return fwd_nhwc(dtype, x_nhwc, code, info, B, Cin, h, w, Cout, wfwd, bias, residual_nhwc, out_nhwc, plan, ws,
                  stream);
}

static int bwd_data(int dtype, const void* gout_nhwc, const uint8_t* code, int B, int Cin, int h, int w, int Cout,
                    const void* wbwd, const void* gin_nchw, const void* gin_nhwc, void* dx_nchw, void* dx_nhwc,
                    const void* planned, void* ws, void* stream) {
  RGBD_REQUIRE(!planned || dtype == RGBD_BF16, RGBD_E_DTYPE);
  RGBD_REQUIRE(gout_nhwc && code && wbwd && (dx_nchw || dx_nhwc), RGBD_E_ARG);
  // the residual comes in the layout of the pass that adds it: NCHW with an NCHW output, NHWC
  // (bf16 only) without one
  RGBD_REQUIRE(!gin_nhwc || (dtype == RGBD_BF16 && !dx_nchw && !gin_nchw), RGBD_E_ARG);
  RGBD_REQUIRE(!gin_nchw || dx_nchw, RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && h > 0 && w > 0 && Cout > 0 && Cin > 0, RGBD_E_ARG);
  RGBD_REQUIRE(Cout % 8 == 0, RGBD_E_SHAPE);
  ConvArgs a = dx_args(B, Cin, h, w, Cout);
  a.x = gout_nhwc; a.code = code; a.w = wbwd;
  a.residual = gin_nchw; a.residual_nhwc = gin_nhwc; a.out_nchw = dx_nchw; a.out_nhwc = dx_nhwc;
  a.partial = (float*)ws;
  RGBD_REQUIRE(ws || dtype != RGBD_BF16, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == RGBD_F32) return launch_conv<float>(a, s);
  if (dtype == RGBD_BF16) return launch_conv<bf16_t>(a, s, planned);
  return RGBD_E_DTYPE;
}
int rgbd_dsam_bwd_data(int dtype, const void* gout_nhwc, const uint8_t* code, int B, int Cin, int h,
                       int w, int Cout, const void* wbwd, const void* gin_nchw, const void* gin_nhwc,
                       void* dx_nchw, void* dx_nhwc, void* ws, void* stream) {
  return bwd_data(dtype, gout_nhwc, code, B, Cin, h, w, Cout, wbwd, gin_nchw, gin_nhwc, dx_nchw, dx_nhwc, nullptr, ws,
                  stream);
}
int rgbd_dsam_bwd_data_planned(int dtype, const void* gout_nhwc, const uint8_t* code, int B, int Cin, int h,
                               int w, int Cout, const void* wbwd, const void* gin_nchw, const void* gin_nhwc,
                               void* dx_nchw, void* dx_nhwc, const void* plan, void* ws, void* stream) {
  RGBD_REQUIRE(plan, RGBD_E_ARG);
  return bwd_data(dtype, gout_nhwc, code, B, Cin, h, w, Cout, wbwd, gin_nchw, gin_nhwc, dx_nchw, dx_nhwc, plan, ws,
                  stream);
}

// bf16 workspace: the plan part [presence table [B][units] u16 | live entry list | their tap
// masks | items | counters | zero row] (plan_total bytes; rgbd_dsam_plan can fill it ahead),
// then [items][Cout][9 Cin] f32 partials | channel sums
struct WgradWs {
  size_t pres, gmask, list, masks, items, counts, zero, plan_total, partial, csum, total;
};
static WgradWs wgrad_ws(int dtype, int B, int Cin, int h, int w, int Cout) {
  WgradWs o;
  size_t off = 0;
  size_t part, npres = 1, nent = 1, nitems = 1;
  if (dtype == RGBD_BF16) {
    const WgPlan p = wg_plan(B, Cin, h, w, Cout);
    nitems = wg_max_items(p);
    part = nitems * Cout * 9 * Cin;
    npres = (size_t)B * p.nunit;
    nent = p.max_entries;
  } else {
    part = (size_t)dsam_wgrad_splits(B, Cin, Cout) * Cout * 45 * Cin;
  }
  o.pres = off;
  off += align256(sizeof(uint16_t) * npres);
  o.gmask = off;
  off += 256;
  o.list = off;
  off += align256(sizeof(int) * nent);
  o.masks = off;
  off += align256(sizeof(unsigned long long) * 9 * nent);
  o.items = off;
  off += align256(sizeof(int4) * nitems);
  o.counts = off;
  off += 256;
  o.zero = off;
  off += LD_ZERO_BYTES;
  o.plan_total = off;
  o.partial = off;
  off += align256(sizeof(float) * part);
  o.csum = off;
  off += align256(sizeof(float) * (size_t)CS_SPLIT_MAX * B * Cout);
  o.total = off;
  return o;
}

// dW launch arguments over a plan part (wgrad_ws offsets below plan_total) and the partials
static WgArgs wg_args(const WgradWs& L, const WgPlan& P, char* plan, float* partial, const void* gout_nhwc,
                      const void* x_nhwc, const uint8_t* code, int B, int Cin, int h, int w, int Cout) {
  WgArgs a;
  a.gout = (const bf16_t*)gout_nhwc;
  a.x = (const bf16_t*)x_nhwc;
  a.code = code;
  a.pres = (uint16_t*)(plan + L.pres);
  a.list = (int*)(plan + L.list);
  a.masks = (unsigned long long*)(plan + L.masks);
  a.items = (int4*)(plan + L.items);
  a.counts = (int*)(plan + L.counts);
  a.B = B; a.Cin = Cin; a.h = h; a.w = w; a.Cout = Cout;
  a.ho = (h + 1) / 2; a.wo = (w + 1) / 2;
  a.nunit = P.nunit;
  a.ntile_kk = P.ntile_kk;
  a.ntile_o = P.ntile_o;
  a.target = wg_target(P);
  a.inv_wo = 1.0f / (float)a.wo;
  a.zero = (const bf16_t*)(plan + L.zero);
  a.partial = partial;
  return a;
}
static bool wg_shape_ok(int B, int Cin, int h, int w, int Cout, const WgPlan& P) {
  const long long hwo = (long long)((h + 1) / 2) * ((w + 1) / 2);
  return Cin % 32 == 0 && Cout % 32 == 0 && hwo < (1ll << 22) && (long long)B * h * w < (1ll << 31) &&
         (long long)B * P.nunit < (1 << 24);
}
// the code-dependent part of n dW legs: unit presence, the per-code live lists and items, tap
// masks — three launches for all legs
static void wg_plan_launch(int n, const WgArgs* a, const WgPlan* P, hipStream_t s) {
  WgLegs L = {};
  L.n = n;
  long long pres_blocks = 1, mask_blocks = 1;
  for (int i = 0; i < n; ++i) {
    L.a[i] = a[i];
    L.max_entries[i] = P[i].max_entries;
    pres_blocks = std::max<long long>(pres_blocks, ceil_div((long long)a[i].B * P[i].nunit * 64, 256));
    mask_blocks = std::max<long long>(mask_blocks, ceil_div((long long)P[i].max_entries, 4));
  }
  k_code_presence_legs<<<dim3((unsigned)pres_blocks, 1, n), 256, 0, s>>>(L);
  k_wg_plan_legs<<<dim3(1, 1, n), 1024, 0, s>>>(L);
  k_wg_masks_legs<<<dim3((unsigned)mask_blocks, 1, n), 256, 0, s>>>(L);
}

size_t rgbd_dsam_bwd_weight_workspace_size(int dtype, int B, int Cin, int h, int w, int Cout) {
  if (B <= 0 || h <= 0 || w <= 0 || Cin <= 0 || Cout <= 0) return 256;
  return wgrad_ws(dtype, B, Cin, h, w, Cout).total;
}

static CombArgs comb_args(const WgArgs& a, bool nchw_sums, const float* csum, const rgbd_decomp_info* info,
                          float* dconv_w, float* dproj_w, float* dbias) {
  CombArgs c;
  c.partial = a.partial;
  c.items = a.items;
  c.counts = a.counts;
  c.Cin = a.Cin;
  c.Cout = a.Cout;
  c.dconv_w = dconv_w;
  c.dproj_w = dproj_w;
  c.csum = csum;
  c.info = info;
  c.B = a.B;
  c.nsplit = nchw_sums ? 1 : chan_sum_splits(a.ho * a.wo);
  c.dbias = dbias;
  return c;
}

// bf16 dW after the GEMM: the upstream gradient's channel sums (bias), then the combine of the
// item partials into the reference filters (it also writes the bias gradients)
static int wg_finish(const WgArgs& a, const void* gout_nchw, float* csum, const rgbd_decomp_info* info,
                     float* dconv_w, float* dproj_w, float* dbias, hipStream_t s, bool sums_folded) {
  const int hwo = a.ho * a.wo;
  if (gout_nchw)
    k_chan_sum<bf16_t><<<a.B * a.Cout, 256, 0, s>>>((const bf16_t*)gout_nchw, hwo, csum);
  else if (!sums_folded)
    k_chan_sum_nhwc<<<dim3(a.B, ceil_div(a.Cout, 64), chan_sum_splits(hwo)), 256, 0, s>>>(a.gout, hwo, a.Cout, csum);
  RGBD_REQUIRE(a.Cin % FOLD_C == 0, RGBD_E_SHAPE);
  const CombArgs c = comb_args(a, gout_nchw != nullptr, csum, info, dconv_w, dproj_w, dbias);
  k_dsam_wgrad_fold<<<dim3(a.Cin / FOLD_C, a.Cout, 1), FOLD_T, 0, s>>>(c, c);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

static int bwd_weight(int dtype, const void* gout_nchw, const void* gout_nhwc, const void* x_nhwc,
                      const uint8_t* code, const rgbd_decomp_info* info, int B, int Cin, int h, int w, int Cout,
                      float* dconv_w, float* dproj_w, float* dbias, const void* planned, void* ws, void* stream) {
  RGBD_REQUIRE((gout_nchw || dtype == RGBD_BF16) && x_nhwc && code && info && dconv_w && dproj_w && dbias && ws,
               RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && h > 0 && w > 0 && Cout > 0 && Cin > 0, RGBD_E_ARG);
  RGBD_REQUIRE(Cin % 8 == 0, RGBD_E_SHAPE);
  hipStream_t s = (hipStream_t)stream;
  const WgradWs L = wgrad_ws(dtype, B, Cin, h, w, Cout);
  // planned ahead: ws holds only [partials | channel sums]
  const size_t run0 = planned ? L.plan_total : 0;
  float* partial = (float*)((char*)ws + L.partial - run0);
  float* csum = (float*)((char*)ws + L.csum - run0);
  TimerScope ts("dsam_wgrad", s);
  const int ho = (h + 1) / 2, wo = (w + 1) / 2, hwo = ho * wo;
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
    RGBD_REQUIRE(gout_nhwc, RGBD_E_ARG);
    const WgPlan P = wg_plan(B, Cin, h, w, Cout);
    RGBD_REQUIRE(wg_shape_ok(B, Cin, h, w, Cout, P), RGBD_E_SHAPE);
    char* plan = planned ? (char*)planned : (char*)ws;
    WgMulti<1> m;
    m.a[0] = wg_args(L, P, plan, partial, gout_nhwc, x_nhwc, code, B, Cin, h, w, Cout);
    m.n = 1;
    m.csum[0] = csum;
    m.fold = gout_nchw == nullptr;  // NHWC bias sums drained by the GEMM's workgroups
    if (!planned) wg_plan_launch(1, &m.a[0], &P, s);
    const hipError_t e = launch_wg_fm(P.fm, m, s);
    if (e != hipSuccess) return (int)e;
    return wg_finish(m.a[0], gout_nchw, csum, info, dconv_w, dproj_w, dbias, s, m.fold);
  } else {
    return RGBD_E_DTYPE;
  }
  const int nsplit = (dtype == RGBD_BF16 && !gout_nchw) ? chan_sum_splits(hwo) : 1;
  k_dsam_bias_grad<<<Cout, 256, 0, s>>>(csum, info, B, Cout, nsplit, dbias);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_dsam_bwd_weight(int dtype, const void* gout_nchw, const void* gout_nhwc, const void* x_nhwc,
                         const uint8_t* code, const rgbd_decomp_info* info, int B, int Cin, int h, int w,
                         int Cout, float* dconv_w, float* dproj_w, float* dbias, void* ws, void* stream) {
  return bwd_weight(dtype, gout_nchw, gout_nhwc, x_nhwc, code, info, B, Cin, h, w, Cout, dconv_w, dproj_w, dbias,
                    nullptr, ws, stream);
}
int rgbd_dsam_bwd_weight_planned(int dtype, const void* gout_nchw, const void* gout_nhwc, const void* x_nhwc,
                                 const uint8_t* code, const rgbd_decomp_info* info, int B, int Cin, int h, int w,
                                 int Cout, float* dconv_w, float* dproj_w, float* dbias, const void* plan, void* ws,
                                 void* stream) {
  RGBD_REQUIRE(plan && dtype == RGBD_BF16, RGBD_E_ARG);
  return bwd_weight(dtype, gout_nchw, gout_nhwc, x_nhwc, code, info, B, Cin, h, w, Cout, dconv_w, dproj_w, dbias,
                    plan, ws, stream);
}

int rgbd_dsam_bwd_weight_planned_multi(int n, const rgbd_dsam_dw_run* runs, const rgbd_decomp_info* info,
                                       void* stream) {
  RGBD_REQUIRE(n >= 1 && n <= 2 && runs && info, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  TimerScope ts("dsam_wgrad", s);
  WgMulti<2> m;
  int fm[2];
  m.fold = 1;
  for (int i = 0; i < n; ++i) {
    const rgbd_dsam_dw_run& r = runs[i];
    RGBD_REQUIRE(r.gout_nhwc && r.x_nhwc && r.code && r.dconv_w && r.dproj_w && r.dbias && r.plan && r.ws, RGBD_E_ARG);
    RGBD_REQUIRE(r.B > 0 && r.h > 0 && r.w > 0 && r.Cout > 0 && r.Cin > 0 && r.Cin % 8 == 0, RGBD_E_SHAPE);
    const WgradWs L = wgrad_ws(RGBD_BF16, r.B, r.Cin, r.h, r.w, r.Cout);
    const WgPlan P = wg_plan(r.B, r.Cin, r.h, r.w, r.Cout);
    RGBD_REQUIRE(wg_shape_ok(r.B, r.Cin, r.h, r.w, r.Cout, P), RGBD_E_SHAPE);
    float* partial = (float*)((char*)r.ws + L.partial - L.plan_total);
    m.a[i] = wg_args(L, P, (char*)r.plan, partial, r.gout_nhwc, r.x_nhwc, r.code, r.B, r.Cin, r.h, r.w, r.Cout);
    m.csum[i] = (float*)((char*)r.ws + L.csum - L.plan_total);
    fm[i] = P.fm;
  }
  for (int i = 0; i + 1 < n; ++i)  // distinct buffers: the legs run together
    RGBD_REQUIRE(runs[i].ws != runs[i + 1].ws && runs[i].plan != runs[i + 1].plan, RGBD_E_ARG);
  hipError_t e;
  if (n == 2 && fm[0] == fm[1]) {
    m.n = 2;
    e = launch_wg_fm(fm[0], m, s);
  } else {  // one leg, or tile shapes that differ: one launch per leg
    e = hipSuccess;
    for (int i = 0; i < n && e == hipSuccess; ++i) {
      WgMulti<1> one;
      one.a[0] = m.a[i];
      one.csum[0] = m.csum[i];
      one.n = 1;
      one.fold = 1;
      e = launch_wg_fm(fm[i], one, s);
    }
  }
  if (e != hipSuccess) return (int)e;
  if (n == 1)  // the bias sums were drained by the GEMM's workgroups (fold)
    return wg_finish(m.a[0], nullptr, m.csum[0], info, runs[0].dconv_w, runs[0].dproj_w, runs[0].dbias, s, true);
  // both legs' folds in one launch
  RGBD_REQUIRE(runs[0].Cin % FOLD_C == 0 && runs[1].Cin % FOLD_C == 0, RGBD_E_SHAPE);
  CombArgs c[2];
  for (int i = 0; i < 2; ++i)
    c[i] = comb_args(m.a[i], false, m.csum[i], info, runs[i].dconv_w, runs[i].dproj_w, runs[i].dbias);
  k_dsam_wgrad_fold<<<dim3(std::max(runs[0].Cin, runs[1].Cin) / FOLD_C, std::max(runs[0].Cout, runs[1].Cout), 2),
                      FOLD_T, 0, s>>>(c[0], c[1]);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}


// ---- planning ahead (bf16): the code-dependent set-up of a leg depends only on the region codes,
// so the hot path plans every leg of the step once, right after the decomposition
static ConvArgs leg_conv_args(const rgbd_dsam_leg& g) {
  ConvArgs a = g.kind == RGBD_LEG_FWD ? fwd_args(g.B, g.Cin, g.h, g.w, g.Cout) : dx_args(g.B, g.Cin, g.h, g.w, g.Cout);
  a.code = g.code;
  return a;
}
static bool leg_ok(const rgbd_dsam_leg& g) {
  return (g.kind == RGBD_LEG_FWD || g.kind == RGBD_LEG_DX || g.kind == RGBD_LEG_DW) && g.B > 0 && g.h > 0 &&
         g.w > 0 && g.Cin > 0 && g.Cout > 0;
}
size_t rgbd_dsam_plan_size(int kind, int B, int Cin, int h, int w, int Cout) {
  const rgbd_dsam_leg g = {kind, nullptr, B, Cin, h, w, Cout, nullptr};
  if (!leg_ok(g)) return 0;
  if (kind == RGBD_LEG_DW) return wgrad_ws(RGBD_BF16, B, Cin, h, w, Cout).plan_total;
  return ld_plan_bytes(ld_plan(leg_conv_args(g)));
}
size_t rgbd_dsam_run_workspace_size(int kind, int B, int Cin, int h, int w, int Cout) {
  const rgbd_dsam_leg g = {kind, nullptr, B, Cin, h, w, Cout, nullptr};
  if (!leg_ok(g)) return 0;
  if (kind == RGBD_LEG_DW) {
    const WgradWs L = wgrad_ws(RGBD_BF16, B, Cin, h, w, Cout);
    return L.total - L.plan_total;
  }
  return std::max<size_t>(256, ld_plan(leg_conv_args(g)).partial_bytes);
}
#ifdef RGBD_DIAG
int rgbd_debug_dsam_stamps(void* buf, int launches) {
  RGBD_REQUIRE(buf ? launches > 0 : launches == 0, RGBD_E_ARG);  // (NULL, 0) stops
  g_ld_stamps = (unsigned long long*)buf;
  g_ld_stamp_cap = buf ? launches : 0;
  g_ld_stamp_n = 0;
  return RGBD_OK;
}
int rgbd_debug_dsam_mode(int mode) {
  RGBD_REQUIRE(mode == 0 || mode == 1 || mode == 2 || mode == 3 || mode == 7 || mode == 8 || mode == 15 || mode == 32 ||
                   mode == 64 || mode == 96,
               RGBD_E_ARG);
  g_ld_mode = mode;
  return RGBD_OK;
}
#endif

int rgbd_dsam_plan(int n, const rgbd_dsam_leg* legs, void* stream) {
  RGBD_REQUIRE(n > 0 && legs, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  ConvArgs conv[PLAN_MAXLEG];
  WgArgs wga[WG_MAXLEG];
  WgPlan wgp[WG_MAXLEG];
  int nconv = 0, nwg = 0;
  for (int i = 0; i < n; ++i) {
    const rgbd_dsam_leg& g = legs[i];
    RGBD_REQUIRE(leg_ok(g) && g.code && g.plan, RGBD_E_ARG);
    if (g.kind == RGBD_LEG_DW) {
      RGBD_REQUIRE(nwg < WG_MAXLEG, RGBD_E_ARG);
      const WgPlan P = wg_plan(g.B, g.Cin, g.h, g.w, g.Cout);
      RGBD_REQUIRE(wg_shape_ok(g.B, g.Cin, g.h, g.w, g.Cout, P), RGBD_E_SHAPE);
      const WgradWs L = wgrad_ws(RGBD_BF16, g.B, g.Cin, g.h, g.w, g.Cout);
      wgp[nwg] = P;
      wga[nwg++] = wg_args(L, P, (char*)g.plan, nullptr, nullptr, nullptr, g.code, g.B, g.Cin, g.h, g.w, g.Cout);
      continue;
    }
    RGBD_REQUIRE(nconv < PLAN_MAXLEG, RGBD_E_ARG);
    const ConvArgs a = leg_conv_args(g);
    const LdPlan P = ld_plan(a);
    RGBD_REQUIRE(conv_shape_ok(a, P), RGBD_E_SHAPE);
    conv[nconv++] = conv_carve(a, P, (char*)g.plan, nullptr);
  }
  if (nconv) {
    const hipError_t e = plan_convs(nconv, conv, s);
    if (e != hipSuccess) return (int)e;
  }
  if (nwg) wg_plan_launch(nwg, wga, wgp, s);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
