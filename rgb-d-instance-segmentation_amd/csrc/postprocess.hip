// f4: Mask2FormerImageProcessor.post_process_instance_segmentation on the device (transformers
// 5.15 image_processing_mask2former.py:627-744), as the reference's process_prediction calls it
// (mask2former/predictor.py:697-700) with target_sizes = the original image sizes.
//
// Per image (Q queries, C classes + no-object):
//   scores = softmax(class logits)[:, :C] (Q*C)     -> k_pp_topk: one workgroup; the top-Q
//     in the order ATen's CPU topk(sorted=False) leaves them: libstdc++ std::nth_element
//     (introselect) over (value, index) pairs, restated step for step on one lane over LDS
//     (oracle/postprocess.py pins the restatement against torch.topk itself)
//   masks = bilinear (align_corners=False) of the selected queries' logits to 384 x 384
//     -> k_pp_masks: one workgroup per selected entry: binary mask (logit > 0) as a bitmap,
//     mask score = sum(sigmoid * binary) / (sum(binary) + 1e-6), pred score = score * mask score
//   target size: nearest resize of the bitmaps (ATen's legacy 'nearest' index rule), an entry is
//     kept when its resized mask is non-empty and its pred score >= threshold; kept entries get
//     consecutive segment ids in top-k order and later entries overwrite earlier ones
//     -> k_pp_keep (one workgroup per entry) + k_pp_paint (per target pixel: the last kept entry
//     covering it), float32 map initialised to -1 like the reference.
#include "common.hpp"

using namespace rgbd;

namespace {

constexpr int PP_S = 384;                  // HF's fixed intermediate size
constexpr int PP_WORDS = PP_S * PP_S / 64;  // u64 words of one bitmap

// libstdc++ nth_element on parallel LDS arrays (value, index); comp = greater with NaN first.
struct Sel {
  float* v;
  int* ix;
  __device__ bool comp(int a, int b) const {
    const float x = v[a], y = v[b];
    return (x != x && y == y) || x > y;
  }
  __device__ bool comp_val(int a, float val) const {
    const float x = v[a];
    return (x != x && val == val) || x > val;
  }
  __device__ bool comp_val2(float val, int b) const {
    const float y = v[b];
    return (val != val && y == y) || val > y;
  }
  __device__ void swap(int a, int b) {
    const float tv = v[a];
    v[a] = v[b];
    v[b] = tv;
    const int ti = ix[a];
    ix[a] = ix[b];
    ix[b] = ti;
  }
  __device__ void move_median_to_first(int result, int a, int b, int c) {
    if (comp(a, b)) {
      if (comp(b, c)) swap(result, b);
      else if (comp(a, c)) swap(result, c);
      else swap(result, a);
    } else if (comp(a, c)) {
      swap(result, a);
    } else if (comp(b, c)) {
      swap(result, c);
    } else {
      swap(result, b);
    }
  }
  __device__ int unguarded_partition(int first, int last, int pivot) {
    while (true) {
      while (comp(first, pivot)) ++first;
      --last;
      while (comp(pivot, last)) --last;
      if (!(first < last)) return first;
      swap(first, last);
      ++first;
    }
  }
  __device__ void push_heap(int first, int hole, int top, float val, int vix) {
    int parent = (hole - 1) / 2;
    while (hole > top && comp_val(first + parent, val)) {
      v[first + hole] = v[first + parent];
      ix[first + hole] = ix[first + parent];
      hole = parent;
      parent = (hole - 1) / 2;
    }
    v[first + hole] = val;
    ix[first + hole] = vix;
  }
  __device__ void adjust_heap(int first, int hole, int len, float val, int vix) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
      second = 2 * (second + 1);
      if (comp(first + second, first + second - 1)) --second;
      v[first + hole] = v[first + second];
      ix[first + hole] = ix[first + second];
      hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
      second = 2 * (second + 1);
      v[first + hole] = v[first + second - 1];
      ix[first + hole] = ix[first + second - 1];
      hole = second - 1;
    }
    push_heap(first, hole, top, val, vix);
  }
  __device__ void heap_select(int first, int middle, int last) {
    const int len = middle - first;
    if (len >= 2)
      for (int parent = (len - 2) / 2;; --parent) {
        adjust_heap(first, parent, len, v[first + parent], ix[first + parent]);
        if (parent == 0) break;
      }
    for (int i = middle; i < last; ++i)
      if (comp(i, first)) {  // __pop_heap(first, middle, i)
        const float val = v[i];
        const int vix = ix[i];
        v[i] = v[first];
        ix[i] = ix[first];
        adjust_heap(first, 0, len, val, vix);
      }
  }
  __device__ void insertion_sort(int first, int last) {
    if (first == last) return;
    for (int i = first + 1; i < last; ++i) {
      const float val = v[i];
      const int vix = ix[i];
      if (comp(i, first)) {
        for (int j = i; j > first; --j) {
          v[j] = v[j - 1];
          ix[j] = ix[j - 1];
        }
        v[first] = val;
        ix[first] = vix;
      } else {
        int l = i, nx = i - 1;
        while (comp_val2(val, nx)) {
          v[l] = v[nx];
          ix[l] = ix[nx];
          l = nx;
          --nx;
        }
        v[l] = val;
        ix[l] = vix;
      }
    }
  }
  __device__ void nth_element(int nth, int n) {
    if (n == 0 || nth == n) return;
    int first = 0, last = n;
    int depth = 2 * (31 - __clz(n));  // std::__lg(n) * 2
    while (last - first > 3) {
      if (depth == 0) {
        heap_select(first, nth + 1, last);
        swap(first, nth);
        return;
      }
      --depth;
      const int mid = first + (last - first) / 2;
      move_median_to_first(first, first + 1, mid, last - 1);
      const int cut = unguarded_partition(first + 1, last, first);
      if (cut <= nth) first = cut;
      else last = cut;
    }
    insertion_sort(first, last);
  }
};

// One workgroup per image: softmax rows (thread per query), then lane 0 selects.
__global__ __launch_bounds__(256) void k_pp_topk(const float* __restrict__ cls, int Q, int C1, float* __restrict__ topv,
                                                 int* __restrict__ topi) {
  extern __shared__ char sm[];
  const int C = C1 - 1, n = Q * C, b = blockIdx.x;
  float* v = (float*)sm;
  int* ix = (int*)(sm + (size_t)n * 4);
  for (int q = threadIdx.x; q < Q; q += blockDim.x) {
    const float* row = cls + ((long long)b * Q + q) * C1;
    float m = row[0];
    for (int c = 1; c < C1; ++c) {
      const float x = row[c];
      m = (x != x || m != m) ? __int_as_float(0x7fc00000) : fmaxf(m, x);
    }
    float s = 0.f;
    for (int c = 0; c < C1; ++c) s += expf(row[c] - m);
    for (int c = 0; c < C; ++c) {
      v[q * C + c] = div_rn(expf(row[c] - m), s);
      ix[q * C + c] = q * C + c;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    Sel sel{v, ix};
    sel.nth_element(Q - 1, n);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < Q; j += blockDim.x) {
    topv[(long long)b * Q + j] = v[j];
    topi[(long long)b * Q + j] = ix[j];
  }
}

// Bilinear source index / weights (ATen compute_source_index_and_lambda, align_corners=False):
// identity at equal sizes, else src = max(scale * (dst + 0.5) - 0.5, 0) with scale = in / out in
// float, i0 = min(floor(src), in - 1), i1 = i0 + (i0 < in - 1), l1 = clamp(src - i0, 0, 1),
// l0 = 1 - l1.  The interpolated value (x inner, y outer, no contraction) agrees with the CPU
// kernel to a few ulp and in sign (oracle/postprocess.py's fixture checks).
struct Lin {
  int i0, i1;
  float l0, l1;
};
__device__ __forceinline__ Lin lin_index(int dst, int in, int out) {
  Lin o;
  if (in == out) {
    o.i0 = o.i1 = dst;
    o.l0 = 1.f;
    o.l1 = 0.f;
    return o;
  }
  const float scale = (float)in / (float)out;
  float src = scale * ((float)dst + 0.5f) - 0.5f;
  src = src < 0.f ? 0.f : src;
  o.i0 = min((int)floorf(src), in - 1);
  o.i1 = o.i0 + (o.i0 < in - 1 ? 1 : 0);
  o.l1 = fminf(fmaxf(src - (float)o.i0, 0.f), 1.f);
  o.l0 = 1.f - o.l1;
  return o;
}

// One workgroup per (selected entry, image): the entry's 384x384 interpolated logits, the binary
// bitmap (one u64 per 64 consecutive pixels, by ballot) and the mask score, reduced in a fixed
// order (thread partials, then the 4 waves in order).
__global__ __launch_bounds__(256) void k_pp_masks(const float* __restrict__ masks, int Q, int C, int h, int w,
                                                  const float* __restrict__ topv, const int* __restrict__ topi,
                                                  unsigned long long* __restrict__ bits, float* __restrict__ pscore,
                                                  float* __restrict__ cnt_out) {
  __shared__ float red[2][4];
  const int j = blockIdx.x, b = blockIdx.y, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int q = topi[(long long)b * Q + j] / C;
  const float* m = masks + ((long long)b * Q + q) * h * w;
  unsigned long long* bm = bits + ((long long)b * Q + j) * PP_WORDS;
  float s = 0.f, c = 0.f;
  for (int p = threadIdx.x; p < PP_S * PP_S; p += 256) {
    const int oy = p / PP_S, ox = p - oy * PP_S;
    const Lin ly = lin_index(oy, h, PP_S), lx = lin_index(ox, w, PP_S);
    const float* r0 = m + (long long)ly.i0 * w;
    const float* r1 = m + (long long)ly.i1 * w;
    const float t0 = r0[lx.i0] * lx.l0 + r0[lx.i1] * lx.l1;
    const float t1 = r1[lx.i0] * lx.l0 + r1[lx.i1] * lx.l1;
    const float val = t0 * ly.l0 + t1 * ly.l1;
    const bool on = val > 0.f;
    if (on) {
      s += 1.f / (1.f + expf(-val));
      c += 1.f;
    }
    const unsigned long long bal = __ballot(on);
    if (lane == 0) bm[p >> 6] = bal;
  }
  s = wave_sum(s);
  c = wave_sum(c);
  if (lane == 0) {
    red[0][wv] = s;
    red[1][wv] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float ss = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    const float cc = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    pscore[(long long)b * Q + j] = topv[(long long)b * Q + j] * div_rn(ss, cc + 1e-6f);
    cnt_out[(long long)b * Q + j] = cc;
  }
}

// ATen's legacy 'nearest' source index: identity at equal sizes, dst >> 1 at twice the size,
// else min(int(floor(dst * (float)in / out)), in - 1).
__device__ __forceinline__ int nearest_index(int dst, int in, int out) {
  if (in == out) return dst;
  if (out == 2 * in) return dst >> 1;
  const float scale = (float)in / (float)out;
  const int s = (int)floorf((float)dst * scale);
  return s < in - 1 ? s : in - 1;
}

__device__ __forceinline__ bool bit_at(const unsigned long long* bm, int sy, int sx) {
  const int p = sy * PP_S + sx;
  return (bm[p >> 6] >> (p & 63)) & 1ull;
}

// keep[j] = the entry's mask, at the target size, is non-empty and its pred score >= threshold
__global__ __launch_bounds__(256) void k_pp_keep(const unsigned long long* __restrict__ bits, const float* __restrict__ pscore,
                                                 int Q, int b, int Ht, int Wt, double threshold, int* __restrict__ keep) {
  __shared__ int any_s;
  const int j = blockIdx.x;
  if (threadIdx.x == 0) any_s = 0;
  __syncthreads();
  const unsigned long long* bm = bits + ((long long)b * Q + j) * PP_WORDS;
  int any = 0;
  for (long long p = threadIdx.x; p < (long long)Ht * Wt && !any; p += 256) {
    const int ty = (int)(p / Wt), tx = (int)(p - (long long)ty * Wt);
    any = bit_at(bm, nearest_index(ty, PP_S, Ht), nearest_index(tx, PP_S, Wt));
  }
  if (any) any_s = 1;
  __syncthreads();
  // the reference compares the float32 score as a Python float (double) with the threshold
  if (threadIdx.x == 0) keep[(long long)b * Q + j] = any_s && (double)pscore[(long long)b * Q + j] >= threshold;
}

// segment ids (kept entries numbered in top-k order, -1 otherwise), then the map: each target
// pixel takes the id of the last kept entry whose resized mask covers it, -1 if none.
__global__ __launch_bounds__(256) void k_pp_paint(const unsigned long long* __restrict__ bits, const int* __restrict__ keep,
                                                  int Q, int b, int Ht, int Wt, int* __restrict__ seg_id,
                                                  float* __restrict__ seg) {
  extern __shared__ int ids[];  // [Q]
  if (threadIdx.x == 0) {
    int nid = 0;
    for (int j = 0; j < Q; ++j) ids[j] = keep[(long long)b * Q + j] ? nid++ : -1;
  }
  __syncthreads();
  if (blockIdx.x == 0)
    for (int j = threadIdx.x; j < Q; j += 256) seg_id[(long long)b * Q + j] = ids[j];
  const long long np = (long long)Ht * Wt;
  for (long long p = blockIdx.x * 256ll + threadIdx.x; p < np; p += 256ll * gridDim.x) {
    const int ty = (int)(p / Wt), tx = (int)(p - (long long)ty * Wt);
    const int sy = nearest_index(ty, PP_S, Ht), sx = nearest_index(tx, PP_S, Wt);
    float out = -1.f;
    for (int j = Q - 1; j >= 0; --j)
      if (ids[j] >= 0 && bit_at(bits + ((long long)b * Q + j) * PP_WORDS, sy, sx)) {
        out = (float)ids[j];
        break;
      }
    seg[p] = out;
  }
}

// return_binary_maps: the kept entries' resized masks stacked in segment-id order (the
// reference's torch.stack(instance_maps), float 0/1 at the target size); grid (pixel blocks, Q)
__global__ __launch_bounds__(256) void k_pp_binary(const unsigned long long* __restrict__ bits,
                                                   const int* __restrict__ seg_id, int Q, int b, int Ht, int Wt,
                                                   float* __restrict__ out) {
  const int j = blockIdx.y;
  const int id = seg_id[(long long)b * Q + j];
  if (id < 0) return;  // block-uniform
  const unsigned long long* bm = bits + ((long long)b * Q + j) * PP_WORDS;
  const long long np = (long long)Ht * Wt;
  float* o = out + (long long)id * np;
  for (long long p = blockIdx.x * 256ll + threadIdx.x; p < np; p += 256ll * gridDim.x) {
    const int ty = (int)(p / Wt), tx = (int)(p - (long long)ty * Wt);
    o[p] = bit_at(bm, nearest_index(ty, PP_S, Ht), nearest_index(tx, PP_S, Wt)) ? 1.f : 0.f;
  }
}

struct PPWs {
  size_t topv, bits, keep, cnt, total;
};
PPWs pp_ws(int B, int Q) {
  PPWs o;
  size_t off = 0;
  o.topv = off;
  off += align256((size_t)B * Q * 4);
  o.keep = off;
  off += align256((size_t)B * Q * 4);
  o.cnt = off;
  off += align256((size_t)B * Q * 4);
  o.bits = off;
  off += align256((size_t)B * Q * PP_WORDS * 8);
  o.total = off;
  return o;
}

}  // namespace

extern "C" {

size_t rgbd_pp_instance_workspace_size(int B, int Q) { return B > 0 && Q > 0 ? pp_ws(B, Q).total : 256; }

int rgbd_pp_instance(const float* class_logits, const float* mask_logits, int B, int Q, int C1, int h, int w,
                     const int* target_h_host, const int* target_w_host, double threshold, float* const* seg_host,
                     int* topk_idx, float* pred_scores, int* seg_id, void* ws, void* stream) {
  RGBD_REQUIRE(class_logits && mask_logits && target_h_host && target_w_host && seg_host && topk_idx && pred_scores &&
                   seg_id && ws,
               RGBD_E_ARG);
  RGBD_REQUIRE(B > 0 && Q > 0 && C1 >= 2 && h > 0 && w > 0, RGBD_E_ARG);
  const size_t lds = (size_t)Q * (C1 - 1) * 8;
  RGBD_REQUIRE(lds <= 163840, RGBD_E_SHAPE);  // the top-k runs over LDS
  for (int b = 0; b < B; ++b) RGBD_REQUIRE(seg_host[b] && target_h_host[b] > 0 && target_w_host[b] > 0, RGBD_E_ARG);
  hipStream_t s = (hipStream_t)stream;
  const PPWs L = pp_ws(B, Q);
  char* base = (char*)ws;
  float* topv = (float*)(base + L.topv);
  int* keep = (int*)(base + L.keep);
  float* cnt = (float*)(base + L.cnt);
  unsigned long long* bits = (unsigned long long*)(base + L.bits);
  static const hipError_t attr = hipFuncSetAttribute((const void*)k_pp_topk,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  if (attr != hipSuccess) return (int)attr;
  k_pp_topk<<<B, 256, lds, s>>>(class_logits, Q, C1, topv, topk_idx);
  k_pp_masks<<<dim3(Q, B), 256, 0, s>>>(mask_logits, Q, C1 - 1, h, w, topv, topk_idx, bits, pred_scores, cnt);
  for (int b = 0; b < B; ++b) {
    const int Ht = target_h_host[b], Wt = target_w_host[b];
    k_pp_keep<<<Q, 256, 0, s>>>(bits, pred_scores, Q, b, Ht, Wt, threshold, keep);
    const int grid = (int)std::min<long long>(std::max<long long>(1, ((long long)Ht * Wt + 255) / 256), 1024);
    k_pp_paint<<<grid, 256, (size_t)Q * 4, s>>>(bits, keep, Q, b, Ht, Wt, seg_id, seg_host[b]);
  }
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

int rgbd_pp_binary_maps(const void* ws, int B, int Q, int b, int Ht, int Wt, const int* seg_id, float* out,
                        void* stream) {
  RGBD_REQUIRE(ws && seg_id && out && B > 0 && Q > 0 && b >= 0 && b < B && Ht > 0 && Wt > 0, RGBD_E_ARG);
  const PPWs L = pp_ws(B, Q);
  const unsigned long long* bits = (const unsigned long long*)((const char*)ws + L.bits);
  const int gx = (int)std::min<long long>(std::max<long long>(1, ((long long)Ht * Wt + 255) / 256), 256);
  k_pp_binary<<<dim3(gx, Q), 256, 0, (hipStream_t)stream>>>(bits, seg_id, Q, b, Ht, Wt, out);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

}  // extern "C"
