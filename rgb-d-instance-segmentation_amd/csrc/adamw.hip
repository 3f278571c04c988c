// The AdamW step of the training loop (the HF Trainer's AdamW, lr 1e-5 constant: finetuning.py:98
// with config.json:12-13), for a list of fp32 parameters with fp32 gradients and moments,
// in one launch: per element the update torch.optim.AdamW (fused) applies —
//   p -= (lr * wd) * p
//   m  = b1 * m + (1 - b1) * g,   v = b2 * v + (1 - b2) * g * g
//   p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// with the step count t read from device memory (a captured graph replays it; the caller adds 1
// before the launch).  HBM-bound: 16 bytes read and 12 written per element (p, g, m, v; p, m, v).
// A workgroup takes 4096 elements of one tensor (16-byte accesses when the tensor allows them);
// the tensor table travels as a kernel argument, so the launch holds no host-side state.
// rgbd_adamw_multi_shadow also writes each updated parameter's bfloat16 copy (round to nearest
// even, the bits torch's .to(bfloat16) gives) into a caller buffer: the bf16 operand the next
// forward's GEMMs read (dense.cast_weight), without a separate cast launch per weight.
#include "common.hpp"

#include <math.h>

namespace rgbd {
namespace {

constexpr int AW_MAXT = 48;         // tensors per launch (kernel argument table)
constexpr int AW_CHUNK = 4096;      // elements per workgroup
struct AwTable {
  float* p[AW_MAXT];
  const float* g[AW_MAXT];
  float* m[AW_MAXT];
  float* v[AW_MAXT];
  bf16_t* s[AW_MAXT];  // bfloat16 shadow of p (nullptr: none)
  long long n[AW_MAXT];
  int block0[AW_MAXT + 1];  // first workgroup of each tensor
  int nt;
};

struct AwHyper {
  float b1, b2, omb1, omb2;  // beta and 1 - beta (formed in double: 1 - 0.999f is 1.3e-5 off 0.001)
  float lrwd, eps;           // lr * weight_decay
  double b1d, b2d, lr;       // bias corrections in double, per workgroup
};

__device__ __forceinline__ void aw_elem(float& p, float g, float& m, float& v, const AwHyper& h, float step_size,
                                        float bc2_sqrt) {
  p = p - h.lrwd * p;
  m = h.b1 * m + h.omb1 * g;
  v = h.b2 * v + h.omb2 * g * g;
  const float denom = sqrtf(v) / bc2_sqrt + h.eps;
  p = p - step_size * m / denom;
}

__global__ __launch_bounds__(256) void k_adamw_multi(const AwTable T, const float* __restrict__ step,
                                                     const AwHyper h) {
  int t = 0;
  for (int i = 1; i < T.nt; ++i)
    if ((int)blockIdx.x >= T.block0[i]) t = i;
  // the bias corrections in double once per workgroup (one lane; double pow is hundreds of
  // instructions), broadcast through LDS
  __shared__ float s_corr[2];
  if (threadIdx.x == 0) {
    const double st = *step;
    const double bc1 = 1.0 - pow(h.b1d, st), bc2 = 1.0 - pow(h.b2d, st);
    s_corr[0] = (float)(h.lr / bc1);
    s_corr[1] = (float)sqrt(bc2);
  }
  __syncthreads();
  const float step_size = s_corr[0], bc2_sqrt = s_corr[1];
  const long long n = T.n[t];
  const long long e0 = (long long)(blockIdx.x - T.block0[t]) * AW_CHUNK;
  float* __restrict__ P = T.p[t];
  const float* __restrict__ G = T.g[t];
  float* __restrict__ M = T.m[t];
  float* __restrict__ V = T.v[t];
  bf16_t* __restrict__ S = T.s[t];
  const bool vec = ((((uintptr_t)P) | ((uintptr_t)G) | ((uintptr_t)M) | ((uintptr_t)V)) & 15) == 0 &&
                   (((uintptr_t)S) & 7) == 0;
  if (vec && e0 + AW_CHUNK <= n) {
#pragma unroll
    for (int k = 0; k < AW_CHUNK / 1024; ++k) {
      const long long e = e0 + 4ll * (threadIdx.x + 256 * k);
      float4 p = *reinterpret_cast<const float4*>(P + e), g = *reinterpret_cast<const float4*>(G + e);
      float4 m = *reinterpret_cast<const float4*>(M + e), v = *reinterpret_cast<const float4*>(V + e);
      aw_elem(p.x, g.x, m.x, v.x, h, step_size, bc2_sqrt);
      aw_elem(p.y, g.y, m.y, v.y, h, step_size, bc2_sqrt);
      aw_elem(p.z, g.z, m.z, v.z, h, step_size, bc2_sqrt);
      aw_elem(p.w, g.w, m.w, v.w, h, step_size, bc2_sqrt);
      *reinterpret_cast<float4*>(P + e) = p;
      *reinterpret_cast<float4*>(M + e) = m;
      *reinterpret_cast<float4*>(V + e) = v;
      if (S) *reinterpret_cast<uint2*>(S + e) = make_uint2(pack_bf16x2(p.x, p.y), pack_bf16x2(p.z, p.w));
    }
    return;
  }
  for (long long e = e0 + threadIdx.x; e < e0 + AW_CHUNK && e < n; e += 256) {
    float p = P[e], m = M[e], v = V[e];
    aw_elem(p, G[e], m, v, h, step_size, bc2_sqrt);
    P[e] = p;
    M[e] = m;
    V[e] = v;
    if (S) S[e] = f32_to_bf16(p);
  }
}

}  // namespace
}  // namespace rgbd

using namespace rgbd;

static int adamw_launch(int n, float* const* params, const float* const* grads, float* const* exp_avg,
                        float* const* exp_avg_sq, void* const* shadows, const long long* numel, const float* step,
                        double lr, double beta1, double beta2, double eps, double weight_decay, void* stream) {
  RGBD_REQUIRE(n >= 1 && n <= AW_MAXT && params && grads && exp_avg && exp_avg_sq && numel && step, RGBD_E_ARG);
  AwTable T;
  long long blocks = 0;
  for (int i = 0; i < n; ++i) {
    RGBD_REQUIRE(numel[i] >= 0, RGBD_E_ARG);
    RGBD_REQUIRE(numel[i] == 0 || (params[i] && grads[i] && exp_avg[i] && exp_avg_sq[i]), RGBD_E_ARG);
    T.p[i] = params[i];
    T.g[i] = grads[i];
    T.m[i] = exp_avg[i];
    T.v[i] = exp_avg_sq[i];
    T.s[i] = shadows ? (bf16_t*)shadows[i] : nullptr;
    T.n[i] = numel[i];
    T.block0[i] = (int)blocks;
    blocks += (numel[i] + AW_CHUNK - 1) / AW_CHUNK;
  }
  RGBD_REQUIRE(blocks < (1ll << 31), RGBD_E_SHAPE);
  T.block0[n] = (int)blocks;
  T.nt = n;
  if (blocks == 0) return RGBD_OK;
  AwHyper h;
  h.b1 = (float)beta1;
  h.b2 = (float)beta2;
  h.omb1 = (float)(1.0 - beta1);
  h.omb2 = (float)(1.0 - beta2);
  h.lrwd = (float)lr * (float)weight_decay;
  h.eps = (float)eps;
  h.b1d = beta1;
  h.b2d = beta2;
  h.lr = lr;
  k_adamw_multi<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(T, step, h);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}

extern "C" {

int rgbd_adamw_multi(int n, float* const* params, const float* const* grads, float* const* exp_avg,
                     float* const* exp_avg_sq, const long long* numel, const float* step, double lr, double beta1,
                     double beta2, double eps, double weight_decay, void* stream) {
  return adamw_launch(n, params, grads, exp_avg, exp_avg_sq, nullptr, numel, step, lr, beta1, beta2, eps,
                      weight_decay, stream);
}

int rgbd_adamw_multi_shadow(int n, float* const* params, const float* const* grads, float* const* exp_avg,
                            float* const* exp_avg_sq, void* const* shadows, const long long* numel, const float* step,
                            double lr, double beta1, double beta2, double eps, double weight_decay, void* stream) {
  RGBD_REQUIRE(shadows, RGBD_E_ARG);
  return adamw_launch(n, params, grads, exp_avg, exp_avg_sq, shadows, numel, step, lr, beta1, beta2, eps,
                      weight_decay, stream);
}

}  // extern "C"
