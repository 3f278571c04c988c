// f3: the Hungarian matcher's linear sum assignment on the GPU.
//
// Reference call: Mask2FormerHungarianMatcher.forward (transformers 5.15 modeling_mask2former.py:474)
// runs scipy.optimize.linear_sum_assignment(cost_matrix.cpu()) per image and per decoder output —
// a device->host sync and a CPU solve, ten times per image per training step.  This kernel solves
// a batch of cost matrices in one launch, one wavefront per matrix, with scipy 1.15's algorithm
// (rectangular_lsap.cpp, Crouse's shortest augmenting path; restated in oracle/lsap.py and pinned
// against scipy) step for step in float64, so it returns the same optimum scipy returns, ties
// included:
//   * tall matrices are solved transposed (rows = the shorter side);
//   * per augmenting path, `remaining` starts in reverse column order and a removed column is
//     replaced by the last one (swap-with-last), and the column picked among equal shortest-path
//     costs is the last free one in `remaining` order, else the first one;
//   * duals and path costs use the same float64 expressions, no FMA contraction.
// The scan over the remaining columns (the O(C) part of every Dijkstra step) is spread over the
// 64 lanes, the argmin is a wave reduction under the tie rule above (a total order, so the
// reduction equals scipy's sequential scan), the bookkeeping steps run in lane 0 with the state in
// LDS.  Bound: latency (a few microseconds per augmenting step); the point is removing the host
// round trip, not FLOPs.
#include "common.hpp"

#include <algorithm>

namespace rgbd {
namespace {

constexpr int LSA_MAX_C = 2048;

struct Cand {
  double val;
  int free_;  // 1 when the column has no row yet
  int pos;    // position in `remaining`
};

// scipy's sequential scan keeps the first position reaching the minimum, then moves to any later
// equal-cost position whose column is free: result = the last free position among the minima,
// else the first minimum.
__device__ __forceinline__ bool cand_better(const Cand& a, const Cand& b) {
  if (a.val != b.val) return a.val < b.val;
  if (a.free_ != b.free_) return a.free_ > b.free_;
  if (a.free_) return a.pos > b.pos;
  return a.pos < b.pos;
}

__global__ __launch_bounds__(64) void k_lsa(const float* __restrict__ cost, const long long* __restrict__ meta,
                                            int64_t* __restrict__ rows_out, int64_t* __restrict__ cols_out,
                                            int* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x;
  const long long* m = meta + 4ll * blockIdx.x;
  const long long coff = m[0], ooff = m[3];
  const int nr0 = (int)m[1], nc0 = (int)m[2];
  if (nr0 == 0 || nc0 == 0) {
    if (lane == 0) status[blockIdx.x] = 0;
    return;
  }
  const bool tr = nc0 < nr0;
  const int R = tr ? nc0 : nr0, C = tr ? nr0 : nc0;
  const float* cb = cost + coff;
  auto cost_at = [&](int i, int j) -> double {
    return (double)(tr ? cb[(long long)j * nc0 + i] : cb[(long long)i * nc0 + j]);
  };
  // LDS state
  double* u = (double*)smem;
  double* v = u + R;
  double* spc = v + C;
  int* path = (int*)(spc + C);
  int* col4row = path + C;
  int* row4col = col4row + R;
  int* remaining = row4col + C;
  uint8_t* SR = (uint8_t*)(remaining + C);
  uint8_t* SC = SR + R;
  __shared__ int sh_i, sh_sink, sh_num;
  __shared__ double sh_min;

  // invalid entries (NaN, -inf) -> scipy raises ValueError
  int bad = 0;
  for (long long e = lane; e < (long long)R * C; e += 64) {
    const float x = cb[e];
    bad |= (x != x) || (x == -INFINITY);
  }
  bad = __any(bad);
  if (bad) {
    if (lane == 0) status[blockIdx.x] = 2;
    return;
  }
  for (int i = lane; i < R; i += 64) {
    u[i] = 0.0;
    col4row[i] = -1;
  }
  for (int j = lane; j < C; j += 64) {
    v[j] = 0.0;
    row4col[j] = -1;
    path[j] = -1;
  }
  __syncthreads();

  for (int cur = 0; cur < R; ++cur) {
    // ---- shortest augmenting path from row cur
    for (int it = lane; it < C; it += 64) {
      remaining[it] = C - it - 1;
      spc[it] = INFINITY;
      SC[it] = 0;
    }
    for (int i = lane; i < R; i += 64) SR[i] = 0;
    if (lane == 0) {
      sh_i = cur;
      sh_sink = -1;
      sh_num = C;
      sh_min = 0.0;
    }
    __syncthreads();
    while (true) {
      const int i = sh_i, num = sh_num;
      const double minVal = sh_min;
      if (lane == 0) SR[i] = 1;
      const double ui = u[i];
      Cand best{INFINITY, 0, -1};
      for (int it = lane; it < num; it += 64) {
        const int j = remaining[it];
        const double r = minVal + cost_at(i, j) - ui - v[j];
        double s = spc[j];
        if (r < s) {
          path[j] = i;
          spc[j] = r;
          s = r;
        }
        const Cand c{s, row4col[j] == -1 ? 1 : 0, it};
        if (best.pos < 0 || cand_better(c, best)) best = c;
      }
      for (int o = 32; o > 0; o >>= 1) {
        Cand other;
        other.val = __shfl_xor(best.val, o);
        other.free_ = __shfl_xor(best.free_, o);
        other.pos = __shfl_xor(best.pos, o);
        if (other.pos >= 0 && (best.pos < 0 || cand_better(other, best))) best = other;
      }
      __syncthreads();  // every lane's spc / path writes and reads of this step are done
      if (best.val == INFINITY) {  // infeasible
        if (lane == 0) status[blockIdx.x] = 1;
        return;
      }
      if (lane == 0) {
        const int j = remaining[best.pos];
        sh_min = best.val;
        if (row4col[j] == -1)
          sh_sink = j;
        else
          sh_i = row4col[j];
        SC[j] = 1;
        sh_num = num - 1;
        remaining[best.pos] = remaining[num - 1];
      }
      __syncthreads();
      if (sh_sink != -1) break;
    }
    const double minVal = sh_min;
    // ---- dual update
    if (lane == 0) u[cur] += minVal;
    __syncthreads();
    for (int i = lane; i < R; i += 64)
      if (SR[i] && i != cur) u[i] += minVal - spc[col4row[i]];
    for (int j = lane; j < C; j += 64)
      if (SC[j]) v[j] -= minVal - spc[j];
    __syncthreads();
    // ---- augment along the path
    if (lane == 0) {
      int j = sh_sink;
      while (true) {
        const int i = path[j];
        row4col[j] = i;
        const int t = col4row[i];
        col4row[i] = j;
        j = t;
        if (i == cur) break;
      }
    }
    __syncthreads();
  }
  // ---- output in scipy's order
  int64_t* ro = rows_out + ooff;
  int64_t* co = cols_out + ooff;
  if (!tr) {
    for (int i = lane; i < R; i += 64) {
      ro[i] = i;
      co[i] = col4row[i];
    }
  } else {
    // argsort(col4row): original rows (the transposed columns) ascending, each with its column
    int base = 0;
    for (int j0 = 0; j0 < C; j0 += 64) {
      const int j = j0 + lane;
      const bool hit = j < C && row4col[j] != -1;
      const unsigned long long mask = __ballot(hit);
      const int k = base + __popcll(mask & ((1ull << lane) - 1ull));
      if (hit) {
        ro[k] = j;
        co[k] = row4col[j];
      }
      base += __popcll(mask);
    }
  }
  if (lane == 0) status[blockIdx.x] = 0;
}

}  // namespace
}  // namespace rgbd

using namespace rgbd;

extern "C" size_t rgbd_lsa_lds_bytes(int max_rows, int max_cols) {
  // R <= C after the transpose; arrays: u[R], col4row[R], SR[R]; v, spc, path, row4col, remaining, SC [C]
  const size_t R = (size_t)std::min(max_rows, max_cols), C = (size_t)std::max(max_rows, max_cols);
  return 8 * R + 8 * C + 8 * C + 4 * C + 4 * R + 4 * C + 4 * C + R + C + 16;
}

extern "C" int rgbd_lsa_batch(int n, const float* cost, const long long* meta, int max_rows, int max_cols,
                              int64_t* rows_out, int64_t* cols_out, int* status, void* stream) {
  RGBD_REQUIRE(n >= 0 && max_rows >= 0 && max_cols >= 0, RGBD_E_ARG);
  if (n == 0) return RGBD_OK;
  RGBD_REQUIRE(cost && meta && rows_out && cols_out && status, RGBD_E_ARG);
  RGBD_REQUIRE(std::max(max_rows, max_cols) <= LSA_MAX_C, RGBD_E_SHAPE);
  const size_t lds = rgbd_lsa_lds_bytes(max_rows, max_cols);
  if (lds > 65536) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_lsa, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  k_lsa<<<n, 64, lds, (hipStream_t)stream>>>(cost, meta, rows_out, cols_out, status);
  RGBD_CHECK_LAUNCH();
  return RGBD_OK;
}
