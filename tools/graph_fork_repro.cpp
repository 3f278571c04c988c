// Stand-alone HIP reproducer for the hipGraphLaunch host segfault of round 2:
// a captured step whose main stream forks to two side streams (or to one side stream twice from
// the same capture point) segfaulted in hipGraphLaunch at its first replay, once the process had
// captured, replayed and destroyed other graphs.  This program has no torch in it: if it crashes,
// the fault is in the HIP runtime's graph path; if it does not, it is in what torch adds around
// the capture (memory pool, event lifetime, record_stream).
//
// usage: graph_fork_repro <mode> <n_prior_graphs> <n_replays>
//   mode 0: one side stream, one fork per branch point (the structure the hot path keeps)
//   mode 1: two side streams forked from the same capture point
//   mode 2: the same side stream forked twice from the same capture point
//   mode 3: mode 1 with fresh events per fork/join destroyed right after use (torch's
//           Stream.wait_stream creates and drops an event per call)
// prints one line per stage; exit 0 = no fault.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(2);                                                                  \
    }                                                                                \
  } while (0)

__global__ void k_axpy(float* y, const float* x, float a, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = a * x[i] + y[i];
}

static void launch(hipStream_t s, float* y, const float* x, float a, int n) {
  hipLaunchKernelGGL(k_axpy, dim3((n + 255) / 256), dim3(256), 0, s, y, x, a, n);
  CK(hipGetLastError());
}

struct Fork {
  hipStream_t main;
  bool fresh;  // create + destroy an event per fork / join (torch's wait_stream)
  hipEvent_t ev_keep[8];
  int used = 0;
  hipEvent_t ev() {
    if (!fresh) return ev_keep[used++ % 8];
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
  }
  void done(hipEvent_t e) {
    if (fresh) CK(hipEventDestroy(e));
  }
  void fork(hipStream_t side) {  // side waits for main
    hipEvent_t e = ev();
    CK(hipEventRecord(e, main));
    CK(hipStreamWaitEvent(side, e, 0));
    done(e);
  }
  void join(hipStream_t side) {  // main waits for side
    hipEvent_t e = ev();
    CK(hipEventRecord(e, side));
    CK(hipStreamWaitEvent(main, e, 0));
    done(e);
  }
};

int main(int argc, char** argv) {
  const int mode = argc > 1 ? std::atoi(argv[1]) : 1;
  const int prior = argc > 2 ? std::atoi(argv[2]) : 20;
  const int replays = argc > 3 ? std::atoi(argv[3]) : 3;
  const int n = 1 << 20;
  float *x, *y0, *y1, *y2;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y0, n * 4));
  CK(hipMalloc(&y1, n * 4));
  CK(hipMalloc(&y2, n * 4));
  CK(hipMemset(x, 0, n * 4));
  hipStream_t cap, s1, s2;
  CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  Fork f{cap, mode == 3, {}};
  for (auto& e : f.ev_keep) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));

  // other graphs first: captured (some with a fork to s1), replayed, destroyed; plus allocator
  // churn between them
  for (int g = 0; g < prior; ++g) {
    hipGraph_t gr;
    hipGraphExec_t ex;
    CK(hipStreamBeginCapture(cap, hipStreamCaptureModeGlobal));
    launch(cap, y0, x, 1.f, n);
    if (g & 1) {
      f.fork(s1);
      launch(s1, y1, x, 1.f, n);
      f.join(s1);
    }
    launch(cap, y0, x, 2.f, n);
    CK(hipStreamEndCapture(cap, &gr));
    CK(hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0));
    for (int r = 0; r < 2; ++r) CK(hipGraphLaunch(ex, cap));
    CK(hipStreamSynchronize(cap));
    CK(hipGraphExecDestroy(ex));
    CK(hipGraphDestroy(gr));
    void* tmp;
    CK(hipMalloc(&tmp, (size_t)(g + 1) << 20));
    CK(hipFree(tmp));
  }
  std::printf("prior graphs: %d done\n", prior);

  // the step under test
  hipGraph_t gr;
  hipGraphExec_t ex;
  CK(hipStreamBeginCapture(cap, hipStreamCaptureModeGlobal));
  launch(cap, y0, x, 1.f, n);
  if (mode == 0) {
    f.fork(s1);
    launch(s1, y1, x, 1.f, n);
    launch(cap, y0, x, 1.f, n);
    f.join(s1);
  } else if (mode == 1 || mode == 3) {
    f.fork(s1);
    f.fork(s2);
    launch(s1, y1, x, 1.f, n);
    launch(s2, y2, x, 1.f, n);
    launch(cap, y0, x, 1.f, n);
    f.join(s1);
    launch(cap, y0, x, 1.f, n);
    f.join(s2);
  } else {
    f.fork(s1);
    launch(s1, y1, x, 1.f, n);
    f.fork(s1);
    launch(s1, y2, x, 1.f, n);
    launch(cap, y0, x, 1.f, n);
    f.join(s1);
  }
  launch(cap, y0, x, 3.f, n);
  CK(hipStreamEndCapture(cap, &gr));
  size_t nn = 0;
  CK(hipGraphGetNodes(gr, nullptr, &nn));
  CK(hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0));
  CK(hipGraphDebugDotPrint(gr, "gpurun_out/graph_fork_repro.dot", 0));
  std::printf("mode %d: captured %zu nodes, instantiated\n", mode, nn);
  std::fflush(stdout);
  for (int r = 0; r < replays; ++r) {
    CK(hipGraphLaunch(ex, cap));
    CK(hipStreamSynchronize(cap));
    std::printf("replay %d ok\n", r);
    std::fflush(stdout);
  }
  CK(hipGraphExecDestroy(ex));
  CK(hipGraphDestroy(gr));
  std::printf("mode %d: no fault\n", mode);
  return 0;
}
