// Optional per-kernel timing with HIP events recorded on the launch stream (bench.py's
// roofline numbers).  Disabled by default: a TimerScope is then two branches and nothing
// else, so graph capture is unaffected.  Not thread-safe (one host thread drives a device).
#pragma once
#include <hip/hip_runtime.h>

namespace rgbd {
struct TimerScope {
  int slot = -1;
  hipStream_t stream;
  TimerScope(const char* name, hipStream_t s);
  ~TimerScope();
};
}  // namespace rgbd
