#include "timing.hpp"

#include <string.h>

#include <string>
#include <vector>

#include "common.hpp"

namespace {
struct Entry {
  std::string name;
  std::vector<hipEvent_t> start, stop;
  int used = 0;
};
bool g_on = false;
std::vector<Entry> g_entries;

Entry& entry(const char* name) {
  for (auto& e : g_entries)
    if (e.name == name) return e;
  g_entries.push_back(Entry{});
  g_entries.back().name = name;
  return g_entries.back();
}
}  // namespace

namespace rgbd {
TimerScope::TimerScope(const char* name, hipStream_t s) : stream(s) {
  if (!g_on) return;
  Entry& e = entry(name);
  if (e.used == (int)e.start.size()) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
    e.start.push_back(a);
    e.stop.push_back(b);
  }
  slot = (int)(&e - g_entries.data()) * 1000000 + e.used;
  (void)hipEventRecord(e.start[e.used], s);
}
TimerScope::~TimerScope() {
  if (slot < 0) return;
  Entry& e = g_entries[slot / 1000000];
  (void)hipEventRecord(e.stop[slot % 1000000], stream);
  e.used++;
}
}  // namespace rgbd

extern "C" {
int rgbd_timing_enable(int on) {
  g_on = on != 0;
  for (auto& e : g_entries) e.used = 0;
  return RGBD_OK;
}

double rgbd_timing_read(const char* name, int* count) {
  double total = 0.0;
  int n = 0;
  for (auto& e : g_entries) {
    if (e.name != name) continue;
    for (int i = 0; i < e.used; ++i) {
      float ms = 0.f;
      if (hipEventSynchronize(e.stop[i]) == hipSuccess && hipEventElapsedTime(&ms, e.start[i], e.stop[i]) == hipSuccess) {
        total += ms;
        ++n;
      }
    }
    e.used = 0;
  }
  if (count) *count = n;
  return total;
}
}
