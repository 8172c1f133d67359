#include "prof.h"

#include <atomic>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "../../include/wdr.h"

namespace wdr {

namespace {
struct Rec {
  hipEvent_t a, b;
};
std::mutex g_mu;
int g_cls = PROF_NONE;
bool g_broken = false;
std::atomic<unsigned> g_tick{0};
constexpr unsigned kEvery = 8;
std::vector<Rec> g_pending;
std::vector<hipEvent_t> g_pool;
double g_ms = 0, g_bytes = 0, g_flops = 0;
long long g_n = 0;

void drain_locked() {
  for (auto& r : g_pending) {
    float ms = 0;
    if (hipEventSynchronize(r.b) != hipSuccess || hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) {
      (void)hipGetLastError();
      g_broken = true;
    }
    g_ms += ms;
    g_pool.push_back(r.a);
    g_pool.push_back(r.b);
  }
  g_pending.clear();
}
}  // namespace

std::atomic<unsigned> g_step{0}, g_tick_out{0};
constexpr unsigned kStepEvery = 8;
thread_local bool t_capture = false;
thread_local bool t_step = false;   // inside a sampled (eager) decode step

// every launch of the class is timed with probability 1 / (kEvery * kStepEvery): 1 in kEvery
// inside the sampled steps, 1 in kEvery * kStepEvery elsewhere (prefill, language detection),
// so the average is over a uniform sample of the class's launches
bool prof_on(int cls) {
  if (g_cls == PROF_NONE || g_cls != cls || t_capture) return false;
  if (t_step) return (g_tick++ % kEvery) == 0;
  return (g_tick_out++ % (kEvery * kStepEvery)) == 0;
}
bool prof_step() {
  if (g_cls == PROF_NONE) return false;
  return (g_step++ % kStepEvery) == 0;
}
void prof_capture(bool on) { t_capture = on; }
void prof_in_step(bool on) { t_step = on; }
int prof_class() { return g_cls; }

std::mutex* launch_lock() {
  static std::mutex mu;
  static const bool on = [] {
    const char* e = getenv("WDR_LAUNCH_LOCK");
    return e && atoi(e) != 0;
  }();
  return on ? &mu : nullptr;
}

hipEvent_t prof_event() {
  std::lock_guard<std::mutex> l(g_mu);
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  WDR_HIP(hipEventCreate(&e));
  return e;
}

void prof_push(hipEvent_t a, hipEvent_t b, double bytes, double flops) {
  std::lock_guard<std::mutex> l(g_mu);
  g_pending.push_back({a, b});
  g_bytes += bytes;
  g_flops += flops;
  g_n++;
  if (g_pending.size() > 4096) drain_locked();
}

}  // namespace wdr

extern "C" {
int wdr_prof_set(int32_t cls) {
  std::lock_guard<std::mutex> l(wdr::g_mu);
  wdr::drain_locked();
  wdr::g_cls = cls;
  wdr::g_broken = false;
  wdr::g_tick = 0;
  wdr::g_step = 0;
  wdr::g_tick_out = 0;
  wdr::g_ms = wdr::g_bytes = wdr::g_flops = 0;
  wdr::g_n = 0;
  return 0;
}
int wdr_prof_read(double* total_ms, int64_t* launches, double* algo_bytes, double* algo_flops) {
  std::lock_guard<std::mutex> l(wdr::g_mu);
  wdr::drain_locked();
  if (wdr::g_broken) return -2;
  *total_ms = wdr::g_ms;
  *launches = wdr::g_n;
  *algo_bytes = wdr::g_bytes;
  *algo_flops = wdr::g_flops;
  return 0;
}
}
