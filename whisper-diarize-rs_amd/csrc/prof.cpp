#include "prof.h"

#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "../../include/wdr.h"

namespace wdr {

namespace {
struct Rec {
  hipEvent_t a, b;
  int cls;
};
struct ClkRec {
  long long slot;   // kernel-clock slot in the ring
  int cls;
  double bytes, flops;
  double w;         // 1 / the launch's sampling probability
};
std::vector<ClkRec> g_clk_pending;
constexpr int kClasses = 8;
std::mutex g_mu;
std::atomic<int> g_mask{0};   // enabled classes, bit (1 << cls)
bool g_broken = false;
constexpr unsigned kEvery = 2;    // launches timed inside a sampled (eager) decode step
std::vector<Rec> g_pending;
std::vector<hipEvent_t> g_pool;
struct Acc {
  double ms = 0, bytes = 0, flops = 0;
  long long n = 0;
  // launches whose kernel clock span was read, each weighted by 1 / its sampling probability
  double clk_ms = 0, clk_bytes = 0, clk_flops = 0, clk_w = 0;
  long long clk_n = 0;
} g_acc[kClasses];

// kernel-clock ring: per slot PROF_CLK_LANES start words (init ~0) then PROF_CLK_LANES end words
// (init 0) -- workgroups stamp lane (block id % PROF_CLK_LANES), so the atomics of a
// many-workgroup launch spread over that many addresses instead of serialising on one (which
// inflated a 7680-workgroup launch by hundreds of us); slots are handed out in order and read
// back (with a device synchronisation) only at drain time
constexpr long long kSlotWords = 2 * PROF_CLK_LANES;
constexpr long long kRing = 1 << 16;
unsigned long long* g_ring = nullptr;
int g_ring_dev = -1;   // the device the ring (and the pooled events) live on
std::atomic<long long> g_next{0};
double g_tick_ms = 0.0;   // wall_clock64 period in ms

void ring_reset_locked() {
  if (!g_ring) {
    if (hipMalloc(&g_ring, (size_t)kRing * kSlotWords * 8) != hipSuccess) {
      (void)hipGetLastError();
      g_ring = nullptr;
      return;
    }
    int dev = 0, khz = 0;
    (void)hipGetDevice(&dev);
    g_ring_dev = dev;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
    g_tick_ms = 1.0 / (double)khz;
  }
  std::vector<unsigned long long> init((size_t)kRing * kSlotWords);
  for (long long i = 0; i < kRing; ++i)
    for (int j = 0; j < PROF_CLK_LANES; ++j) {
      init[i * kSlotWords + j] = ~0ull;
      init[i * kSlotWords + PROF_CLK_LANES + j] = 0ull;
    }
  if (hipMemcpy(g_ring, init.data(), init.size() * 8, hipMemcpyHostToDevice) != hipSuccess) (void)hipGetLastError();
  g_next = 0;
}

// the clock spans of recs (slots of `words`): earliest wave start -> latest wave end, weighted
void fold_clocks(const std::vector<ClkRec>& recs, const unsigned long long* words, size_t n_words) {
  for (const auto& r : recs) {
    if ((size_t)((r.slot + 1) * kSlotWords) > n_words) continue;
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int j = 0; j < PROF_CLK_LANES; ++j) {
      t0 = std::min(t0, words[r.slot * kSlotWords + j]);
      t1 = std::max(t1, words[r.slot * kSlotWords + PROF_CLK_LANES + j]);
    }
    if (t0 == ~0ull || t1 < t0) continue;
    Acc& A = g_acc[r.cls];
    A.clk_ms += r.w * (double)(t1 - t0) * g_tick_ms;
    A.clk_w += r.w;
    A.clk_n++;
    A.clk_bytes += r.w * r.bytes;
    A.clk_flops += r.w * r.flops;
  }
}

// events: waited for and folded in (batches during the run); kernel clocks (read_ring): read
// back once, after a device synchronisation, at read time
void drain_locked(bool read_ring = true) {
  for (auto& r : g_pending) {
    float ms = 0;
    if (hipEventSynchronize(r.b) != hipSuccess || hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) {
      (void)hipGetLastError();
      g_broken = true;
    }
    g_acc[r.cls].ms += ms;
    g_pool.push_back(r.a);
    g_pool.push_back(r.b);
  }
  g_pending.clear();
  if (!read_ring || g_clk_pending.empty() || !g_ring) return;
  std::vector<unsigned long long> ring((size_t)std::min<long long>(g_next.load(), kRing) * kSlotWords);
  int dev = 0;
  (void)hipGetDevice(&dev);
  const bool ok = hipSetDevice(g_ring_dev) == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
                  hipMemcpy(ring.data(), g_ring, ring.size() * 8, hipMemcpyDeviceToHost) == hipSuccess;
  (void)hipSetDevice(dev);
  if (!ok) {
    (void)hipGetLastError();
    g_broken = true;
    return;
  }
  fold_clocks(g_clk_pending, ring.data(), ring.size());
  g_clk_pending.clear();
}
}  // namespace

// the profiler samples the launches of ONE device (the current one when the mask was set): a
// multi-GPU context (gpu_device None) launches on peer devices too, whose kernels must not touch
// this device's ring and whose streams must not record this device's pooled events
static bool on_ring_device() {
  int dev = -1;
  return hipGetDevice(&dev) == hipSuccess && dev == g_ring_dev;
}

unsigned long long* prof_slot() {
  if (!g_ring || !on_ring_device()) return nullptr;
  const long long i = g_next++;
  return i < kRing ? g_ring + kSlotWords * i : nullptr;
}

// WDR_SEGV_TRACE=1: a fatal signal prints the faulting address, the thread and the native
// backtrace to stderr before the default action (root-causing faults under rocprofv3)
namespace {
void fatal_handler(int sig, siginfo_t* si, void*) {
  char buf[160];
  const int n = snprintf(buf, sizeof buf, "\n[wdr] fatal signal %d at address %p in thread %ld\n", sig,
                         si ? si->si_addr : nullptr, (long)syscall(SYS_gettid));
  if (n > 0) (void)!write(2, buf, (size_t)n);
  void* bt[64];
  const int k = backtrace(bt, 64);
  backtrace_symbols_fd(bt, k, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
struct FatalInit {
  FatalInit() {
    const char* e = getenv("WDR_SEGV_TRACE");
    if (!e || atoi(e) == 0) return;
    struct sigaction sa {};
    sa.sa_sigaction = fatal_handler;
    sa.sa_flags = SA_SIGINFO;
    sigaction(SIGSEGV, &sa, nullptr);
    sigaction(SIGBUS, &sa, nullptr);
    sigaction(SIGABRT, &sa, nullptr);
  }
} g_fatal_init;
}  // namespace


constexpr unsigned kStepEvery = 32;   // decode steps run eagerly for sampling: 1 in 32 (was 1 in
                                      // 8: the eager steps cost the 1-h bench ~2 %)
constexpr unsigned kEncEvery = 32;    // full encode batches run eagerly for sampling: 1 in 32 (1 in
                                      // 8 cost the profiled 1-h run 2-5 %: an eager batch holds its
                                      // chain's thread ~1 ms, fragmenting the batched steps --
                                      // profiles/r04/ab_prof_cost.txt)
// WDR_PROF_STEP_EVERY (A/B of the profiler's cost): decode steps run eagerly 1 in 16 / 32 / 64
// (default 64, every launch of such a step clocked: 1 in 32 with 1 in 2 clocked cost the profiled
// 1-h run ~3 % against ~1.6 %, profiles/r04/ab_prof_cost.txt), their launches clocked at the rate
// that keeps every launch's probability 1 / (kEvery * kStepEvery)
static unsigned step_every() {
  static const unsigned v = [] {
    const char* e = getenv("WDR_PROF_STEP_EVERY");
    const unsigned n = e ? (unsigned)atoi(e) : 64;
    return n == 16 || n == 32 ? n : 64;
  }();
  return v;
}
thread_local bool t_capture = false;
thread_local unsigned t_rate = 0;   // inside a sampled (eager) step / batch: its launches' rate

// every launch of the class is timed with probability 1 / (kEvery * kStepEvery): 1 in kEvery
// inside the sampled steps, 1 in kEvery * kStepEvery elsewhere (prefill, language detection),
// so the average is over a uniform sample of the class's launches.  The picks are pseudo-random
// (a per-thread xorshift), not every k-th launch: a fixed stride aliases with the fixed launch
// sequence of an encode batch (131 GEMM / flash launches) and sampled, round 4, the 1.26-TFLOP
// cross-K/V GEMM at another rate than the rest -- 16 % low on flops per launch vs the trace.
static bool pick(unsigned every) {
  thread_local uint64_t x = 0x9e3779b97f4a7c15ull ^ (uint64_t)(uintptr_t)&x;
  x ^= x << 13;
  x ^= x >> 7;
  x ^= x << 17;
  return (x >> 33) % every == 0;
}
bool prof_on(int cls) {
  if (!(g_mask.load(std::memory_order_relaxed) & (1 << cls)) || t_capture) return false;
  if (!on_ring_device()) return false;
  return pick(t_rate ? t_rate : kEvery * kStepEvery);
}
bool prof_step() {
  if (!g_mask.load(std::memory_order_relaxed)) return false;
  return pick(step_every());
}
bool prof_enc_batch() {
  if (!g_mask.load(std::memory_order_relaxed)) return false;
  return pick(kEncEvery);
}
void prof_capture(bool on) { t_capture = on; }
void prof_in_step(bool on) { t_rate = on ? kEvery * kStepEvery / step_every() : 0; }
void prof_in_enc(bool on) { t_rate = on ? kEvery * kStepEvery / kEncEvery : 0; }
int prof_class() { return g_mask.load(); }

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

void prof_shutdown() {
  std::lock_guard<std::mutex> l(g_mu);
  g_mask = 0;
  for (auto& r : g_pending) {
    (void)hipEventSynchronize(r.b);
    g_pool.push_back(r.a);
    g_pool.push_back(r.b);
  }
  g_pending.clear();
  g_clk_pending.clear();
  for (hipEvent_t e : g_pool) (void)hipEventDestroy(e);
  g_pool.clear();
  if (g_ring) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipSetDevice(g_ring_dev);
    (void)hipFree(g_ring);
    (void)hipSetDevice(dev);
    g_ring = nullptr;
  }
  (void)hipGetLastError();
}

void prof_push(int cls, hipEvent_t a, hipEvent_t b, unsigned long long* ts, double bytes, double flops) {
  std::lock_guard<std::mutex> l(g_mu);
  g_pending.push_back({a, b, cls});
  if (ts && g_ring)
    g_clk_pending.push_back({(long long)((ts - g_ring) / kSlotWords), cls, bytes, flops, (double)(kEvery * kStepEvery)});
  g_acc[cls].bytes += bytes;
  g_acc[cls].flops += flops;
  g_acc[cls].n++;
  if (g_pending.size() > 4096) drain_locked(false);
}

void stream_note(const char* what, hipStream_t s) {
  static const bool on = getenv("WDR_STREAM_LOG") && atoi(getenv("WDR_STREAM_LOG")) != 0;
  if (on) {
    fprintf(stderr, "[wdr-stream] %s %p\n", what, (void*)s);
    fflush(stderr);
  }
}

}  // namespace wdr

extern "C" {
int wdr_prof_set_mask(int32_t mask) {
  std::lock_guard<std::mutex> l(wdr::g_mu);
  wdr::drain_locked();
  wdr::g_mask = mask & ((1 << wdr::kClasses) - 2);
  wdr::g_clk_pending.clear();
  if (wdr::g_mask) wdr::ring_reset_locked();
  wdr::g_broken = false;
  for (auto& a : wdr::g_acc) a = wdr::Acc{};
  return 0;
}
int wdr_prof_set(int32_t cls) { return wdr_prof_set_mask(cls > 0 && cls < wdr::kClasses ? (1 << cls) : 0); }
int wdr_prof_read_class(int32_t cls, double* total_ms, int64_t* launches, double* algo_bytes, double* algo_flops) {
  std::lock_guard<std::mutex> l(wdr::g_mu);
  wdr::drain_locked();
  if (wdr::g_broken) return -2;
  if (cls <= 0 || cls >= wdr::kClasses) return -1;
  *total_ms = wdr::g_acc[cls].ms;
  *launches = wdr::g_acc[cls].n;
  *algo_bytes = wdr::g_acc[cls].bytes;
  *algo_flops = wdr::g_acc[cls].flops;
  return 0;
}
int wdr_prof_read_clock(int32_t cls, double* total_ms, int64_t* launches, double* algo_bytes, double* algo_flops) {
  std::lock_guard<std::mutex> l(wdr::g_mu);
  wdr::drain_locked();
  if (wdr::g_broken) return -2;
  if (cls <= 0 || cls >= wdr::kClasses) return -1;
  // weighted sums: total_ms / launches = the class's mean launch span, algo_bytes / launches its
  // mean bytes per launch (launches = the weight total, an estimate of the class's launch count)
  *total_ms = wdr::g_acc[cls].clk_ms;
  *launches = (int64_t)(wdr::g_acc[cls].clk_w + 0.5);
  *algo_bytes = wdr::g_acc[cls].clk_bytes;
  *algo_flops = wdr::g_acc[cls].clk_flops;
  return 0;
}
int wdr_prof_read(double* total_ms, int64_t* launches, double* algo_bytes, double* algo_flops) {
  // the sum over the enabled classes (one class: that class)
  double ms = 0, by = 0, fl = 0;
  int64_t n = 0;
  for (int c = 1; c < wdr::kClasses; ++c) {
    if (!(wdr::g_mask.load() & (1 << c))) continue;
    double a, b, d;
    int64_t k;
    if (wdr_prof_read_class(c, &a, &k, &b, &d) != 0) return -2;
    ms += a; n += k; by += b; fl += d;
  }
  *total_ms = ms;
  *launches = n;
  *algo_bytes = by;
  *algo_flops = fl;
  return 0;
}
}
