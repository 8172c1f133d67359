// Live per-kernel-class timing for bench.py's roofline figures.  Any set of classes can be
// enabled at once (each accumulates separately); 1 in 64 launches of that class is issued with hipExtLaunchKernelGGL start/stop events
// (timestamps of the dispatch itself, the same interval rocprofv3 reports), together with the
// launch's algorithmic bytes and flops.  Graph replay is bypassed while a class is enabled.
#pragma once
#include <hip/hip_ext.h>

#include <mutex>
#include <vector>

#include "common.h"

namespace wdr {

enum ProfClass : int { PROF_NONE = 0, PROF_GEMM = 1, PROF_GEMV = 2, PROF_FLASH = 3, PROF_XATTN = 4, PROF_SKINNY = 5 };

bool prof_on(int cls);
int prof_class();
// decode steps and full encode batches replay hipGraphs; while a class is enabled, 1 in
// kStepEvery steps (prof_step) or 1 in kEncEvery encode batches (prof_enc_batch) runs its kernels
// eagerly instead (events recorded inside a graph cannot be read on this ROCm), and those launches
// are sampled at the rate that makes every launch's probability 1 / (kEvery * kStepEvery).  Only
// work that would otherwise replay a graph draws: work that always runs eagerly (mixed batches,
// partial encode batches) is sampled at the base rate, or it would be over-represented.
// prof_capture(true) around a stream capture keeps event launches out of the graph.
bool prof_step();
bool prof_enc_batch();
void prof_capture(bool on);
// WDR_STREAM_LOG=1: every libwdr stream creation noted on stderr (with AMD_LOG_LEVEL=3 the
// runtime's hardware-queue choice is printed just before it; tools/queue_log.py pairs them)
void stream_note(const char* what, hipStream_t s);
void prof_in_step(bool on);    // around the eager launches of a step prof_step() picked
void prof_in_enc(bool on);     // around the eager launches of a batch prof_enc_batch() picked
hipEvent_t prof_event();
// frees the kernel-clock ring and the pooled events (wdr_shutdown)
void prof_shutdown();
// WDR_LAUNCH_LOCK=1: kernel launches and graph replays from all host threads go through one
// process-wide mutex (profiling runs: rocprofv3's kernel-trace interception of a launch faults
// inside the tool when several threads launch at once -- tools/prof_crash_ab.sh)
std::mutex* launch_lock();

void prof_push(int cls, hipEvent_t a, hipEvent_t b, unsigned long long* ts, double bytes, double flops);


// async copies / fills under WDR_LAUNCH_LOCK too: HIP runs them as blit kernels, whose
// dispatches the profiler intercepts like any launch
inline hipError_t wdr_memcpy_async(void* dst, const void* src, size_t n, hipMemcpyKind kind, hipStream_t s) {
  std::mutex* mu = launch_lock();
  if (mu) mu->lock();
  const hipError_t e = hipMemcpyAsync(dst, src, n, kind, s);
  if (mu) mu->unlock();
  return e;
}
inline hipError_t wdr_memset_async(void* dst, int v, size_t n, hipStream_t s) {
  std::mutex* mu = launch_lock();
  if (mu) mu->lock();
  const hipError_t e = hipMemsetAsync(dst, v, n, s);
  if (mu) mu->unlock();
  return e;
}

// a plain kernel launch under WDR_LAUNCH_LOCK (every launch site of libwdr goes through it or
// wdr_launch, the graph replays through launch_lock() too)
#define WDR_KLAUNCH(...)                                    \
  do {                                                      \
    std::mutex* mu_ = ::wdr::launch_lock();                 \
    if (mu_) mu_->lock();                                   \
    hipLaunchKernelGGL(__VA_ARGS__);                        \
    if (mu_) mu_->unlock();                                 \
  } while (0)

// a sampled launch carries HIP start/stop events and, for argument structs with a ProfClock
// slot (ProjArgs, FlashArgs, XAttnArgs: prof_attach), the kernel's own clock span
template <typename F, typename A0, typename... Args>
inline void wdr_launch(int cls, double bytes, double flops, F kernel, dim3 grid, dim3 block, uint32_t shmem,
                       hipStream_t s, A0 a0, Args... args) {
  std::mutex* mu = launch_lock();
  if (mu) mu->lock();
  if (prof_on(cls)) {
    hipEvent_t a = prof_event(), b = prof_event();
    unsigned long long* ts = prof_attach(a0);
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, a, b, 0, a0, args...);
    prof_push(cls, a, b, ts, bytes, flops);
  } else {
    hipLaunchKernelGGL(kernel, grid, block, shmem, s, a0, args...);
  }
  if (mu) mu->unlock();
}

}  // namespace wdr
