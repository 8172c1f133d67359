// Live per-kernel-class timing with HIP events (bench.py's roofline figure).
// One class is enabled at a time; every launch of that class records an event pair on
// the stream it runs on, plus its algorithmic bytes and flops.
#pragma once
#include "common.h"

#include <vector>

namespace wdr {

enum ProfClass : int { PROF_NONE = 0, PROF_GEMM = 1, PROF_GEMV = 2, PROF_FLASH = 3, PROF_XATTN = 4, PROF_MEL = 5,
                       PROF_DTW = 6, PROF_LOGITS = 7 };

bool prof_on(int cls);
int prof_class();
void prof_begin(hipStream_t s, hipEvent_t* e0);
void prof_end(hipStream_t s, hipEvent_t e0, double bytes, double flops);

// Graph support: while a stream capture is open, prof_end() appends the event pair to the
// capture list instead of the pending list; each replay of the graph re-records the same
// events, and prof_replayed() (after the replay completed) accumulates their elapsed times.
struct ProfPair {
  hipEvent_t a, b;
  double bytes, flops;
};
void prof_capture_begin(std::vector<ProfPair>* into);
void prof_capture_end();
void prof_replayed(const std::vector<ProfPair>& pairs);

}  // namespace wdr
