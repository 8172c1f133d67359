// Whisper context / state: weights in HBM, encoder + decoder forward, and the
// whisper_full_with_state decode loop as the reference drives it
// (src/transcribe.rs:20-87 params, :389 state.full).  Mirrors oracle/whisper_full.py.
#include "whisper.h"
#include "rows.h"
#include "ggml_file.h"
#include "prof.h"

#include <algorithm>
#include <functional>
#include <chrono>
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <map>
#include <random>
#include <exception>
#include <condition_variable>
#include <deque>
#include <set>
#include <pthread.h>
#include <thread>
#include <mutex>
#include <sstream>

namespace wdr {

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ------------------------------------------------------------------ hparams / presets
bool hparams_for(const std::string& name, HParams* hp) {
  HParams h;
  if (name == "base.en" || name == "base") {
    if (name == "base") h.n_vocab = 51865;
  } else if (name == "tiny.en" || name == "tiny") {
    h.n_audio_state = h.n_text_state = 384;
    h.n_audio_head = h.n_text_head = 6;
    h.n_audio_layer = h.n_text_layer = 4;
    if (name == "tiny") h.n_vocab = 51865;
  } else if (name == "small.en" || name == "small") {
    h.n_audio_state = h.n_text_state = 768;
    h.n_audio_head = h.n_text_head = 12;
    h.n_audio_layer = h.n_text_layer = 12;
    if (name == "small") h.n_vocab = 51865;
  } else if (name == "medium.en" || name == "medium") {
    h.n_audio_state = h.n_text_state = 1024;
    h.n_audio_head = h.n_text_head = 16;
    h.n_audio_layer = h.n_text_layer = 24;
    if (name == "medium") h.n_vocab = 51865;
  } else if (name == "large-v3" || name == "large-v3-turbo") {
    h.n_vocab = 51866;
    h.n_mels = 128;
    h.n_audio_state = h.n_text_state = 1280;
    h.n_audio_head = h.n_text_head = 20;
    h.n_audio_layer = 32;
    h.n_text_layer = name == "large-v3" ? 32 : 4;
  } else if (name == "tiny-test") {
    h.n_audio_state = h.n_text_state = 128;
    h.n_audio_head = h.n_text_head = 2;
    h.n_audio_layer = h.n_text_layer = 2;
  } else if (name == "tiny-test-ml") {
    h.n_vocab = 51866;
    h.n_mels = 128;
    h.n_audio_state = h.n_text_state = 128;
    h.n_audio_head = h.n_text_head = 2;
    h.n_audio_layer = h.n_text_layer = 2;
  } else {
    return false;
  }
  *hp = h;
  return true;
}

// whisper.cpp g_aheads_* presets (OpenAI _ALIGNMENT_HEADS); src/transcribe.rs:117-129 maps
// model names to presets and falls back to Small for unknown names.
std::vector<std::pair<int, int>> alignment_heads_for(const std::string& n) {
  static const std::map<std::string, std::vector<std::pair<int, int>>> tab = {
      {"tiny.en", {{1, 0}, {2, 0}, {2, 5}, {3, 0}, {3, 1}, {3, 2}, {3, 3}, {3, 4}}},
      {"tiny", {{2, 2}, {3, 0}, {3, 2}, {3, 3}, {3, 4}, {3, 5}}},
      {"base.en", {{3, 3}, {4, 7}, {5, 1}, {5, 5}, {5, 7}}},
      {"base", {{3, 1}, {4, 2}, {4, 3}, {4, 7}, {5, 1}, {5, 2}, {5, 4}, {5, 6}}},
      {"small.en", {{6, 6}, {7, 0}, {7, 3}, {7, 8}, {8, 2}, {8, 5}, {8, 7}, {9, 0}, {9, 4}, {9, 8},
                    {9, 10}, {10, 0}, {10, 1}, {10, 2}, {10, 3}, {10, 6}, {10, 11}, {11, 2}, {11, 4}}},
      {"small", {{5, 3}, {5, 9}, {8, 0}, {8, 4}, {8, 7}, {8, 8}, {9, 0}, {9, 7}, {9, 9}, {10, 5}}},
      {"medium.en", {{11, 4}, {14, 1}, {14, 12}, {14, 14}, {15, 4}, {16, 0}, {16, 4}, {16, 9}, {17, 12},
                     {17, 14}, {18, 7}, {18, 10}, {18, 15}, {20, 0}, {20, 3}, {20, 9}, {20, 14}, {21, 12}}},
      {"medium", {{13, 15}, {15, 4}, {15, 15}, {16, 1}, {20, 0}, {23, 4}}},
      {"large-v3", {{7, 0}, {10, 17}, {12, 18}, {13, 12}, {16, 1}, {17, 14}, {19, 11}, {21, 4}, {24, 1}, {25, 6}}},
      {"large-v3-turbo", {{2, 4}, {2, 11}, {3, 3}, {3, 6}, {3, 11}, {3, 14}}},
      {"tiny-test", {{1, 0}, {1, 1}}},
      {"tiny-test-ml", {{1, 0}, {1, 1}}},
  };
  auto it = tab.find(n);
  return it != tab.end() ? it->second : tab.at("small");
}

// ------------------------------------------------------------------ device memory
// Allocation / free and hipGraph capture are serialised by one process-wide mutex: several host
// threads capture graphs (step batchers, encode-ahead threads) while others run, and a
// synchronising call (hipFree, a legacy-stream memset, pinned host allocation) issued by one
// thread while another captures invalidates that capture on ROCm 7.2 ("operation would make the
// legacy stream depend on a capturing blocking stream"), whatever the capture mode.
std::recursive_mutex& hip_alloc_mutex() {
  static std::recursive_mutex mu;
  return mu;
}

// A stream on a hardware queue of its own.  HIP multiplexes the process's streams onto at most
// GPU_MAX_HW_QUEUES (4) hardware queues per priority level, in order: a kernel of the step batcher
// then waits behind whatever another stream sharing its queue has in front of it (an encoder GEMM
// launch, a barrier packet waiting on a slot event).  A stream created with a CU mask gets a
// dedicated queue; the mask here is every CU of the device.  kind: a WDR_<kind>_HWQ env knob
// (0 = the shared priority pool, A/B runs), default `def`.
// WDR_NO_GRAPH: eager decode steps and encode batches (no hipGraph replay); read once
static bool no_graph() {
  static const bool v = getenv("WDR_NO_GRAPH") != nullptr;
  return v;
}

// WDR_HOST_FENCE (default 1): a state's own (decode) stream does not carry barrier packets.  HIP
// maps the 40 states' highest-priority streams and the step batcher's onto GPU_MAX_HW_QUEUES
// shared hardware queues, and a queue runs its packets in order: a hipStreamWaitEvent on a state
// stream waiting for a low-priority DTW pass held back every batched step queued behind it on
// that queue (configs[2]'s VAD line: long segments, windows encoded on demand on the state
// stream after such a wait; profiles/r05/vad_line_queues.txt).  The chain's host thread waits
// for the event instead -- it synchronises on that stream right after anyway.
// A chain's wait for its encoded window: hipEventQuery every WDR_READY_POLL_US (default 50 us)
// with the thread asleep in between, instead of hipEventSynchronize, which spins.  At a run's
// start all 40 chains wait for their first encode batches together (0.1-0.6 s in); spinning, they
// spent the process's CPU quota (16 CPUs a 100-ms period on the box) in each of those periods and
// the kernel froze every thread of the process for the rest of it -- 5 throttled periods in a row
// (bench.py host_cpu.throttle_at_s).  0: hipEventSynchronize.
static void wait_event_polled(hipEvent_t ev) {
  static const int us = getenv("WDR_READY_POLL_US") ? atoi(getenv("WDR_READY_POLL_US")) : 50;
  if (us <= 0) {
    WDR_HIP(hipEventSynchronize(ev));
    return;
  }
  for (;;) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) WDR_HIP(q);
    std::this_thread::sleep_for(std::chrono::microseconds(us));
  }
}

static bool host_fence() {
  static const bool v = !(getenv("WDR_HOST_FENCE") && atoi(getenv("WDR_HOST_FENCE")) == 0);
  return v;
}

static void stream_fence(hipStream_t s, hipEvent_t ev, bool host) {
  if (host)
    WDR_HIP(hipEventSynchronize(ev));
  else
    WDR_HIP(hipStreamWaitEvent(s, ev, 0));
}

hipStream_t dedicated_stream(const char* knob, bool def, int prio) {
  const char* e = getenv(knob);
  const bool on = e ? atoi(e) != 0 : def;
  hipStream_t s = nullptr;
  if (!on) {
    WDR_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio));
    stream_note(knob, s);
    return s;
  }
  int dev = 0, ncu = 0;
  WDR_HIP(hipGetDevice(&dev));
  WDR_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  // knob = 2 (A/B, MI355X): only the CUs the encode-ahead pool leaves free (WDR_ENC_MASK under
  // WDR_ENC_MASK_PAT=1: 4 per XCD), so this stream's workgroups never wait behind encoder tiles
  const int n_res = getenv("WDR_ENC_MASK") ? atoi(getenv("WDR_ENC_MASK")) : 32;
  const bool reserved = atoi(e) == 2 && ncu == 256 && n_res > 0 && n_res <= 32 && n_res % 8 == 0;
  for (int c = 0; c < ncu; ++c) {
    const int x = c / 32, r = c % 32;   // the encoder pool's pattern-1 reservation
    const bool res = r % 8 == x && r / 8 < n_res / 8;
    if (!reserved || res) mask[c / 32] |= 1u << (c % 32);
  }
  WDR_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  stream_note(knob, s);
  return s;
}

// The encode-ahead streams of all states: WDR_ENC_POOL (default 2) CU-masked streams per device,
// a dedicated hardware queue each, shared round-robin by the states, which leave WDR_ENC_MASK
// (default 32) CUs -- 4 per XCD -- to the decode chain.  1-h bench, A/B on one box
// (profiles/r03/ab_enc_queues.txt): 608-619 xRT with one low-priority stream per state (24 streams
// on HIP's 4 shared low-priority queues) against 642-646 with 2 or 3 masked queues; 4 or 8
// masked queues 576, one 547 (the encoder starves), 24 (one per state) 398.  Both knobs -1: one
// low-priority stream per state.  Returns null then.
// A stream of a pool of `pool` CU-masked streams (dedicated hardware queues) per (tag, device),
// handed out round-robin, that leave n_res CUs free (WDR_ENC_MASK_PAT=1: spread over the 8 XCDs
// whether mask bit c is CU c % 32 of XCD c / 32 or CU c / 8 of XCD c % 8 -- bits 32x + 8j + x,
// j < n/8 -- since a decode launch's workgroups go round-robin over the XCDs, every XCD needs free
// CUs; 0: the top n bits).  pool <= 0: a stream of its own.
using StreamPools = std::map<std::pair<std::string, int>, std::pair<std::vector<hipStream_t>, int>>;
static std::mutex& stream_pools_mu() {
  static std::mutex mu;
  return mu;
}
static StreamPools& stream_pools() {
  static StreamPools* p = new StreamPools();   // outlives static destruction (exit hook)
  return *p;
}

void destroy_stream_pools() {
  std::lock_guard<std::mutex> g(stream_pools_mu());
  for (auto& kv : stream_pools()) {
    (void)hipSetDevice(kv.first.second);
    for (hipStream_t st : kv.second.first) {
      (void)hipStreamSynchronize(st);
      (void)hipStreamDestroy(st);
    }
  }
  stream_pools().clear();
  (void)hipGetLastError();
}

static hipStream_t masked_pool_stream(const char* tag, int n_res, int pool, bool* shared) {
  int dev = 0, ncu = 0;
  WDR_HIP(hipGetDevice(&dev));
  WDR_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  WDR_CHECK(n_res < ncu, "masked stream: must leave at least one CU");
  static const int pat = getenv("WDR_ENC_MASK_PAT") ? atoi(getenv("WDR_ENC_MASK_PAT")) : 1;
  auto make = [&] {
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    std::vector<char> res(ncu, 0);
    if (pat == 1 && ncu == 256) {
      WDR_CHECK(n_res % 8 == 0 && n_res <= 32, "WDR_ENC_MASK_PAT=1: 0, 8, 16, 24 or 32 CUs");
      for (int x = 0; x < 8; ++x)
        for (int j = 0; j < std::max(0, n_res) / 8; ++j) res[32 * x + 8 * j + x] = 1;
    } else {
      for (int c = ncu - std::max(0, n_res); c < ncu; ++c) res[c] = 1;
    }
    for (int c = 0; c < ncu; ++c)
      if (!res[c]) mask[c / 32] |= 1u << (c % 32);
    hipStream_t st = nullptr;
    WDR_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
    stream_note(tag, st);
    return st;
  };
  *shared = false;
  if (pool <= 0) return make();
  std::lock_guard<std::mutex> g(stream_pools_mu());
  auto& P = stream_pools()[{tag, dev}];
  if (P.first.empty())
    for (int i = 0; i < pool; ++i) P.first.push_back(make());
  *shared = true;
  return P.first[P.second++ % pool];
}

// The encode-ahead streams of all states: WDR_ENC_POOL (default 2) CU-masked streams per device,
// a dedicated hardware queue each, shared round-robin by the states, which leave WDR_ENC_MASK
// (default 32) CUs -- 4 per XCD -- to the decode chain.  1-h bench, A/B on one box
// (profiles/r03/ab_enc_queues.txt): 608-619 xRT with one low-priority stream per state (24 streams
// on HIP's 4 shared low-priority queues) against 642-646 with 2 or 3 masked queues; 4 or 8
// masked queues 576, one 547 (the encoder starves), 24 (one per state) 398.  Both knobs -1: one
// low-priority stream per state.  Returns null then.
static hipStream_t enc_masked_stream(bool* shared) {
  static const int n_res = getenv("WDR_ENC_MASK") ? atoi(getenv("WDR_ENC_MASK")) : 32;
  static const int pool = getenv("WDR_ENC_POOL") ? atoi(getenv("WDR_ENC_POOL")) : 2;
  *shared = false;
  if (n_res < 0 && pool < 0) return nullptr;
  int dev = 0, ncu = 0;
  WDR_HIP(hipGetDevice(&dev));
  WDR_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  if (ncu != 256 && !getenv("WDR_ENC_MASK") && !getenv("WDR_ENC_POOL")) return nullptr;   // tuned on MI355X
  return masked_pool_stream("enc", n_res, pool, shared);
}

// One mutex per pooled stream: a state's encode batch is issued onto a shared stream as one
// unit, so batches run one after another instead of interleaving kernel by kernel (at the start
// of a run every state issues its first batch at once: interleaved, all 12 batches of a stream
// finished together, ~0.6 s in; one after another, the first chains start decoding ~50 ms in).
static std::mutex& stream_issue_mutex(hipStream_t st) {
  static std::mutex mu;
  static std::map<hipStream_t, std::unique_ptr<std::mutex>> m;
  std::lock_guard<std::mutex> g(mu);
  auto& p = m[st];
  if (!p) p = std::make_unique<std::mutex>();
  return *p;
}

// WDR_OWN_POOL=P (A/B): the states' own streams from P masked streams (WDR_OWN_MASK CUs left
// free, default 0) instead of one highest-priority stream each, so no chain's own work (on-demand
// encodes, fix-up passes) shares the step batcher's hardware queue.  Null when unset.
static hipStream_t own_masked_stream(bool* shared) {
  static const int pool = getenv("WDR_OWN_POOL") ? atoi(getenv("WDR_OWN_POOL")) : -1;
  static const int n_res = getenv("WDR_OWN_MASK") ? atoi(getenv("WDR_OWN_MASK")) : 0;
  *shared = false;
  if (pool < 0) return nullptr;
  return masked_pool_stream("own", n_res, pool, shared);
}

// WDR_ODM_POOL (default 4): a long segment's later windows (encoded on demand: they depend on
// the decoded seek) run on P CU-masked streams (dedicated hardware queues, WDR_ODM_MASK CUs left
// free, default 32 as the encode-ahead pool), not on the state's own highest-priority stream.  A
// window's encoder (~70 launches, several ms) on the state stream shared a hardware queue with
// the step batcher, which runs its packets in order, so every batched step queued behind it
// waited (configs[2]'s VAD line: long merged segments; profiles/r05/vad_line_queues.txt,
// profiles/r06/ab_lines_hwq.txt).  -1: the state stream (as before).
static hipStream_t odm_masked_stream(bool* shared) {
  static const int pool = getenv("WDR_ODM_POOL") ? atoi(getenv("WDR_ODM_POOL")) : 4;
  static const int n_res = getenv("WDR_ODM_MASK") ? atoi(getenv("WDR_ODM_MASK")) : 32;
  *shared = false;
  if (pool < 0) return nullptr;
  int dev = 0, ncu = 0;
  WDR_HIP(hipGetDevice(&dev));
  WDR_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  if (ncu != 256 && !getenv("WDR_ODM_POOL")) return nullptr;   // tuned on MI355X
  return masked_pool_stream("odm", n_res, pool, shared);
}

DevMem::DevMem(size_t n) : bytes(n) {
  if (n) {
    std::lock_guard<std::recursive_mutex> g(hip_alloc_mutex());
    WDR_HIP(hipMalloc(&p, n));
  }
}
DevMem::~DevMem() {
  if (p) {
    std::lock_guard<std::recursive_mutex> g(hip_alloc_mutex());
    (void)hipFree(p);
  }
}
DevMem& DevMem::operator=(DevMem&& o) noexcept {
  if (this != &o) {
    if (p) {
      std::lock_guard<std::recursive_mutex> g(hip_alloc_mutex());
      (void)hipFree(p);
    }
    p = o.p;
    bytes = o.bytes;
    o.p = nullptr;
    o.bytes = 0;
  }
  return *this;
}

uint64_t fnv1a64(const std::string& s) {
  uint64_t h = 0xCBF29CE484222325ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 0x100000001B3ull;
  }
  return h;
}

// host restatement of librosa slaney mel filters (oracle/mel.py mel_filters)
static std::vector<float> mel_filters_host(int n_mels) {
  const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = 1000.0 / f_sp, logstep = std::log(6.4) / 27.0;
  auto hz2mel = [&](double f) { return f >= min_log_hz ? min_log_mel + std::log(f / min_log_hz) / logstep : f / f_sp; };
  auto mel2hz = [&](double m) { return m >= min_log_mel ? min_log_hz * std::exp(logstep * (m - min_log_mel)) : f_sp * m; };
  const int nb = 201;
  std::vector<double> fftf(nb), melf(n_mels + 2);
  for (int i = 0; i < nb; ++i) fftf[i] = 8000.0 * i / (nb - 1);
  const double m0 = hz2mel(0.0), m1 = hz2mel(8000.0);
  for (int i = 0; i < n_mels + 2; ++i) melf[i] = mel2hz(m0 + (m1 - m0) * i / (n_mels + 1));
  std::vector<float> w((size_t)n_mels * nb);
  for (int i = 0; i < n_mels; ++i) {
    const double enorm = 2.0 / (melf[i + 2] - melf[i]);
    for (int k = 0; k < nb; ++k) {
      const double lower = -(melf[i] - fftf[k]) / (melf[i + 1] - melf[i]);
      const double upper = (melf[i + 2] - fftf[k]) / (melf[i + 2] - melf[i + 1]);
      const double v = std::max(0.0, std::min(lower, upper));
      w[(size_t)i * nb + k] = (float)(v * enorm);
    }
  }
  return w;
}

// ------------------------------------------------------------------ context (weights)
namespace {
struct Alloc {
  size_t off = 0;
  std::vector<std::pair<size_t*, size_t>> dummy;
  size_t take(size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  }
};
}  // namespace

Context::Context(const std::string& model_name, const HParams& hp, const ContextParams& p, const GgmlFile* gf)
    : name(model_name), cp(p), vocab(hp.n_vocab) {
  WDR_CHECK(cp.use_gpu, "libwdr has no CPU backend: use_gpu=false is not supported (the CPU restatement is test-only)");
  WDR_HIP(hipSetDevice(cp.gpu_device));
  {
    // the latency-bound decode chain runs at the highest priority; the encode-ahead
    // stream (State) fills the CUs it leaves idle
    int lo = 0, hi = 0;
    WDR_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    WDR_HIP(hipStreamCreateWithPriority(&stream, hipStreamNonBlocking, hi));
    stream_note("context", stream);
    // WDR_PRIME_LOWQ (A/B): a lowest-priority stream created -- and its hardware queue
    // instantiated by one launch -- right after the context's own, before the step batcher's
    // and the states' streams
    if (getenv("WDR_PRIME_LOWQ") && atoi(getenv("WDR_PRIME_LOWQ")) != 0) {
      WDR_HIP(hipStreamCreateWithPriority(&low_prime, hipStreamNonBlocking, lo));
      DevMem one(16);
      WDR_HIP(hipMemsetAsync(one.p, 0, 16, low_prime));
      WDR_HIP(hipStreamSynchronize(low_prime));
    }
    // Hardware queues in a fixed order (WDR_PRIME_POOLS, default "lnh" on MI355X; "0" = off):
    // HIP serves each stream priority from a pool of 4 hardware queues; which of them first carried
    // work, and in what order, followed whichever thread launched first -- and that order set a
    // 15-25 % difference in every batched decode launch for the rest of the process (measured;
    // the mechanism inside the command processor is not visible from the runtime).  Every queue
    // of the pools gets its first work here, lowest priority first, then normal, then highest,
    // by one 1-block launch on each of 4 streams per level (kept, so the pools' refcounts stay
    // even).  Measured (profiles/r06/ab_lines_hwq.txt, "Finding the cause" and after): any order
    // with the lowest pool before the highest (lnh / nlh / lhn) runs both the diarized line and
    // configs[2]'s VAD line at 882-895 xRT; highest first (hnl / hln) runs both at 715-742;
    // lowest only fixes the VAD line (883) and costs the diarized one (754) -- the spread the
    // stream-placement experiments of this round kept landing on.
    const char* po_env = getenv("WDR_PRIME_POOLS");
    int ncu_p = 0;
    WDR_HIP(hipDeviceGetAttribute(&ncu_p, hipDeviceAttributeMultiprocessorCount, cp.gpu_device));
    const char* po = po_env ? po_env : (ncu_p == 256 ? "lnh" : "");
    if (po[0] && std::string(po) != "0") {
      DevMem sink(4096);
      for (const char* c = po; *c; ++c) {
        for (int k = 0; k < 4; ++k) {
          hipStream_t ps = nullptr;
          if (*c == 'n') WDR_HIP(hipStreamCreateWithFlags(&ps, hipStreamNonBlocking));
          else WDR_HIP(hipStreamCreateWithPriority(&ps, hipStreamNonBlocking, *c == 'l' ? lo : hi));
          WDR_CHECK(*c == 'l' || *c == 'n' || *c == 'h', "WDR_PRIME_POOLS: letters l / n / h");
          stream_note(*c == 'l' ? "prime-low" : *c == 'n' ? "prime-normal" : "prime-high", ps);
          launch_busy(1, 1000, sink.as<float>(), ps);
          prime_streams.push_back(ps);
        }
      }
      for (hipStream_t ps : prime_streams) WDR_HIP(hipStreamSynchronize(ps));
    }
    // WDR_DTWQ_EARLY (A/B): the DTW queue (its lowest-priority stream) made at the end of the
    // constructor, before the batcher and the states
  }
  Model& m = model;
  m.hp = hp;
  const int d = hp.n_audio_state, dt = hp.n_text_state;
  WDR_CHECK(d == dt, "encoder and decoder widths must match");
  WDR_CHECK(hp.n_audio_state / hp.n_audio_head == 64 && hp.n_text_state / hp.n_text_head == 64, "d_head must be 64");
  WDR_CHECK(d % 128 == 0, "model width must be a multiple of 128");
  m.kp1 = ((hp.n_mels * 3 + 31) / 32) * 32;
  const int L = hp.n_text_layer;

  // ---- layout
  Alloc A;
  auto H = [&](size_t n) { return A.take(n * 2); };
  auto F = [&](size_t n) { return A.take(n * 4); };
  const size_t o_c1w = H((size_t)d * m.kp1), o_c1b = F(d), o_c2w = H((size_t)d * 3 * d), o_c2b = F(d);
  const size_t o_epos = F((size_t)hp.n_audio_ctx * d), o_lnpg = F(d), o_lnpb = F(d);
  struct EO { size_t qkv, bqkv, o, bo, f1, bf1, f2, bf2, l1g, l1b, l2g, l2b; };
  std::vector<EO> eo(hp.n_audio_layer);
  for (auto& e : eo) {
    e.qkv = H((size_t)3 * d * d); e.bqkv = F(3 * d); e.o = H((size_t)d * d); e.bo = F(d);
    e.f1 = H((size_t)4 * d * d); e.bf1 = F(4 * d); e.f2 = H((size_t)4 * d * d); e.bf2 = F(d);
    e.l1g = F(d); e.l1b = F(d); e.l2g = F(d); e.l2b = F(d);
  }
  struct DO { size_t qkv, bqkv, o, bo, xq, bxq, xo, bxo, f1, bf1, f2, bf2, l1g, l1b, l2g, l2b, l3g, l3b; };
  std::vector<DO> dd(L);
  for (auto& e : dd) {
    e.qkv = H((size_t)3 * dt * dt); e.bqkv = F(3 * dt); e.o = H((size_t)dt * dt); e.bo = F(dt);
    e.xq = H((size_t)dt * dt); e.bxq = F(dt); e.xo = H((size_t)dt * dt); e.bxo = F(dt);
    e.f1 = H((size_t)4 * dt * dt); e.bf1 = F(4 * dt); e.f2 = H((size_t)4 * dt * dt); e.bf2 = F(dt);
    e.l1g = F(dt); e.l1b = F(dt); e.l2g = F(dt); e.l2b = F(dt); e.l3g = F(dt); e.l3b = F(dt);
  }
  const size_t o_xkv = H((size_t)L * 2 * dt * d), o_bxkv = F((size_t)L * 2 * dt);
  const size_t o_tok = H((size_t)hp.n_vocab * dt), o_dpos = F((size_t)hp.n_text_ctx * dt);
  const size_t o_lng = F(dt), o_lnb = F(dt);
  const size_t o_filt = F((size_t)hp.n_mels * 201), o_hann = F(400), o_cos = F(400), o_sin = F(400);
  m.weight_bytes = A.off;
  m.storage = DevMem(A.off);
  char* base = m.storage.as<char>();
  auto h16 = [&](size_t o) { return (f16*)(base + o); };
  auto f32 = [&](size_t o) { return (float*)(base + o); };
  m.conv1_w = h16(o_c1w); m.conv1_b = f32(o_c1b); m.conv2_w = h16(o_c2w); m.conv2_b = f32(o_c2b);
  m.enc_pos = f32(o_epos); m.ln_post_g = f32(o_lnpg); m.ln_post_b = f32(o_lnpb);
  for (auto& e : eo)
    m.enc.push_back({h16(e.qkv), h16(e.o), h16(e.f1), h16(e.f2), f32(e.bqkv), f32(e.bo), f32(e.bf1), f32(e.bf2),
                     f32(e.l1g), f32(e.l1b), f32(e.l2g), f32(e.l2b)});
  for (auto& e : dd)
    m.dec.push_back({h16(e.qkv), h16(e.o), h16(e.xq), h16(e.xo), h16(e.f1), h16(e.f2), f32(e.bqkv), f32(e.bo),
                     f32(e.bxq), f32(e.bxo), f32(e.bf1), f32(e.bf2), f32(e.l1g), f32(e.l1b), f32(e.l2g), f32(e.l2b),
                     f32(e.l3g), f32(e.l3b)});
  m.w_xkv = h16(o_xkv); m.b_xkv = f32(o_bxkv); m.tok_emb = h16(o_tok); m.dec_pos = f32(o_dpos);
  m.ln_g = f32(o_lng); m.ln_b = f32(o_lnb);
  m.mel_filters = f32(o_filt); m.hann = f32(o_hann); m.cos_tab = f32(o_cos); m.sin_tab = f32(o_sin);

  // ---- weights: from a whisper.cpp ggml file (gf), else synthetic (oracle/weights.py naming +
  // hash).  Both paths name every tensor as whisper.cpp does.
  hipStream_t s = stream;
  const double sq3 = std::sqrt(3.0);
  auto fill = [&](void* dst, const std::string& nm, long long rows, int src_cols, int dst_cols, bool is16, double sd) {
    if (!gf) {
      launch_synth_fill(dst, rows, src_cols, dst_cols, fnv1a64(nm), (float)(sd * sq3), is16, 0, 0.f, s);
      return;
    }
    const int64_t n = rows * (int64_t)src_cols;
    if (is16) {
      std::vector<uint16_t> v = gf->as_f16(nm, n), padded;
      if (dst_cols != src_cols) {
        padded.assign((size_t)rows * dst_cols, 0);
        for (long long r = 0; r < rows; ++r) memcpy(&padded[r * dst_cols], &v[r * src_cols], (size_t)src_cols * 2);
        v.swap(padded);
      }
      WDR_HIP(hipMemcpy(dst, v.data(), v.size() * 2, hipMemcpyHostToDevice));
    } else {
      WDR_CHECK(dst_cols == src_cols, "ggml load: padded f32 tensor");
      const std::vector<float> v = gf->as_f32(nm, n);
      WDR_HIP(hipMemcpy(dst, v.data(), v.size() * 4, hipMemcpyHostToDevice));
    }
  };
  auto cfill = [&](float* dst, long long n, float v) { launch_synth_fill(dst, 1, (int)n, (int)n, 0, 0.f, false, 1, v, s); };
  // LayerNorm parameters: gamma 1 / beta 0 in synthetic mode, the named tensor from a file
  auto lnfill = [&](float* dst, const std::string& nm, long long n, float v) {
    if (gf) fill(dst, nm, 1, (int)n, (int)n, false, 0.0);
    else cfill(dst, n, v);
  };
  const double sd = cp.weight_std;
  fill(m.conv1_w, "encoder.conv1.weight", d, hp.n_mels * 3, m.kp1, true, sd);
  fill(m.conv1_b, "encoder.conv1.bias", 1, d, d, false, sd);
  fill(m.conv2_w, "encoder.conv2.weight", d, 3 * d, 3 * d, true, sd);
  fill(m.conv2_b, "encoder.conv2.bias", 1, d, d, false, sd);
  fill(m.enc_pos, "encoder.positional_embedding", hp.n_audio_ctx, d, d, false, sd);
  for (int i = 0; i < hp.n_audio_layer; ++i) {
    const std::string p = "encoder.blocks." + std::to_string(i) + ".";
    const EncLayer& e = m.enc[i];
    fill(e.w_qkv, p + "attn.query.weight", d, d, d, true, sd);
    fill(e.w_qkv + (size_t)d * d, p + "attn.key.weight", d, d, d, true, sd);
    fill(e.w_qkv + (size_t)2 * d * d, p + "attn.value.weight", d, d, d, true, sd);
    fill(e.b_qkv, p + "attn.query.bias", 1, d, d, false, sd);
    cfill(e.b_qkv + d, d, 0.f);
    fill(e.b_qkv + 2 * d, p + "attn.value.bias", 1, d, d, false, sd);
    fill(e.w_o, p + "attn.out.weight", d, d, d, true, sd);
    fill(e.b_o, p + "attn.out.bias", 1, d, d, false, sd);
    fill(e.w_fc1, p + "mlp.0.weight", 4 * d, d, d, true, sd);
    fill(e.b_fc1, p + "mlp.0.bias", 1, 4 * d, 4 * d, false, sd);
    fill(e.w_fc2, p + "mlp.2.weight", d, 4 * d, 4 * d, true, sd);
    fill(e.b_fc2, p + "mlp.2.bias", 1, d, d, false, sd);
    lnfill(e.ln1_g, p + "attn_ln.weight", d, 1.f); lnfill(e.ln1_b, p + "attn_ln.bias", d, 0.f);
    lnfill(e.ln2_g, p + "mlp_ln.weight", d, 1.f); lnfill(e.ln2_b, p + "mlp_ln.bias", d, 0.f);
  }
  lnfill(m.ln_post_g, "encoder.ln_post.weight", d, 1.f);
  lnfill(m.ln_post_b, "encoder.ln_post.bias", d, 0.f);
  fill(m.tok_emb, "decoder.token_embedding.weight", hp.n_vocab, dt, dt, true, cp.emb_std);
  fill(m.dec_pos, "decoder.positional_embedding", hp.n_text_ctx, dt, dt, false, sd);
  for (int i = 0; i < L; ++i) {
    const std::string p = "decoder.blocks." + std::to_string(i) + ".";
    const DecLayer& e = m.dec[i];
    fill(e.w_qkv, p + "attn.query.weight", dt, dt, dt, true, sd);
    fill(e.w_qkv + (size_t)dt * dt, p + "attn.key.weight", dt, dt, dt, true, sd);
    fill(e.w_qkv + (size_t)2 * dt * dt, p + "attn.value.weight", dt, dt, dt, true, sd);
    fill(e.b_qkv, p + "attn.query.bias", 1, dt, dt, false, sd);
    cfill(e.b_qkv + dt, dt, 0.f);
    fill(e.b_qkv + 2 * dt, p + "attn.value.bias", 1, dt, dt, false, sd);
    fill(e.w_o, p + "attn.out.weight", dt, dt, dt, true, sd);
    fill(e.b_o, p + "attn.out.bias", 1, dt, dt, false, sd);
    fill(e.w_xq, p + "cross_attn.query.weight", dt, dt, dt, true, sd);
    fill(e.b_xq, p + "cross_attn.query.bias", 1, dt, dt, false, sd);
    fill(m.w_xkv + (size_t)i * 2 * dt * d, p + "cross_attn.key.weight", dt, d, d, true, sd);
    fill(m.w_xkv + (size_t)(i * 2 + 1) * dt * d, p + "cross_attn.value.weight", dt, d, d, true, sd);
    cfill(m.b_xkv + (size_t)i * 2 * dt, dt, 0.f);
    fill(m.b_xkv + (size_t)(i * 2 + 1) * dt, p + "cross_attn.value.bias", 1, dt, dt, false, sd);
    fill(e.w_xo, p + "cross_attn.out.weight", dt, dt, dt, true, sd);
    fill(e.b_xo, p + "cross_attn.out.bias", 1, dt, dt, false, sd);
    fill(e.w_fc1, p + "mlp.0.weight", 4 * dt, dt, dt, true, sd);
    fill(e.b_fc1, p + "mlp.0.bias", 1, 4 * dt, 4 * dt, false, sd);
    fill(e.w_fc2, p + "mlp.2.weight", dt, 4 * dt, 4 * dt, true, sd);
    fill(e.b_fc2, p + "mlp.2.bias", 1, dt, dt, false, sd);
    lnfill(e.ln1_g, p + "attn_ln.weight", dt, 1.f); lnfill(e.ln1_b, p + "attn_ln.bias", dt, 0.f);
    lnfill(e.ln2_g, p + "cross_attn_ln.weight", dt, 1.f); lnfill(e.ln2_b, p + "cross_attn_ln.bias", dt, 0.f);
    lnfill(e.ln3_g, p + "mlp_ln.weight", dt, 1.f); lnfill(e.ln3_b, p + "mlp_ln.bias", dt, 0.f);
  }
  lnfill(m.ln_g, "decoder.ln.weight", dt, 1.f);
  lnfill(m.ln_b, "decoder.ln.bias", dt, 0.f);
  // mel front-end constants
  std::vector<float> filt = mel_filters_host(hp.n_mels), hann(400), cs(400), sn(400);
  if (gf) {   // the file's own filter bank (whisper.cpp uses it as stored)
    WDR_CHECK(gf->n_mel == hp.n_mels && gf->n_fft == 201, "ggml load: mel filter bank shape");
    filt = gf->filters;
    // the file's vocabulary replaces the synthetic token texts (special tokens past the file's
    // list keep whisper.cpp's generated names); token_to_id rebuilt in id order, last wins
    for (size_t i = 0; i < gf->vocab.size() && (int)i < vocab.n_vocab; ++i) vocab.id_to_token[i] = gf->vocab[i];
    vocab.token_to_id.clear();
    for (int i = 0; i < vocab.n_vocab; ++i) vocab.token_to_id[vocab.id_to_token[i]] = i;
  }
  for (int i = 0; i < 400; ++i) {
    hann[i] = (float)(0.5 * (1.0 - std::cos(2.0 * M_PI * i / 400.0)));
    cs[i] = (float)std::cos(2.0 * M_PI * i / 400.0);
    sn[i] = (float)(-std::sin(2.0 * M_PI * i / 400.0));
  }
  WDR_HIP(wdr_memcpy_async(m.mel_filters, filt.data(), filt.size() * 4, hipMemcpyHostToDevice, s));
  WDR_HIP(wdr_memcpy_async(m.hann, hann.data(), 1600, hipMemcpyHostToDevice, s));
  WDR_HIP(wdr_memcpy_async(m.cos_tab, cs.data(), 1600, hipMemcpyHostToDevice, s));
  WDR_HIP(wdr_memcpy_async(m.sin_tab, sn.data(), 1600, hipMemcpyHostToDevice, s));

  // ---- DTW preset
  if (cp.dtw) {
    aheads = alignment_heads_for(name);
    aheads_per_layer.assign(L, {});
    for (auto& a : aheads) {
      WDR_CHECK(a.first < L && a.second < hp.n_text_head, "alignment head out of range for this model");
      aheads_per_layer[a.first].push_back(a.second);
    }
    std::vector<int> flat;
    for (int l = 0; l < L; ++l) {
      aheads_dev_off.push_back((int)flat.size());
      for (int h : aheads_per_layer[l]) flat.push_back(h);
    }
    aheads_dev = DevMem(std::max<size_t>(4, flat.size() * 4));
    if (!flat.empty()) WDR_HIP(wdr_memcpy_async(aheads_dev.p, flat.data(), flat.size() * 4, hipMemcpyHostToDevice, s));
  }
  WDR_HIP(hipStreamSynchronize(s));
  {
    // KV pool for the decode chains of every State of this context (multi-chain pipeline)
    const char* e = getenv("WDR_DECODE_CHAINS");
    max_chains = std::max(1, std::min(64, e ? atoi(e) : 40));   // 24 -> 40: +2.6 % (profiles/r04/ab_chains*.txt)
    const char* nb = getenv("WDR_BATCHERS");
    n_batchers = std::max(1, std::min(8, nb ? atoi(nb) : 1));
    prefill_split = getenv("WDR_PREFILL_SPLIT") && atoi(getenv("WDR_PREFILL_SPLIT")) != 0;
    fp8_encoder = getenv("WDR_FP8_ENCODER") && atoi(getenv("WDR_FP8_ENCODER")) != 0;
    fp8_plan = fp8_plan_for(hp.n_audio_layer);
    const size_t per = (size_t)hp.n_text_layer * 21 * hp.n_text_ctx * hp.n_text_state;   // NSLOT = 21
    kv_k = DevMem(per * max_chains * 2);
    kv_v = DevMem(per * max_chains * 2);
    kv_seq_stride = (long long)hp.n_text_ctx * hp.n_text_state;
    kv_layer_stride = (long long)max_chains * 21 * kv_seq_stride;
  }
  if (getenv("WDR_DTWQ_EARLY") && atoi(getenv("WDR_DTWQ_EARLY")) != 0 && !aheads.empty()) {
    DtwQueue& q = dtw_queue();
    (void)q;
  }
}

Context::~Context() {
  dtwq.reset();
  batchers.clear();
  prefill_b.reset();
  if (stream) (void)hipStreamDestroy(stream);
  if (low_prime) (void)hipStreamDestroy(low_prime);
  for (hipStream_t ps : prime_streams) (void)hipStreamDestroy(ps);
}

// ------------------------------------------------------------------ state buffers
static constexpr int RMAX = 448;   // max decoder rows in one forward (n_text_ctx)
static constexpr int NSEQ = 8;     // max decoder rows in one step
static constexpr int NSLOT = 21;   // self-attention KV-cache sequences (beams + reorder scratch + DTW + lang)
static constexpr int DTW_SEQ = 16;  // the DTW re-forward's own sequence (runs on its own stream)
static constexpr int LANG_SEQ = 17; // encode-ahead language detection: sequences 17..20, one per window of a batch


struct State::Impl {
  int d, L, H, V, n_mels, kp1;
  // encoder activations for nb windows stacked along M (rows b*1500 ..): one set for the
  // encode-ahead stream (nb = kBatch), one single-window set for on-demand windows
  struct EncBufs {
    int nb = 0;
    DevMem im2col, c1, ex, eh, eqkv, eatt, emlp;
    // fp8 encoder (MX e4m3): the d-wide GEMM operand (LN1 / attention output / LN2) and the 4d-wide
    // fc2 operand (fc1's GELU epilogue), each with its scale image [K/128][rows rounded to 256]
    DevMem q8a, qsa, q8m, qsm;
  };
  EncBufs eb, e1;
  // cross-K/V ring: one slot per in-flight speech segment, [slot][1500][L*2d] f16, plus a
  // scratch slot (index S) for un-planned calls.  Each slot also owns its segment's samples,
  // log-mel and global max, so later windows of a long segment encode from the slot.
  struct Slot {
    DevMem x, mel, gmax, pcm;
    int16_t* h_pcm = nullptr;   // pinned staging for the H2D copy of the segment's PCM
    // the segment's signal energy (heuristic timestamps), computed on the encode-ahead stream
    // and copied back before `ready`: the decode chain reads it without a GPU round trip
    DevMem energy_d;
    float* h_energy = nullptr;
    int energy_cap = 0, energy_n = -1;
    int pcm_cap = 0, x_cap = 0, mel_cap = 0, n_fft_frames = 0, n_samples = 0;
    hipEvent_t ready = nullptr, freed = nullptr;
    std::shared_ptr<DtwQJob> dtw;   // the queued DTW re-forward that reads this slot (DtwQueue)
  };
  std::vector<Slot> slots;
  int S = 0;                  // ring slots (multiple of kBatch)
  DevMem xkv_ring;
  size_t xkv_slot_elems = 0;
  int cur = 0;                // slot the decoder reads (cross-K/V, samples)
  bool own_shared = false;    // own from the WDR_OWN_POOL pool
  bool es_shared = false;     // es from the WDR_ENC_MASK pool (not destroyed with the state)
  hipStream_t es = nullptr;   // encode-ahead stream (lower priority than the decode stream)
  struct Plan {
    std::vector<const int16_t*> pcm;
    std::vector<int> n;
    size_t next_enq = 0;
    bool detect_lang = false;   // lang "auto": the SOT pass runs right after each window-0 encode
  } plan;
  // encode-ahead language detection: its own prefill working set and the 100 language
  // logits of each slot's window 0 (pinned, written by the encode stream before `ready`)
  RowsBufs lb;                   // its rows forward (kBatch rows)
  std::unique_ptr<RowBatch> tlb;
  // full encode-ahead batches (kBatch windows: encoder + cross-K/V + language detection) as one
  // hipGraph per ring slot group (and fp8 mode): ~560 launches become one replay, which keeps
  // the chain thread's host time between its batched steps short (top_up runs on it).  Each
  // group has its own language-detection table (its slots' cross-K/V pointers are constant).
  struct EncGraph {
    hipGraphExec_t exec = nullptr;
    std::unique_ptr<RowBatch> tl;
  };
  std::map<int, EncGraph> enc_graphs;
  hipStream_t es_cap = nullptr;   // the stream those graphs are captured on (never launched on)
  // WDR_CHAIN_LOG: DTW-queue waits / encoder launch host time (ns; the encode-ahead thread adds too)
  std::atomic<long long> t_fence{0}, t_enc_launch{0};
  // the encode-ahead host thread: issues the plan's batches (top_up_batch) up to the lookahead of
  // the highest segment whose full() has started (enc_target), so the ~600 launches / copies of
  // a batch leave the chain thread (which waits only when its segment's batch is not issued yet)
  std::thread enc_th;
  std::mutex enc_mu;
  std::condition_variable enc_cv;
  int enc_target = -1;
  bool enc_stop = false, enc_busy = false;
  std::exception_ptr enc_err;
  std::atomic<long long> enc_windows{0};
  std::atomic<long long> lang_passes{0}, lang_rows{0};   // encode-ahead language-detection passes
  float* h_lang = nullptr;      // [(S + 1)][100]
  // lang_src[slot]: the plan segment whose language logits h_lang[slot] holds (-1: none yet) --
  // from the encode-ahead batch's detection pass, or from a detection row that rode in one of
  // the chain's batched steps (lang_piggyback)
  std::vector<int> lang_src;    // [S + 1]
  // set by full() for the segment's decode (lang_piggyback): attach the next segment's detection
  // row to a batched request / take its logits after the step (decode_beam uses them too)
  std::function<bool(StepBatcher::Req&)> lang_ride;
  std::function<void(const StepBatcher::Req&)> lang_after;
  DevMem energy_d; int energy_cap = 0;
  const f16* xkv() const { return xkv_ring.as<f16>() + (size_t)(xsel >= 0 ? S + 1 : cur) * xkv_slot_elems; }
  // a segment's later windows (encoded on demand) alternate between the slot's cross-K/V and
  // the chain's spare one (ring index S + 1; WDR_ODM_ALT): xsel >= 0 -> the spare, alt_dtw the
  // queued DTW pass that reads it
  int xsel = -1;
  std::shared_ptr<DtwQJob> alt_dtw;
  // decoder: this state's own rows forwards (prompt prefills, beam / sampling steps, test seams)
  // on the decode stream, and the DTW re-forwards on the DTW stream, each with its own working
  // set and row tables (rows.h)
  RowsBufs mb, db;
  std::unique_ptr<RowBatch> tb, tdb;
  DevMem work, tokout, ctl, cap;
  DevMem beamc, kvpairs;       // beam candidates [NSEQ][BEAM_KMAX], KV reorder (src, dst) pairs
  BeamCand* h_beam = nullptr;
  DevMem sprobs, slogp;        // [NSEQ][V] sampled rows (t > 0)
  std::vector<float> hp_probs, hp_logp;
  std::mt19937 rng[NSEQ];      // whisper_decoder::rng
  int* h_pairs = nullptr;
  f16* kc = nullptr;          // this chain's sequences in the context's KV pool (layer 0)
  f16* vc = nullptr;
  int nslot_tot = 0;          // sequences per layer in the pool (layer stride / seq_stride)
  long long seq_stride = 0;   // elements per (layer, seq)
  hipStream_t own = nullptr;  // this state's decode stream
  hipStream_t eo = nullptr;   // on-demand window encodes (WDR_ODM_POOL; null: the decode stream)
  bool eo_shared = false;
  // dtw
  DevMem nrm, xdtw, times;
  struct DtwSet {
    DevMem cap, nrm, xdtw, times;
  } dset;
  hipStream_t sd = nullptr;        // DTW stream
  hipEvent_t ev_sync = nullptr;    // decode-stream point the DTW stream waits for
  hipEvent_t ev_dtw = nullptr;     // last DTW job enqueued (on-demand encodes wait for it)
  hipEvent_t ev_p0 = nullptr, ev_p1 = nullptr;   // prompt-prefill timing
  struct DtwJob {
    int i0 = 0, n = 0;             // result_all range of the full() call that produced it
    int* blk = nullptr;            // pinned: tokens [3*RMAX] then times [RMAX + 8]
    hipEvent_t done = nullptr;
    std::shared_ptr<DtwQJob> q;    // queued to the context's DtwQueue (multi-chain run)
  };
  std::vector<std::shared_ptr<DtwQJob>> qlive;   // queued re-forwards that may still write DTW_SEQ
  std::vector<DtwJob> jobs;        // enqueued by the current full() call
  // multi-chain run: the last window's DTW re-forward waits to ride in the chain's next batcher
  // request (the next segment's prompt prefill), one request instead of two per segment
  struct PendingDtw {
    bool on = false;
    std::vector<int> toks;
    const f16* xkv = nullptr;
    int slot = -1;                 // slot whose release waits for the re-forward (-1: none)
    int sot_len = 0, seek = 0, n_audio = 0;
    int* blk = nullptr;
    hipEvent_t done = nullptr;
  } pend;
  std::vector<int*> blk_pool;
  std::vector<hipEvent_t> ev_pool;
  // host pinned
  TokOut* h_tok = nullptr;
  LogitsCtl* h_ctl = nullptr;
  int* h_times = nullptr;
  VocabIds vids;
  struct StepGraph {
    hipGraphExec_t exec = nullptr;
    VocabIds vids{};
  };
  std::map<int, StepGraph> graphs;   // key: (K, R); the rows' slots are table entries
};

// ------------------------------------------------------------------ fp8 encoder weights
// The fp8 plan: one nibble per encoder layer (Context::F8_*).  Default: every projection of every
// layer.  WDR_FP8_PLAN = one hex digit per layer (layer 0 first; missing layers take the last
// digit); else WDR_FP8_PROJ (hex nibble, default f) on every layer but the first WDR_FP8_F16_HEAD
// and the last WDR_FP8_F16_TAIL, which stay f16.
std::vector<uint8_t> fp8_plan_for(int n_layer) {
  std::vector<uint8_t> plan(n_layer, 0xf);
  if (const char* e = getenv("WDR_FP8_PLAN"); e && *e) {
    uint8_t last = 0xf;
    for (int l = 0; l < n_layer; ++l) {
      if (e[l] && isxdigit((unsigned char)e[l])) {
        const char c = (char)tolower(e[l]);
        last = (uint8_t)(c <= '9' ? c - '0' : c - 'a' + 10);
      } else if (e[l]) {
        throw std::runtime_error("WDR_FP8_PLAN: one hex digit per encoder layer");
      }
      plan[l] = last;
      if (!e[l]) {
        for (int r = l + 1; r < n_layer; ++r) plan[r] = last;
        break;
      }
    }
    return plan;
  }
  const uint8_t proj = getenv("WDR_FP8_PROJ") ? (uint8_t)(strtol(getenv("WDR_FP8_PROJ"), nullptr, 16) & 0xf) : 0xf;
  const int head = getenv("WDR_FP8_F16_HEAD") ? atoi(getenv("WDR_FP8_F16_HEAD")) : 0;
  const int tail = getenv("WDR_FP8_F16_TAIL") ? atoi(getenv("WDR_FP8_F16_TAIL")) : 0;
  for (int l = 0; l < n_layer; ++l) plan[l] = (l < head || l >= n_layer - tail) ? 0 : proj;
  return plan;
}

void Context::fp8_build() {
  WDR_HIP(hipSetDevice(cp.gpu_device));
  const HParams& hp = model.hp;
  const int d = hp.n_audio_state;
  // every weight row (output channel) as e4m3 with one E8M0 scale per 32 k, scale image
  // [K/128][N] (launch_quant_f8); k_gemm8 applies both operands' block scales in the MFMA
  auto quant = [&](const f16* w, int N, int K) {
    Fp8W q;
    q.w = DevMem((size_t)N * K);
    q.s = DevMem((size_t)K / 128 * N * 4);
    launch_quant_f8(w, K, N, K, q.w.as<uint8_t>(), K, q.s.as<uint32_t>(), N, stream);
    return q;
  };
  std::vector<Fp8Layer> L(hp.n_audio_layer);
  for (int l = 0; l < hp.n_audio_layer; ++l) {
    const EncLayer& e = model.enc[l];
    L[l].qkv = quant(e.w_qkv, 3 * d, d);
    L[l].o = quant(e.w_o, d, d);
    L[l].fc1 = quant(e.w_fc1, 4 * d, d);
    L[l].fc2 = quant(e.w_fc2, d, 4 * d);
  }
  WDR_HIP(hipStreamSynchronize(stream));
  fp8_layers_ = std::move(L);
}
const std::vector<Context::Fp8Layer>& Context::fp8_layers() {
  std::lock_guard<std::mutex> g(fp8_mu_);
  if (fp8_layers_.empty()) fp8_build();
  return fp8_layers_;
}

static constexpr int kBatch = 4;     // encoder windows per encode-ahead launch (M = 6000 rows)
// the batch's language-detection pass gives every window its own KV sequence LANG_SEQ + r of the
// chain's NSLOT: a larger batch would write into the next chain's sequences (round 4's 8-window
// A/B faulted exactly so), so the pool layout bounds the batch at compile time
static_assert(LANG_SEQ + kBatch <= NSLOT, "encode-ahead batch: language-detection sequences past the chain's NSLOT");
static_assert(DTW_SEQ < LANG_SEQ && NSEQ * 2 <= DTW_SEQ, "KV sequences: decoders + reorder scratch, DTW, language");
static constexpr int kSlots = 16;    // in-flight segments in the cross-K/V ring (most)
// WDR_SLOTS: ring slots per chain (a multiple of kBatch, 4..16); default 16 up to 24 chains and 8
// above (large-v3: 40 chains x 9 slots x 245.8 MB = 88 GB of cross-K/V; 48 chains of 17 slots
// did not fit in 288 GB beside the KV pool, profiles/r04/ab_flash_occ.txt)
static int ring_slots(int max_chains) {
  const char* e = getenv("WDR_SLOTS");
  const int n = e ? atoi(e) / kBatch * kBatch : max_chains > 24 ? 8 : kSlots;
  return std::max(kBatch, std::min(kSlots, n));
}

static void alloc_enc(State::Impl::EncBufs& e, int nb, int d, int kp1) {
  e.nb = nb;
  e.im2col = DevMem((size_t)nb * 3000 * std::max(kp1, 3 * d) * 2);
  e.c1 = DevMem((size_t)nb * 3000 * d * 2);
  e.ex = DevMem((size_t)nb * 1500 * d * 4);
  e.eh = DevMem((size_t)nb * 1500 * d * 2);
  e.eqkv = DevMem((size_t)nb * 1500 * 3 * d * 2);
  e.eatt = DevMem((size_t)nb * 1500 * d * 2);
  e.emlp = DevMem((size_t)nb * 1500 * 4 * d * 2);
  // fp8 MX operands (configs[4]): rows padded to the GEMM's 256-row tiles for the scale images
  const size_t mp = (size_t)cdiv(nb * 1500, 256) * 256;
  e.q8a = DevMem(mp * d);
  e.qsa = DevMem((size_t)d / 128 * mp * 4);
  e.q8m = DevMem(mp * 4 * d);
  e.qsm = DevMem((size_t)4 * d / 128 * mp * 4);
}

State::State(Context& ctx, int chain_) : ctx_(ctx), s_(nullptr), m_(new Impl) {
  WDR_HIP(hipSetDevice(ctx.cp.gpu_device));
  const HParams& hp = ctx.model.hp;
  Impl& m = *m_;
  chain = chain_;
  WDR_CHECK(chain >= 0 && chain < ctx.max_chains, "decode chain index out of range");
  {
    // every state has its own highest-priority decode stream (chains run concurrently)
    int lo = 0, hi = 0;
    WDR_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    // WDR_OWN_PRIO=1|2 (A/B): the state's own stream at the normal / lowest priority
    static const int op = getenv("WDR_OWN_PRIO") ? atoi(getenv("WDR_OWN_PRIO")) : 0;
    m.own = own_masked_stream(&m.own_shared);
    if (m.own) {
    } else if (op == 1) WDR_HIP(hipStreamCreateWithFlags(&m.own, hipStreamNonBlocking));
    else WDR_HIP(hipStreamCreateWithPriority(&m.own, hipStreamNonBlocking, op == 2 ? lo : hi));
    s_ = m.own;
    stream_note("state-own", s_);
  }
  m.d = hp.n_text_state;
  m.L = hp.n_text_layer;
  m.H = hp.n_text_head;
  m.V = hp.n_vocab;
  m.n_mels = hp.n_mels;
  m.kp1 = ctx.model.kp1;
  const int d = m.d;
  alloc_enc(m.e1, 1, d, m.kp1);
  alloc_enc(m.eb, kBatch, d, m.kp1);
  m.S = ring_slots(ctx.max_chains);
  m.slots.resize(m.S + 1);
  for (auto& sl : m.slots) {
    sl.gmax = DevMem(16);
    WDR_HIP(hipEventCreateWithFlags(&sl.ready, hipEventDisableTiming));
    WDR_HIP(hipEventCreateWithFlags(&sl.freed, hipEventDisableTiming));
  }
  m.xkv_slot_elems = (size_t)1500 * m.L * 2 * d;
  m.xkv_ring = DevMem((m.S + 2) * m.xkv_slot_elems * 2);   // + the on-demand spare (xsel)
  m.cur = m.S;
  {
    // the encode-ahead stream at the lowest priority (WDR_ENC_PRIO=1: the middle of the range,
    // 2: the highest; A/B runs)
    int lo = 0, hi = 0;
    WDR_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    static const int ep = getenv("WDR_ENC_PRIO") ? atoi(getenv("WDR_ENC_PRIO")) : 0;
    const int prio = ep == 2 ? hi : ep == 1 ? (lo + hi) / 2 : lo;
    m.es = enc_masked_stream(&m.es_shared);
    if (!m.es) WDR_HIP(hipStreamCreateWithPriority(&m.es, hipStreamNonBlocking, prio));
    stream_note("state-es", m.es);
    m.eo = odm_masked_stream(&m.eo_shared);
  }
  // this state's rows forwards: prompt prefills / DTW re-forwards up to RMAX rows, steps of up
  // to NSEQ logit rows; the DTW set captures; language detection kBatch rows
  const int A = std::max<int>(1, (int)ctx.aheads.size());
  m.mb.alloc(RMAX, NSEQ, d, m.H, m.V);
  m.tb = std::make_unique<RowBatch>(RMAX, NSEQ, RMAX);
  m.db.alloc(RMAX, 1, d, m.H, m.V);
  m.tdb = std::make_unique<RowBatch>(RMAX, 1, RMAX);
  m.lb.alloc(kBatch, kBatch, d, m.H, m.V);
  m.tlb = std::make_unique<RowBatch>(kBatch, kBatch, 0);
  m.work = DevMem((size_t)NSEQ * m.V * 4);
  m.tokout = DevMem(NSEQ * sizeof(TokOut));
  m.ctl = DevMem(NSEQ * sizeof(LogitsCtl));
  m.cap = DevMem((size_t)A * RMAX * 1500 * 4);
  m.beamc = DevMem(NSEQ * BEAM_KMAX * sizeof(BeamCand));
  m.sprobs = DevMem((size_t)NSEQ * m.V * 4);
  m.slogp = DevMem((size_t)NSEQ * m.V * 4);
  m.rng[0] = std::mt19937(0);   // decoder 0: seeded once per state
  m.kvpairs = DevMem(2 * 2 * NSEQ * 4);
  WDR_HIP(hipHostMalloc((void**)&m.h_beam, NSEQ * BEAM_KMAX * sizeof(BeamCand), hipHostMallocDefault));
  WDR_HIP(hipHostMalloc((void**)&m.h_pairs, 2 * 2 * NSEQ * 4, hipHostMallocDefault));
  m.seq_stride = (long long)hp.n_text_ctx * d;
  m.nslot_tot = ctx.max_chains * NSLOT;
  m.kc = ctx.kv_k.as<f16>() + (size_t)chain * NSLOT * m.seq_stride;
  m.vc = ctx.kv_v.as<f16>() + (size_t)chain * NSLOT * m.seq_stride;
  {
    Impl::DtwSet& D = m.dset;
    D.cap = DevMem((size_t)A * RMAX * 1500 * 4);
    D.nrm = DevMem((size_t)A * RMAX * 1500 * 4);
    D.xdtw = DevMem((size_t)RMAX * 1500 * 4);
    D.times = DevMem((RMAX + 8) * 4);
    WDR_HIP(hipHostMalloc((void**)&m.h_lang, (size_t)(kSlots + 1) * 100 * 4, hipHostMallocDefault));
    m.lang_src.assign(kSlots + 1, -1);
    int lo = 0, hi = 0;
    WDR_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    WDR_HIP(hipStreamCreateWithPriority(&m.sd, hipStreamNonBlocking, lo));
    stream_note("state-sd", m.sd);
    WDR_HIP(hipEventCreateWithFlags(&m.ev_sync, hipEventDisableTiming));
    WDR_HIP(hipEventCreateWithFlags(&m.ev_dtw, hipEventDisableTiming));
    WDR_HIP(hipEventCreate(&m.ev_p0));
    WDR_HIP(hipEventCreate(&m.ev_p1));
  }
  WDR_HIP(hipHostMalloc((void**)&m.h_tok, NSEQ * sizeof(TokOut), hipHostMallocDefault));
  WDR_HIP(hipHostMalloc((void**)&m.h_ctl, NSEQ * sizeof(LogitsCtl), hipHostMallocDefault));
  WDR_HIP(hipHostMalloc((void**)&m.h_times, (RMAX + 8) * 4, hipHostMallocDefault));
  const Vocab& v = ctx.vocab;
  m.vids = VocabIds{v.n_vocab, v.eot, v.sot, v.translate, v.transcribe, v.solm, v.prev, v.nosp, v.not_, v.beg,
                    v.token_to_id.at(" "), v.sot + 1, 100, -1, 1};
}

State::~State() {
  if (m_ && m_->enc_th.joinable()) {
    {
      std::lock_guard<std::mutex> g(m_->enc_mu);
      m_->enc_stop = true;
    }
    m_->enc_cv.notify_all();
    m_->enc_th.join();
  }
  if (m_) {
    try {   // queued passes read this state's slots and write its pinned blocks
      for (auto& q : m_->qlive) {
        ctx_.dtw_queue().wait_issued(q);
        (void)hipEventSynchronize(q->done);
      }
    } catch (...) {
    }
    m_->qlive.clear();
    for (auto& g : m_->graphs)
      if (g.second.exec) (void)hipGraphExecDestroy(g.second.exec);
    if (m_->es) (void)hipStreamSynchronize(m_->es);
    for (auto& g : m_->enc_graphs)
      if (g.second.exec) (void)hipGraphExecDestroy(g.second.exec);
    if (m_->es_cap) (void)hipStreamDestroy(m_->es_cap);
    (void)hipHostFree(m_->h_tok);
    (void)hipHostFree(m_->h_ctl);
    (void)hipHostFree(m_->h_times);
    (void)hipHostFree(m_->h_beam);
    (void)hipHostFree(m_->h_pairs);
    if (m_->es) {
      (void)hipStreamSynchronize(m_->es);
      if (!m_->es_shared) (void)hipStreamDestroy(m_->es);
    }
    if (m_->sd) {
      (void)hipStreamSynchronize(m_->sd);
      (void)hipStreamDestroy(m_->sd);
    }
    if (m_->own) {
      (void)hipStreamSynchronize(m_->own);
      if (!m_->own_shared) (void)hipStreamDestroy(m_->own);
    }
    if (m_->eo) {
      (void)hipStreamSynchronize(m_->eo);
      if (!m_->eo_shared) (void)hipStreamDestroy(m_->eo);
    }
    for (auto& j : m_->jobs) {
      if (j.blk) m_->blk_pool.push_back(j.blk);
      if (j.done) m_->ev_pool.push_back(j.done);
    }
    for (int* b : m_->blk_pool) (void)hipHostFree(b);
    for (hipEvent_t e : m_->ev_pool) (void)hipEventDestroy(e);
    if (m_->ev_sync) (void)hipEventDestroy(m_->ev_sync);
    if (m_->h_lang) (void)hipHostFree(m_->h_lang);
    if (m_->ev_dtw) (void)hipEventDestroy(m_->ev_dtw);
    for (auto& sl : m_->slots) {
      if (sl.h_pcm) (void)hipHostFree(sl.h_pcm);
      if (sl.h_energy) (void)hipHostFree(sl.h_energy);
      if (sl.ready) (void)hipEventDestroy(sl.ready);
      if (sl.freed) (void)hipEventDestroy(sl.freed);
    }
  }
}

// ------------------------------------------------------------------ front-end
// Samples -> slot: f32 samples and the whole segment's log-mel (+ its global max, which
// normalises every window of the segment: whisper.cpp log_mel_spectrogram).
static void slot_mel(Context& ctx, State::Impl& m, State::Impl::Slot& sl, int n, hipStream_t s) {
  const int n_len = (n + 480000 + 400 - 400) / 160;
  const int n_eff = n + 200;
  sl.n_fft_frames = std::min(n_eff / 160 + 1, n_len);
  sl.n_samples = n;
  if (sl.n_fft_frames > sl.mel_cap) {
    sl.mel = DevMem((size_t)sl.n_fft_frames * m.n_mels * 4);
    sl.mel_cap = sl.n_fft_frames;
  }
  launch_gmax_init(sl.gmax.as<int>(), s);
  MelArgs a{sl.x.as<float>(), n, sl.n_fft_frames, m.n_mels, ctx.model.hann, ctx.model.cos_tab, ctx.model.sin_tab,
            ctx.model.mel_filters, sl.mel.as<float>(), sl.gmax.as<int>()};
  launch_mel(a, s);
}

static void slot_reserve_x(State::Impl::Slot& sl, int n) {
  if (n > sl.x_cap) {
    sl.x = DevMem((size_t)std::max(n, 1) * 4);
    sl.x_cap = n;
  }
}

// a slot's buffers for segments of up to n samples (PCM staging, samples, energy, log-mel)
static void slot_reserve_all(State::Impl::Slot& sl, int n, int n_mels) {
  if (n <= 0) return;
  std::lock_guard<std::recursive_mutex> g(hip_alloc_mutex());
  if (n > sl.pcm_cap) {
    if (sl.h_pcm) WDR_HIP(hipHostFree(sl.h_pcm));
    sl.h_pcm = nullptr;
    WDR_HIP(hipHostMalloc((void**)&sl.h_pcm, (size_t)n * 2, hipHostMallocDefault));
    sl.pcm = DevMem((size_t)n * 2);
    sl.pcm_cap = n;
  }
  slot_reserve_x(sl, n);
  if (n > sl.energy_cap) {
    if (sl.h_energy) WDR_HIP(hipHostFree(sl.h_energy));
    sl.h_energy = nullptr;
    WDR_HIP(hipHostMalloc((void**)&sl.h_energy, (size_t)n * 4, hipHostMallocDefault));
    sl.energy_d = DevMem((size_t)n * 4);
    sl.energy_cap = n;
  }
  const int frames = std::min((n + 200) / 160 + 1, (n + 480000) / 160);   // slot_mel's n_fft_frames
  if (frames > sl.mel_cap) {
    sl.mel = DevMem((size_t)frames * n_mels * 4);
    sl.mel_cap = frames;
  }
}

void State::compute_mel(const float* x_host, int n) {
  Impl& m = *m_;
  m.cur = m.S;
  stream_fence(s_, m.ev_dtw, host_fence());   // the scratch slot may still feed a DTW job
  Impl::Slot& sl = m.slots[m.S];
  slot_reserve_x(sl, n);
  if (n > 0) WDR_HIP(wdr_memcpy_async(sl.x.p, x_host, (size_t)n * 4, hipMemcpyHostToDevice, s_));
  slot_mel(ctx_, m, sl, n, s_);
}

void State::read_mel_window(int seek, float* out) {
  Impl& m = *m_;
  Impl::Slot& sl = m.slots[m.cur];
  DevMem tmp((size_t)m.n_mels * 3000 * 4);
  launch_mel_window(sl.mel.as<float>(), m.n_mels, sl.n_fft_frames, sl.gmax.as<int>(), seek, tmp.as<float>(), s_);
  WDR_HIP(wdr_memcpy_async(out, tmp.p, tmp.bytes, hipMemcpyDeviceToHost, s_));
  WDR_HIP(hipStreamSynchronize(s_));
}

// ------------------------------------------------------------------ encoder
static void proj(hipStream_t s, const f16* A, int lda, const f16* W, int ldw, const float* bias, void* out, int ldo, int M,
                 int N, int K, int epi, const float* pos = nullptr, int pos_rows = 0) {
  ProjArgs a{A, lda, W, ldw, bias, out, ldo, pos, pos_rows, M, N, K, epi};
  launch_proj(a, s);
}

// nb windows whose conv1 im2col rows are already in e.im2col ([nb*3000][kp1]); writes the
// cross K/V of window b to xkv_out + b * xkv_slot_elems.  Every GEMM runs with M = nb*1500
// (or nb*3000 for conv1) so one launch covers the batch.
static void encoder_body(Context& ctx, State::Impl& m, State::Impl::EncBufs& e, int nb, f16* xkv_out, hipStream_t s) {
  const Model& md = ctx.model;
  const HParams& hp = md.hp;
  const int d = hp.n_audio_state;
  const int M = nb * 1500;
  // conv1 (+GELU) -> c1 f16 [nb*3000][d]
  proj(s, e.im2col.as<f16>(), md.kp1, md.conv1_w, md.kp1, md.conv1_b, e.c1.p, d, 2 * M, d, md.kp1, EPI_F16_GELU);
  launch_im2col_conv2(e.c1.as<f16>(), d, nb, e.im2col.as<f16>(), s);
  // conv2 (+GELU) + positional -> ex f32 [nb*1500][d]
  proj(s, e.im2col.as<f16>(), 3 * d, md.conv2_w, 3 * d, md.conv2_b, e.ex.p, d, M, d, 3 * d, EPI_F32_GELU_POS,
       md.enc_pos, hp.n_audio_ctx);
  const float scale = 1.0f / 8.0f;   // d_head^-1/2
  const long long bs = 1500ll * 3 * d, obs = 1500ll * d;
  // fp8 encoder (BASELINE configs[4]): the four projections of every layer on the MX fp8 GEMM
  // (k_gemm8, twice the f16 MFMA rate); their A operands are written as e4m3 + E8M0 block scales
  // by their producers -- LN1 / LN2 (k_layernorm_f8), fc1's GELU epilogue (EPI_F8_GELU) -- or
  // quantised once behind the attention (k_quant_f8); the weights were quantised once
  // (Context::fp8_layers).  The residual stream, attention, the final LayerNorm and the cross-K/V
  // projection the decoder reads stay f16 / f32.
  // per layer and projection (Context::fp8_plan): an fp8 projection's A operand is written as
  // e4m3 + scales by its producer (LN1 / LN2 -> k_layernorm_f8; fc1's GELU -> EPI_F8_GELU when fc2
  // is fp8 too; the attention output, or an f16 GELU output, -> k_quant_f8), an f16 one as f16
  const bool f8 = ctx.fp8_encoder.load() && d % 128 == 0;
  const std::vector<Context::Fp8Layer>* F8 = f8 ? &ctx.fp8_layers() : nullptr;
  const int mp = cdiv(M, 256) * 256;
  uint8_t* qa = e.q8a.as<uint8_t>();
  uint8_t* qm = e.q8m.as<uint8_t>();
  uint32_t* sa = e.qsa.as<uint32_t>();
  uint32_t* sm = e.qsm.as<uint32_t>();
  auto gemm8 = [&](const uint8_t* A, const uint32_t* asc, int K, const Context::Fp8W& W, const float* bias, void* out,
                   int ldo, int N, int epi) {
    ProjArgs p{nullptr, K, nullptr, K, bias, out, ldo, nullptr, 0, M, N, K, epi};
    p.A8 = A;
    p.a_sc = asc;
    p.ld_asc = mp;
    p.B8 = W.w.as<uint8_t>();
    p.b_sc = W.s.as<uint32_t>();
    p.ld_bsc = N;
    if (epi == EPI_F8_GELU) {
      p.o_sc = sm;
      p.ld_osc = mp;
    }
    launch_proj_fp8(p, s);
  };
  for (int l = 0; l < hp.n_audio_layer; ++l) {
    const EncLayer& w = md.enc[l];
    const int pl = f8 ? ctx.fp8_plan[l] : 0;
    const Context::Fp8Layer* w8 = pl ? &(*F8)[l] : nullptr;
    if (pl & Context::F8_QKV) {
      launch_layernorm_f8(e.ex.as<float>(), d, w.ln1_g, w.ln1_b, qa, d, sa, mp, M, d, s);
      gemm8(qa, sa, d, w8->qkv, w.b_qkv, e.eqkv.p, 3 * d, 3 * d, EPI_F16);
    } else {
      launch_layernorm(e.ex.as<float>(), d, w.ln1_g, w.ln1_b, e.eh.as<f16>(), d, M, d, s);
      proj(s, e.eh.as<f16>(), d, w.w_qkv, d, w.b_qkv, e.eqkv.p, 3 * d, M, 3 * d, d, EPI_F16);
    }
    FlashArgs fa{e.eqkv.as<f16>(), 3 * d, bs, e.eqkv.as<f16>() + d, 3 * d, bs, e.eqkv.as<f16>() + 2 * d, 3 * d, bs,
                 e.eatt.as<f16>(), d, obs, nullptr, 1500, 1500, hp.n_audio_head, 0, scale};
    launch_flash_attn(fa, nb, s);
    if (pl & Context::F8_O) {
      launch_quant_f8(e.eatt.as<f16>(), d, M, d, qa, d, sa, mp, s);
      gemm8(qa, sa, d, w8->o, w.b_o, e.ex.p, d, d, EPI_F32_RESID);
    } else {
      proj(s, e.eatt.as<f16>(), d, w.w_o, d, w.b_o, e.ex.p, d, M, d, d, EPI_F32_RESID);
    }
    if (pl & Context::F8_FC1) {
      launch_layernorm_f8(e.ex.as<float>(), d, w.ln2_g, w.ln2_b, qa, d, sa, mp, M, d, s);
      if (pl & Context::F8_FC2)
        gemm8(qa, sa, d, w8->fc1, w.b_fc1, qm, 4 * d, 4 * d, EPI_F8_GELU);
      else
        gemm8(qa, sa, d, w8->fc1, w.b_fc1, e.emlp.p, 4 * d, 4 * d, EPI_F16_GELU);
    } else {
      launch_layernorm(e.ex.as<float>(), d, w.ln2_g, w.ln2_b, e.eh.as<f16>(), d, M, d, s);
      proj(s, e.eh.as<f16>(), d, w.w_fc1, d, w.b_fc1, e.emlp.p, 4 * d, M, 4 * d, d, EPI_F16_GELU);
      if (pl & Context::F8_FC2) launch_quant_f8(e.emlp.as<f16>(), 4 * d, M, 4 * d, qm, 4 * d, sm, mp, s);
    }
    if (pl & Context::F8_FC2)
      gemm8(qm, sm, 4 * d, w8->fc2, w.b_fc2, e.ex.p, d, d, EPI_F32_RESID);
    else
      proj(s, e.emlp.as<f16>(), 4 * d, w.w_fc2, 4 * d, w.b_fc2, e.ex.p, d, M, d, 4 * d, EPI_F32_RESID);
  }
  launch_layernorm(e.ex.as<float>(), d, md.ln_post_g, md.ln_post_b, e.eh.as<f16>(), d, M, d, s);
  // cross K/V for every decoder layer in one GEMM (N = L*2d), scattered by the epilogue into the
  // windows' head-major slots (common.h XKV_*; the batch's slots are contiguous)
  const int L = hp.n_text_layer;
  ProjArgs px{e.eh.as<f16>(), d, md.w_xkv, d, md.b_xkv, xkv_out, L * 2 * d, nullptr, 0, M, L * 2 * d, d, EPI_XKV};
  px.seq_stride = (long long)m.xkv_slot_elems;   // window b -> slot b
  launch_proj(px, s);
}

// one window of the current slot's segment on the decode stream (on-demand path)
// (on m.eo when set, else on the decode stream; the caller synchronises the stream it returns).
// The decode stream's earlier work (the scratch slot's log-mel) is awaited on the HOST, and only
// if any is pending: an event recorded on the decode stream would sit behind every step the
// batcher has queued on the hardware queue the two share (in order), and the encode would wait
// for them -- round 6's first on-demand pool did that and left the VAD line where it was.
hipStream_t State::encode_window(int seek) {
  Impl& m = *m_;
  Impl::Slot& sl = m.slots[m.cur];
  hipStream_t s = s_;
  if (m.eo) {
    const hipError_t q = hipStreamQuery(s_);
    if (q == hipErrorNotReady) WDR_HIP(hipStreamSynchronize(s_));
    else WDR_HIP(q);
    s = m.eo;
  }
  // a shared stream: the window's launches issued as one unit (as the encode-ahead batches)
  std::unique_lock<std::mutex> issue_lk;
  if (m.eo_shared) issue_lk = std::unique_lock<std::mutex>(stream_issue_mutex(m.eo));
  Im2colMelArgs ia{sl.mel.as<float>(), m.n_mels, sl.n_fft_frames, sl.gmax.as<int>(), seek, m.kp1, m.e1.im2col.as<f16>()};
  launch_im2col_mel(ia, s);
  encoder_body(ctx_, m, m.e1, 1, const_cast<f16*>(m.xkv()), s);
  return s;
}

void State::encode_from_mel_window(const float* w) {
  Impl& m = *m_;
  m.cur = m.S;
  std::vector<f16> col((size_t)3000 * m.kp1, (f16)0.f);
  for (int t = 0; t < 3000; ++t)
    for (int ci = 0; ci < m.n_mels; ++ci)
      for (int k = 0; k < 3; ++k) {
        const int u = t + k - 1;
        if (u >= 0 && u < 3000) col[(size_t)t * m.kp1 + ci * 3 + k] = (f16)w[(size_t)ci * 3000 + u];
      }
  WDR_HIP(wdr_memcpy_async(m.e1.im2col.p, col.data(), col.size() * 2, hipMemcpyHostToDevice, s_));
  encoder_body(ctx_, m, m.e1, 1, const_cast<f16*>(m.xkv()), s_);
  WDR_HIP(hipStreamSynchronize(s_));
}

// the current slot's cross K/V as [1500][L*2d] (key-major, K then V of every layer: the
// reference's per-layer cross-attention K / V projections side by side) from the head-major slot
void State::read_cross_kv(float* out) {
  Impl& m = *m_;
  const int L = ctx_.model.hp.n_text_layer, d = ctx_.model.hp.n_text_state, N = L * 2 * d;
  const size_t n = (size_t)XKV_T * N;
  std::vector<f16> h(n);
  WDR_HIP(wdr_memcpy_async(h.data(), m.xkv(), n * 2, hipMemcpyDeviceToHost, s_));
  WDR_HIP(hipStreamSynchronize(s_));
  for (int c = 0; c < N; ++c)
    for (int t = 0; t < XKV_T; ++t) out[(size_t)t * N + c] = (float)h[(size_t)(c >> 6) * XKV_HS + t * 64 + (c & 63)];
}

void State::read_encoder_out(float* out) {
  Impl& m = *m_;
  std::vector<f16> h((size_t)1500 * m.d);
  WDR_HIP(wdr_memcpy_async(h.data(), m.e1.eh.p, h.size() * 2, hipMemcpyDeviceToHost, s_));
  WDR_HIP(hipStreamSynchronize(s_));
  for (size_t i = 0; i < h.size(); ++i) out[i] = (float)h[i];
}

// ------------------------------------------------------------------ encode-ahead
// run_pipeline hands over the whole list of speech segments up front (the reference loops
// over them one whisper_full call at a time, src/transcribe.rs:372-389).  The first window of
// every segment does not depend on any decode result, so it is encoded ahead on the low-
// priority stream in batches of kBatch windows into the cross-K/V ring; segment j waits only
// on its slot's `ready` event, and slot j % S is reused once segment j - S has recorded `freed`.
// this state's encode-ahead work done: every batch ends by recording its slots' `ready` events
// (the stream itself may be shared with other states' encodes)
static void es_sync(State::Impl& m) {
  for (auto& sl : m.slots) WDR_HIP(hipEventSynchronize(sl.ready));
}

void State::plan(const int16_t* const* pcm, const int* n, int count, bool detect_lang) {
  Impl& m = *m_;
  enc_quiesce();
  es_sync(m);
  // every ring slot sized for the plan's longest segment here, on the chain thread: no device
  // or pinned allocation happens on the encode-ahead thread while other threads capture graphs
  int nmax = 0;
  for (int i = 0; i < count; ++i) nmax = std::max(nmax, n[i]);
  for (int k = 0; k < m.S; ++k) slot_reserve_all(m.slots[k], nmax, m.n_mels);
  {
    std::lock_guard<std::mutex> g(m.enc_mu);
    m.plan.detect_lang = detect_lang;
    m.plan.pcm.assign(pcm, pcm + count);
    m.plan.n.assign(n, n + count);
    m.plan.next_enq = 0;
    m.enc_err = nullptr;
    std::fill(m.lang_src.begin(), m.lang_src.end(), -1);
  }
  top_up(0);
}

void State::unplan() {
  Impl& m = *m_;
  enc_quiesce();
  flush_dtw();
  es_sync(m);
  std::lock_guard<std::mutex> g(m.enc_mu);
  m.plan.pcm.clear();
  m.plan.n.clear();
  m.plan.next_enq = 0;
  times.windows += m.enc_windows.exchange(0);
  times.lang_passes += m.lang_passes.exchange(0);
  times.lang_rows += m.lang_rows.exchange(0);
}

// Segments the encode-ahead stream may run ahead of the decoder (WDR_ENC_AHEAD, kBatch..S;
// default 6: a chain's next batch is issued once it is 2 segments into the current one).  With
// 16 chains planned at once, a 16-segment lookahead queues 256 windows up front and each chain's
// FIRST batch waits behind other chains' later ones: 8 let every chain start decoding sooner
// (1-h bench: 461 vs 446 xRT, mean of 3 / 2 runs; 4: 457).  At 40 chains 8 still queued 320 of a
// run's 674 windows in its first second, slowing the batched launches beside them; 6 together
// with no detection pass on the encode stream (lang_first) measured 835.1 vs 810.9 xRT, 4 of 4
// pairs ahead (profiles/r05/ab_ahead6_langfirst0.txt).
static int enc_ahead(int S) {
  static const int a = [] {
    const char* e = getenv("WDR_ENC_AHEAD");
    return e ? atoi(e) : 6;
  }();
  return std::max(kBatch, std::min(a > 0 ? a : S, S));
}

// stream `s` waits until the queued DTW pass reading slot `k` has read it (the pass is started
// at once if it is still queued)
void State::slot_dtw_fence(int k, hipStream_t s) {
  Impl& m = *m_;
  std::shared_ptr<DtwQJob>& q = m.slots[k].dtw;
  if (!q) return;
  const double t = now_s();
  ctx_.dtw_queue().wait_issued(q);
  m.t_fence += (long long)((now_s() - t) * 1e9);
  stream_fence(s, q->fwd, s == s_ && host_fence());
  q.reset();
}

// WDR_ODM_ALT (default 1; read once): see Impl::xsel
static bool odm_alt() {
  static const bool v = !(getenv("WDR_ODM_ALT") && atoi(getenv("WDR_ODM_ALT")) == 0);
  return v;
}

// the host waits until the queued DTW pass reading the spare cross-K/V has read it
void State::alt_dtw_fence() {
  Impl& m = *m_;
  std::shared_ptr<DtwQJob>& q = m.alt_dtw;
  if (!q) return;
  const double t = now_s();
  ctx_.dtw_queue().wait_issued(q);
  m.t_fence += (long long)((now_s() - t) * 1e9);
  WDR_HIP(hipEventSynchronize(q->fwd));
  q.reset();
}

// stream `s` waits for every queued pass that may still write this chain's DTW KV sequence
void State::dtw_queue_fence(hipStream_t s) {
  Impl& m = *m_;
  for (auto& q : m.qlive) {
    ctx_.dtw_queue().wait_issued(q);
    WDR_HIP(hipStreamWaitEvent(s, q->fwd, 0));
  }
  m.qlive.clear();
}

static bool enc_thread_on() {
  static const bool on = !(getenv("WDR_ENC_THREAD") && atoi(getenv("WDR_ENC_THREAD")) == 0);
  return on;
}

// the encode-ahead host thread of this state
void State::enc_loop() {
  Impl& m = *m_;
  std::unique_lock<std::mutex> lk(m.enc_mu);
  try {
    WDR_HIP(hipSetDevice(ctx_.cp.gpu_device));
  } catch (...) {
    m.enc_err = std::current_exception();
  }
  while (!m.enc_stop) {
    if (m.enc_err || m.enc_target < 0) {
      m.enc_cv.wait(lk);
      continue;
    }
    const int j = m.enc_target;
    m.enc_busy = true;
    lk.unlock();
    bool issued = false;
    std::exception_ptr e;
    try {
      issued = top_up_batch(j);
    } catch (...) {
      e = std::current_exception();
    }
    lk.lock();
    m.enc_busy = false;
    if (e) m.enc_err = e;
    m.enc_cv.notify_all();
    if (!issued && !e && m.enc_target == j) m.enc_cv.wait(lk);   // nothing allowed until the target moves
  }
}

// the encode-ahead thread idle (no batch being issued), its target cleared
void State::enc_quiesce() {
  Impl& m = *m_;
  if (!m.enc_th.joinable()) return;
  std::unique_lock<std::mutex> lk(m.enc_mu);
  m.enc_target = -1;
  m.enc_cv.notify_all();
  m.enc_cv.wait(lk, [&] { return !m.enc_busy; });
}

// segment j's encode (and every batch the lookahead allows) issued; on the encode-ahead thread
// when it runs (the chain waits only if j's own batch is not issued yet)
void State::top_up(int j) {
  Impl& m = *m_;
  if (!enc_thread_on()) {
    while (top_up_batch(j)) {
    }
    return;
  }
  if (!m.enc_th.joinable()) m.enc_th = std::thread([this] {
    pthread_setname_np(pthread_self(), "wdr-encode");
    enc_loop();
  });
  std::unique_lock<std::mutex> lk(m.enc_mu);
  m.enc_target = std::max(m.enc_target, j);
  m.enc_cv.notify_all();
  m.enc_cv.wait(lk, [&] { return m.enc_err || (int)m.plan.next_enq > j || m.plan.pcm.empty(); });
  if (m.enc_err) std::rethrow_exception(m.enc_err);
}

// WDR_LANG_PIGGYBACK (default 1; read once): in a multi-chain run, a plan's later segments get
// their language from a detection row (SOT, the segment's cross-K/V) riding in one of the chain's
// batched steps during the segment before (StepBatcher::Req::ln) instead of a 32-layer pass of
// their own on the encode-ahead stream per 4-window batch; the same arithmetic, so the same
// language logits
static bool lang_piggyback() {
  static const bool on = !(getenv("WDR_LANG_PIGGYBACK") && atoi(getenv("WDR_LANG_PIGGYBACK")) == 0);
  return on;
}

// WDR_LANG_FIRST (default 0; read once; with lang_piggyback): 1 = a plan's first encode batch
// carries the detection pass; 0 = its segment 0 detects in a one-row batched step of its own
// (full()) and segments 1..3 ride in the steps of the segments before, like every later one
// (alone: profiles/r05/ab_lang_first.txt, 855.4 vs 848.2 xRT, inside the +-1.5 % bar; with the
// 6-segment encode-ahead, enc_ahead: 835.1 vs 810.9, ab_ahead6_langfirst0.txt)
static bool lang_first() {
  static const bool on = getenv("WDR_LANG_FIRST") && atoi(getenv("WDR_LANG_FIRST")) != 0;
  return on;
}

// issue the plan's next encode-ahead batch if the lookahead of segment j allows it: every group
// of segments whose slots' previous occupants (j - S ...) have finished
bool State::top_up_batch(int j) {
  Impl& m = *m_;
  const int N = (int)m.plan.pcm.size();
  // WDR_ENC_FIRST: windows in the first batch of a plan (A/B: 1 / 2 / 4 measured 491-493 /
  // 495 / 496 xRT on the 1-h bench, so a full batch stays the default); a batch never wraps
  // around the ring (its slots stay contiguous for the cross-K/V GEMM).  Encoder results do not
  // depend on the batch.
  // With the encode-ahead thread, a plan's second batch is issued only once its first has been
  // encoded: at the start of a run every chain waits for its first batch, and with all chains'
  // look-ahead batches queued at once the first batches finished late (1-h bench, chain log:
  // 0.58 -> 0.46 s per chain).  A first batch of 1 or 2 windows (WDR_ENC_FIRST) measured slower
  // (570 / 580 vs 624 xRT: partial, ungraphed batches and a misaligned ring).
  static const int first = [] {
    const char* e = getenv("WDR_ENC_FIRST");
    const int v = e ? atoi(e) : kBatch;
    return std::max(1, std::min(kBatch, v));
  }();
  {
    if ((int)m.plan.next_enq >= N) return false;
    const int g0 = (int)m.plan.next_enq;
    int g1 = std::min(N, g0 + (g0 == 0 ? first : kBatch));
    g1 = std::min(g1, (g0 / m.S + 1) * m.S);
    if (g1 - 1 > j + enc_ahead(m.S) - 1) return false;
    if (g0 == first && g0 > 0 && enc_thread_on() && std::this_thread::get_id() == m.enc_th.get_id())
      WDR_HIP(hipEventSynchronize(m.slots[(g0 - 1) % m.S].ready));   // the first window encoded
    const int slot0 = g0 % m.S;
    // a shared (pooled) encode stream: the whole batch issued as one unit (WDR_ENC_ATOMIC=0: A/B)
    static const bool atomic_issue = !(getenv("WDR_ENC_ATOMIC") && atoi(getenv("WDR_ENC_ATOMIC")) == 0);
    std::unique_lock<std::mutex> issue_lk;
    if (m.es_shared && atomic_issue) issue_lk = std::unique_lock<std::mutex>(stream_issue_mutex(m.es));
    for (int k = g0; k < g1; ++k) {
      Impl::Slot& sl = m.slots[k % m.S];
      if (k >= m.S) WDR_HIP(hipStreamWaitEvent(m.es, sl.freed, 0));
      slot_dtw_fence(k % m.S, m.es);   // a queued DTW pass may still read the slot
      const int nk = m.plan.n[k];
      slot_reserve_all(sl, nk, m.n_mels);   // normally sized by plan() already
      if (nk > sl.pcm_cap) {
        // (a fallback: plan() sizes the slots) pinned host memory under the allocation mutex, as
        // every allocation while other threads may be capturing graphs
        std::lock_guard<std::recursive_mutex> g(hip_alloc_mutex());
        if (sl.h_pcm) WDR_HIP(hipHostFree(sl.h_pcm));
        WDR_HIP(hipHostMalloc((void**)&sl.h_pcm, (size_t)std::max(nk, 1) * 2, hipHostMallocDefault));
        sl.pcm = DevMem((size_t)std::max(nk, 1) * 2);
        sl.pcm_cap = nk;
      }
      slot_reserve_x(sl, nk);
      if (nk > 0) {
        // the staging buffer's previous H2D copy (segment k - S) completed before its decode
        memcpy(sl.h_pcm, m.plan.pcm[k], (size_t)nk * 2);
        WDR_HIP(wdr_memcpy_async(sl.pcm.p, sl.h_pcm, (size_t)nk * 2, hipMemcpyHostToDevice, m.es));
        launch_i16_to_f32(sl.pcm.as<int16_t>(), nk, sl.x.as<float>(), m.es);
        if (nk > sl.energy_cap) {
          std::lock_guard<std::recursive_mutex> g(hip_alloc_mutex());
          if (sl.h_energy) WDR_HIP(hipHostFree(sl.h_energy));
          WDR_HIP(hipHostMalloc((void**)&sl.h_energy, (size_t)nk * 4, hipHostMallocDefault));
          sl.energy_d = DevMem((size_t)nk * 4);
          sl.energy_cap = nk;
        }
        launch_energy(sl.x.as<float>(), nk, sl.energy_d.as<float>(), m.es);
        WDR_HIP(wdr_memcpy_async(sl.h_energy, sl.energy_d.p, (size_t)nk * 4, hipMemcpyDeviceToHost, m.es));
      }
      sl.energy_n = nk;
      slot_mel(ctx_, m, sl, nk, m.es);
      Im2colMelArgs ia{sl.mel.as<float>(), m.n_mels, sl.n_fft_frames, sl.gmax.as<int>(), 0, m.kp1,
                       m.eb.im2col.as<f16>() + (size_t)(k - g0) * 3000 * m.kp1};
      launch_im2col_mel(ia, m.es);
    }
    // the batch's encoder + cross-K/V (+ language detection): whisper.cpp's language detection
    // (one SOT pass over window 0, argmax of the language logits) depends on nothing decoded, so
    // it runs here, off the decode chain: the batch's windows as the rows of ONE decode step,
    // each with its own cross-K/V slot and sequence (every window a one-row group: the
    // arithmetic of decoder_prefill(SOT) on the decode stream)
    // a multi-chain run detects the language in its batched steps (lang_piggyback): no pass here,
    // or only for a plan's first batch with WDR_LANG_FIRST=1; a one-chain run keeps it per batch
    const bool ride = batched && lang_piggyback();
    const bool lang_here = m.plan.detect_lang && (!ride || (g0 == 0 && lang_first()));
    if (m.plan.detect_lang)
      for (int k = g0; k < g1; ++k) m.lang_src[k % m.S] = lang_here ? k : -1;
    auto body = [&](RowBatch& tl, bool capturing, hipStream_t es) {
      encoder_body(ctx_, m, m.eb, g1 - g0, m.xkv_ring.as<f16>() + (size_t)slot0 * m.xkv_slot_elems, es);
      if (!lang_here) return;
      const int R = g1 - g0;
      tl.clear();   // waits for the previous batch's table copy
      const int sot = ctx_.vocab.sot;
      for (int r = 0; r < R; ++r) {
        RowGroupDesc g;
        g.n = 1;
        g.tok = &sot;
        g.seq0 = chain * NSLOT + LANG_SEQ + r;
        g.xkv = m.xkv_ring.as<f16>() + (size_t)((g0 + r) % m.S) * m.xkv_slot_elems;
        g.logits = 1;
        tl.add(g);
      }
      RowsIO io = m.lb.io(ctx_, m.V);
      tl.upload(io, es, true, !capturing);
      rows_forward(ctx_, io, R, es);
      for (int r = 0; r < R; ++r)
        WDR_HIP(wdr_memcpy_async(m.h_lang + (size_t)((g0 + r) % m.S) * 100,
                               m.lb.logits.as<float>() + (size_t)r * m.V + sot + 1, 100 * 4,
                               hipMemcpyDeviceToHost, es));
    };
    const double t_el = now_s();
    struct ElT {
      double t0;
      std::atomic<long long>& acc;
      ~ElT() { acc += (long long)((now_s() - t0) * 1e9); }
    } el_t{t_el, m.t_enc_launch};
    static const bool enc_graph = !(getenv("WDR_ENC_GRAPH") && atoi(getenv("WDR_ENC_GRAPH")) == 0);
    // the live profiler (bench.py's roofline) samples eager launches only: while it is on, 1 in
    // kEncEvery graphable batches runs eagerly with its launches sampled at the matching rate
    // (prof.h); partial batches, always eager, are sampled at the base rate -- a uniform sample
    // of the encoder GEMMs
    const bool graphable = enc_graph && g1 - g0 == kBatch && !no_graph();
    const bool sampled = graphable && prof_enc_batch();
    if (graphable && !sampled) {
      const bool f8 = ctx_.fp8_encoder.load();
      const int key = slot0 * 4 + (f8 ? 2 : 0) + (lang_here ? 1 : 0);   // the batch's slots
      Impl::EncGraph& eg = m.enc_graphs[key];
      if (!eg.exec) {
        if (f8) {   // lazily built weights: not inside the capture
          (void)ctx_.fp8_layers();
        }
        if (!eg.tl) eg.tl = std::make_unique<RowBatch>(kBatch, kBatch, 0);
        std::lock_guard<std::recursive_mutex> cap_lock(hip_alloc_mutex());   // no allocation meanwhile
        // captured on a stream of its own: the chain thread waits on events recorded on m.es,
        // which HIP refuses while m.es itself is capturing
        if (!m.es_cap) WDR_HIP(hipStreamCreateWithFlags(&m.es_cap, hipStreamNonBlocking));
        stream_note("state-es_cap", m.es_cap);
        hipGraph_t graph;
        prof_capture(true);
        WDR_HIP(hipStreamBeginCapture(m.es_cap, hipStreamCaptureModeRelaxed));
        try {
          body(*eg.tl, true, m.es_cap);
        } catch (...) {
          hipGraph_t dead = nullptr;
          (void)hipStreamEndCapture(m.es_cap, &dead);
          if (dead) (void)hipGraphDestroy(dead);
          prof_capture(false);
          throw;
        }
        prof_capture(false);
        WDR_HIP(hipStreamEndCapture(m.es_cap, &graph));
        WDR_HIP(hipGraphInstantiate(&eg.exec, graph, nullptr, nullptr, 0));
        WDR_HIP(hipGraphDestroy(graph));
      }
      std::mutex* mu = launch_lock();   // WDR_LAUNCH_LOCK (prof.h)
      if (mu) mu->lock();
      const hipError_t ge = hipGraphLaunch(eg.exec, m.es);
      if (mu) mu->unlock();
      WDR_HIP(ge);
    } else {
      prof_in_enc(sampled);
      try {
        body(*m.tlb, false, m.es);
      } catch (...) {
        prof_in_enc(false);
        throw;
      }
      prof_in_enc(false);
    }
    for (int k = g0; k < g1; ++k) WDR_HIP(hipEventRecord(m.slots[k % m.S].ready, m.es));
    {
      std::lock_guard<std::mutex> g(m.enc_mu);   // the chain reads next_enq under this lock
      m.plan.next_enq = g1;
    }
    m.enc_windows += g1 - g0;
    if (lang_here) {
      m.lang_passes++;
      m.lang_rows += g1 - g0;
    }
  }
  return true;
}

// ------------------------------------------------------------------ decoder
// Every decoder pass of a State is a rows forward (rows.h) -- the arithmetic every other pass
// of the context uses too, so a prompt prefill, a DTW re-forward or a step gives the same result
// here as inside the multi-chain batched step.

// the first layer a capture-only pass (the DTW re-forward) can skip: nothing after the last
// alignment-head layer's cross-attention changes a captured probability
// WDR_DTW_QUEUE=0: multi-chain DTW re-forwards ride in the step batcher's requests (the round-3
// schedule) instead of the DtwQueue
static bool dtw_queue_on() {
  static const bool on = [] {
    const char* e = getenv("WDR_DTW_QUEUE");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

static int capture_l_end(const Context& ctx) {
  const int L = ctx.model.hp.n_text_layer;
  if (ctx.aheads_per_layer.size() != (size_t)L) return L;
  int l = L;
  while (l > 0 && ctx.aheads_per_layer[l - 1].empty()) --l;
  return l == 0 ? L : l;
}

// Prefill of `n` tokens into sequence `seq` (chain-local) from an empty cache (positions
// 0..n-1): whisper.cpp clears the KV cache before the prompt decode and before the DTW pass.
void State::decoder_prefill(const int* toks, int n, int seq, bool want_logits, bool capture) {
  prefill_on(toks, n, seq, want_logits, capture, false, s_, m_->xkv());
}

void State::prefill_on(const int* toks, int n, int seq, bool want_logits, bool capture, bool dtw_set,
                       hipStream_t st, const f16* xkv_base) {
  Impl& m = *m_;
  WDR_CHECK(n >= 1 && n <= RMAX, "decoder prefill: token count out of range");
  RowBatch& tb = dtw_set ? *m.tdb : *m.tb;
  const RowsBufs& B = dtw_set ? m.db : m.mb;
  tb.clear();
  RowGroupDesc g;
  g.n = n;
  g.tok = toks;
  g.seq0 = chain * NSLOT + seq;
  g.xkv = xkv_base;
  g.logits = want_logits ? 1 : 0;
  if (capture) {
    g.cap = dtw_set ? m.dset.cap.as<float>() : m.cap.as<float>();
    if (!want_logits) g.l_end = capture_l_end(ctx_);
  }
  tb.add(g);
  RowsIO io = B.io(ctx_, m.V);
  tb.upload(io, st, true, true);
  if (capture && !want_logits && ctx_.aheads_per_layer.size() == (size_t)ctx_.model.hp.n_text_layer) {
    // a DTW re-forward: the DtwQueue's pass (stops after the last alignment-head layer)
    dtw_rows_forward(ctx_, io, n, capture_l_end(ctx_), st);
  } else {
    rows_forward(ctx_, io, n, st);
  }
  if (st == s_) times.prefills++;
}

// R decoder rows of this state (beams / best_of decoders, chain-local sequences seqs[r]) reading
// the current slot: one group sharing the slot, logits of every row into mb.logits
void State::decoder_step(const int* toks, const int* seqs, const int* pos, int R) {
  Impl& m = *m_;
  WDR_CHECK(R >= 1 && R <= NSEQ, "decoder step: row count out of range");
  RowBatch& tb = *m.tb;
  tb.clear();
  int sq[NSEQ];
  for (int i = 0; i < R; ++i) sq[i] = chain * NSLOT + seqs[i];
  RowGroupDesc g;
  g.n = R;
  g.tok = toks;
  g.seq = sq;
  g.pos = pos;
  g.xkv = m.xkv();
  g.logits = 2;
  tb.add(g);
  RowsIO io = m.mb.io(ctx_, m.V);
  tb.upload(io, s_, true, true);
  rows_forward(ctx_, io, R, s_);
  times.decode_steps++;
}

// decode step + logit rules + greedy pick as ONE hipGraph replay per token (captured once per
// (K, rows); the row tables and per-step inputs live in pinned host buffers the graph's copy
// nodes read).
void State::step_and_sample(const int* toks, const int* seqs, const int* pos, const LogitsCtl* ctl, int R,
                            TokenData* out, int K, BeamCand* cands) {
  Impl& m = *m_;
  WDR_CHECK(R >= 1 && R <= NSEQ, "decoder step: row count out of range");
  const bool sampled = !no_graph() && prof_step();
  if (sampled || no_graph()) {
    // live per-kernel HIP-event timing cannot read events recorded inside a graph on this
    // ROCm: a sampled step runs the same kernels eagerly (prof.h)
    prof_in_step(sampled);
    try {
      decoder_step(toks, seqs, pos, R);
    } catch (...) {
      prof_in_step(false);
      throw;
    }
    prof_in_step(false);
    run_logits(R, ctl, out, nullptr);
    if (K > 0) logits_topk(R, K, cands);
    return;
  }
  RowBatch& tb = *m.tb;
  tb.clear();
  int sq[NSEQ];
  for (int i = 0; i < R; ++i) sq[i] = chain * NSLOT + seqs[i];
  RowGroupDesc grp;
  grp.n = R;
  grp.tok = toks;
  grp.seq = sq;
  grp.pos = pos;
  grp.xkv = m.xkv();
  grp.logits = 2;
  tb.add(grp);
  memcpy(m.h_ctl, ctl, R * sizeof(LogitsCtl));
  RowsIO io = m.mb.io(ctx_, m.V);
  Impl::StepGraph& g = m.graphs[(K << 16) + R];
  if (g.exec && memcmp(&g.vids, &m.vids, sizeof(VocabIds)) != 0) {   // rule constants changed: recapture
    (void)hipGraphExecDestroy(g.exec);
    g.exec = nullptr;
  }
  if (!g.exec) {
    std::lock_guard<std::recursive_mutex> cap_lock(hip_alloc_mutex());   // no allocation meanwhile
    hipGraph_t graph;
    prof_capture(true);
    WDR_HIP(hipStreamBeginCapture(s_, hipStreamCaptureModeRelaxed));
    tb.upload(io, s_, true, false);
    WDR_HIP(wdr_memcpy_async(m.ctl.p, m.h_ctl, R * sizeof(LogitsCtl), hipMemcpyHostToDevice, s_));
    rows_forward(ctx_, io, R, s_);
    launch_logits_process(m.mb.logits.as<float>(), m.V, m.ctl.as<LogitsCtl>(), m.vids, R, m.work.as<float>(),
                          m.tokout.as<TokOut>(), s_);
    WDR_HIP(wdr_memcpy_async(m.h_tok, m.tokout.p, R * sizeof(TokOut), hipMemcpyDeviceToHost, s_));
    if (K > 0) {
      launch_logits_topk(m.mb.logits.as<float>(), m.V, m.ctl.as<LogitsCtl>(), m.vids, R, K, m.work.as<float>(),
                         m.beamc.as<BeamCand>(), s_);
      WDR_HIP(wdr_memcpy_async(m.h_beam, m.beamc.p, (size_t)R * K * sizeof(BeamCand), hipMemcpyDeviceToHost, s_));
    }
    prof_capture(false);
    WDR_HIP(hipStreamEndCapture(s_, &graph));
    WDR_HIP(hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0));
    WDR_HIP(hipGraphDestroy(graph));
    g.vids = m.vids;
  } else {
    tb.upload(io, s_, false, false);   // the captured copy node reads the staging
  }
  {
    std::mutex* mu = launch_lock();   // WDR_LAUNCH_LOCK (prof.h)
    if (mu) mu->lock();
    const hipError_t ge = hipGraphLaunch(g.exec, s_);
    if (mu) mu->unlock();
    WDR_HIP(ge);
  }
  WDR_HIP(hipStreamSynchronize(s_));
  if (K > 0) memcpy(cands, m.h_beam, (size_t)R * K * sizeof(BeamCand));
  for (int r = 0; r < R; ++r) {
    const TokOut& o = m.h_tok[r];
    TokenData t;
    t.id = o.id;
    t.tid = o.tid;
    t.p = o.p;
    t.plog = o.plog;
    t.pt = o.pt;
    t.ptsum = o.ptsum;
    out[r] = t;
  }
  times.decode_steps++;
}

void State::run_logits(int R, const LogitsCtl* ctl, TokenData* out, float* nosp) {
  Impl& m = *m_;
  memcpy(m.h_ctl, ctl, R * sizeof(LogitsCtl));
  WDR_HIP(wdr_memcpy_async(m.ctl.p, m.h_ctl, R * sizeof(LogitsCtl), hipMemcpyHostToDevice, s_));
  launch_logits_process(m.mb.logits.as<float>(), m.V, m.ctl.as<LogitsCtl>(), m.vids, R, m.work.as<float>(),
                        m.tokout.as<TokOut>(), s_);
  WDR_HIP(wdr_memcpy_async(m.h_tok, m.tokout.p, R * sizeof(TokOut), hipMemcpyDeviceToHost, s_));
  WDR_HIP(hipStreamSynchronize(s_));
  for (int r = 0; r < R; ++r) {
    const TokOut& o = m.h_tok[r];
    TokenData t;
    t.id = o.id;
    t.tid = o.tid;
    t.p = o.p;
    t.plog = o.plog;
    t.pt = o.pt;
    t.ptsum = o.ptsum;
    out[r] = t;
    if (nosp) nosp[r] = o.nosp_prob;
  }
}

// top-K candidates of rows whose logits were just processed by run_logits (same ctl)
void State::logits_topk(int R, int K, BeamCand* out) {
  Impl& m = *m_;
  launch_logits_topk(m.mb.logits.as<float>(), m.V, m.ctl.as<LogitsCtl>(), m.vids, R, K, m.work.as<float>(),
                     m.beamc.as<BeamCand>(), s_);
  WDR_HIP(wdr_memcpy_async(m.h_beam, m.beamc.p, (size_t)R * K * sizeof(BeamCand), hipMemcpyDeviceToHost, s_));
  WDR_HIP(hipStreamSynchronize(s_));
  memcpy(out, m.h_beam, (size_t)R * K * sizeof(BeamCand));
}

// beam reorder (whisper_kv_cache_seq_cp through scratch sequences): sequence dst takes the first
// n_rows cached rows of sequence src, for every (src, dst) move; scratch slots NSEQ + dst.
void State::kv_reorder(const std::vector<std::pair<int, int>>& moves, int n_rows) {
  Impl& m = *m_;
  if (moves.empty() || n_rows <= 0) return;
  const int n = (int)moves.size();
  WDR_CHECK(n <= NSEQ, "kv reorder: too many moves");
  for (int i = 0; i < n; ++i) {
    WDR_CHECK(moves[i].first < NSEQ && moves[i].second < NSEQ, "kv reorder: slot out of range");
    m.h_pairs[2 * i] = moves[i].first;
    m.h_pairs[2 * i + 1] = NSEQ + moves[i].second;
    m.h_pairs[2 * NSEQ + 2 * i] = NSEQ + moves[i].second;
    m.h_pairs[2 * NSEQ + 2 * i + 1] = moves[i].second;
  }
  WDR_HIP(wdr_memcpy_async(m.kvpairs.p, m.h_pairs, 4 * NSEQ * 4, hipMemcpyHostToDevice, s_));
  launch_kv_copy(m.kc, m.vc, m.seq_stride, m.nslot_tot, m.L, m.kvpairs.as<int>(), n, n_rows, m.d, s_);
  launch_kv_copy(m.kc, m.vc, m.seq_stride, m.nslot_tot, m.L, m.kvpairs.as<int>() + 2 * NSEQ, n, n_rows,
                 m.d, s_);
  WDR_HIP(hipStreamSynchronize(s_));   // the pinned pair table is rewritten by the next reorder
}

// test seam: prefill toks[0..n-2] into sequence 0, then ONE decode step of toks[n-1] at
// position n-1 (the step's logits; the rows contract makes them equal the n-token prefill's)
void State::dbg_step(const int* toks, int n, float* logits_out) {
  Impl& m = *m_;
  WDR_CHECK(n >= 2 && n <= 448, "dbg_step: need 2..448 tokens");
  decoder_prefill(toks, n - 1, 0, false, false);
  const int tok = toks[n - 1], seq = 0, pos = n - 1;
  decoder_step(&tok, &seq, &pos, 1);
  WDR_HIP(wdr_memcpy_async(logits_out, m.mb.logits.p, (size_t)m.V * 4, hipMemcpyDeviceToHost, s_));
  WDR_HIP(hipStreamSynchronize(s_));
}

// a one-row (greedy) batcher request
static StepBatcher::Req row_req(int tok, int seq, int pos, const f16* xkv, const LogitsCtl& c, const VocabIds& v) {
  StepBatcher::Req q;
  q.n = 1;
  q.tok[0] = tok;
  q.seq[0] = seq;
  q.pos[0] = pos;
  q.ctl[0] = c;
  q.xkv = xkv;
  q.vids = v;
  return q;
}

double State::dbg_batch_step(const int* toks, int n, int R, int iters) {
  Impl& m = *m_;
  WDR_CHECK(n >= 2 && n <= 448 && R >= 1 && R <= 16 && iters >= 1, "dbg_batch_step: bad shape");
  decoder_prefill(toks, n - 1, 0, false, false);
  WDR_HIP(hipStreamSynchronize(s_));
  StepBatcher& b = ctx_.step_batcher(chain);
  std::vector<StepBatcher::Req> rq(R);
  std::vector<StepBatcher::Req*> batch(R);
  for (int r = 0; r < R; ++r) {
    LogitsCtl c{};
    c.n_tokens = 1;
    c.pen_ts = 1;
    c.force_kind = 2;
    // every row reads this window's cross-K/V; rows 1.. attend over an uninitialised cache
    rq[r] = row_req(toks[n - 1], chain * NSLOT + r, n - 1, m.xkv(), c, m.vids);
    batch[r] = &rq[r];
  }
  b.run(batch);
  const double t = now_s();
  for (int i = 0; i < iters; ++i) b.run(batch);
  return (now_s() - t) * 1e3 / iters;
}

void State::reset_rng() { m_->rng[0] = std::mt19937(0); }
std::string State::rng_state() const {
  std::ostringstream o;
  o << m_->rng[0];
  return o.str();
}
void State::set_rng_state(const std::string& st) {
  std::istringstream i(st);
  i >> m_->rng[0];
}

void State::decode_logits(const int* toks, int n, float* logits_out) {
  decoder_prefill(toks, n, 0, true, false);
  WDR_HIP(wdr_memcpy_async(logits_out, m_->mb.logits.p, (size_t)m_->V * 4, hipMemcpyDeviceToHost, s_));
  WDR_HIP(hipStreamSynchronize(s_));
}

void State::dbg_logits(const float* logits, int R, const LogitsCtl* ctl, float max_initial_ts, bool suppress_blank,
                       TokenData* out, float* nosp) {
  Impl& m = *m_;
  WDR_CHECK(R >= 1 && R <= NSEQ, "dbg_logits: 1..8 rows");
  const float precision = 30.0f / ctx_.model.hp.n_audio_ctx;
  m.vids.max_initial_tid = max_initial_ts > 0.0f ? (int)std::round(max_initial_ts / precision) : -1;
  m.vids.suppress_blank = suppress_blank ? 1 : 0;
  WDR_HIP(wdr_memcpy_async(m.mb.logits.p, logits, (size_t)R * m.V * 4, hipMemcpyHostToDevice, s_));
  run_logits(R, ctl, out, nosp);
}

void State::dtw_capture(const int* toks, int n, float* cap_out) {
  decoder_prefill(toks, n, 0, false, true);
  const size_t A = ctx_.aheads.size();
  WDR_HIP(wdr_memcpy_async(cap_out, m_->cap.p, A * n * 1500 * 4, hipMemcpyDeviceToHost, s_));
  WDR_HIP(hipStreamSynchronize(s_));
}

// ------------------------------------------------------------------ timestamps
static float voice_length(const std::string& text) {
  float res = 0.f;
  for (char c : text) {
    if (c == ' ') res += 0.01f;
    else if (c == ',') res += 2.00f;
    else if (c == '.' || c == '!' || c == '?') res += 3.00f;
    else if (c >= '0' && c <= '9') res += 3.00f;
    else res += 1.00f;
  }
  return res;
}

void State::heuristic_timestamps(int i_segment, const FullParams& p) {
  const Vocab& v = ctx_.vocab;
  ResultSeg& seg = result_all[i_segment];
  auto& tk = seg.tokens;
  const int n_samples = (int)energy.size();
  if (n_samples == 0) return;
  const long long t0 = seg.t0, t1 = seg.t1;
  const int n = (int)tk.size();
  if (n == 0) return;
  if (n == 1) {
    tk[0].t0 = t0;
    tk[0].t1 = t1;
    return;
  }
  for (int j = 0; j < n; ++j) {
    TokenData& t = tk[j];
    if (j == 0) {
      if (t.id == v.beg) {
        tk[0].t0 = t0;
        tk[0].t1 = t0;
        tk[1].t0 = t0;
        t_beg = t0;
        t_last = t0;
        tid_last = v.beg;
      } else {
        tk[0].t0 = t_last;
      }
    }
    const long long tt = t_beg + 2 * (long long)(t.tid - v.beg);
    t.vlen = voice_length(v.id_to_token[t.id]);
    if (t.pt > p.thold_pt && t.ptsum > p.thold_ptsum && t.tid > tid_last && tt <= t1) {
      if (j > 0) tk[j - 1].t1 = tt;
      t.t0 = tt;
      tid_last = t.tid;
    }
  }
  tk[n - 2].t1 = t1;
  tk[n - 1].t0 = t1;
  tk[n - 1].t1 = t1;
  t_last = t1;
  {
    int p0 = 0, p1 = 0;
    while (true) {
      while (p1 < n && tk[p1].t1 < 0) p1++;
      if (p1 >= n) p1--;
      if (p1 > p0) {
        double psum = 0.0;
        for (int j = p0; j <= p1; j++) psum += tk[j].vlen;
        const double dt = (double)(tk[p1].t1 - tk[p0].t0);
        for (int j = p0 + 1; j <= p1; j++) {
          const double ct = tk[j - 1].t0 + dt * tk[j - 1].vlen / psum;
          tk[j - 1].t1 = (long long)ct;
          tk[j].t0 = (long long)ct;
        }
      }
      p1++;
      p0 = p1;
      if (p1 >= n) break;
    }
  }
  for (int j = 0; j < n - 1; j++) {
    if (tk[j].t1 < 0) tk[j + 1].t0 = tk[j].t1;
    if (j > 0 && tk[j - 1].t1 > tk[j].t0) {
      tk[j].t0 = tk[j - 1].t1;
      tk[j].t1 = std::max(tk[j].t0, tk[j].t1);
    }
  }
  const int hw = 16000 / 8;
  auto ts2s = [&](long long t) { return (int)std::max(0LL, std::min((long long)n_samples - 1, (t * 16000) / 100)); };
  auto s2ts = [&](int i) { return (100LL * i) / 16000; };
  for (int j = 0; j < n; j++) {
    if (tk[j].id >= v.eot) continue;
    int s0 = ts2s(tk[j].t0);
    int s1 = ts2s(tk[j].t1);
    const int ss0 = std::max(s0 - hw, 0);
    const int ss1 = std::min(s1 + hw, n_samples);
    const int ns = ss1 - ss0;
    float sum = 0.0f;
    for (int k = ss0; k < ss1; k++) sum += energy[k];
    const float thold = 0.5 * sum / ns;
    {
      int k = s0;
      if (energy[k] > thold && j > 0) {
        while (k > 0 && energy[k] > thold) k--;
        tk[j].t0 = s2ts(k);
        if (tk[j].t0 < tk[j - 1].t1) tk[j].t0 = tk[j - 1].t1;
        else s0 = k;
      } else {
        while (energy[k] < thold && k < s1) k++;
        s0 = k;
        tk[j].t0 = s2ts(k);
      }
    }
    {
      int k = s1;
      if (energy[k] > thold) {
        while (k < n_samples - 1 && energy[k] > thold) k++;
        tk[j].t1 = s2ts(k);
        if (j < ns - 1 && j + 1 < n && tk[j].t1 > tk[j + 1].t0) tk[j].t1 = tk[j + 1].t0;
        else s1 = k;
      } else {
        while (energy[k] < thold && k > s0) k--;
        s1 = k;
        tk[j].t1 = s2ts(k);
      }
    }
  }
}

// DTW token timestamps of one window (whisper.cpp whisper_exp_compute_token_level_timestamps_dtw
// as run after each window): the re-forward with alignment-head capture and the DTW kernels
// are enqueued on the DTW stream with their own working set and KV sequence, so they overlap
// the next window's / segment's decode.  The times land in a pinned block; resolve_dtw()
// copies them into the tokens once the job's event has fired.
void State::dtw_timestamps(int i_segment, int n_segments, int seek, int n_frames, const std::string& language) {
  Impl& m = *m_;
  const Vocab& v = ctx_.vocab;
  std::vector<int> toks = {v.sot};
  if (v.multilingual) toks.push_back(v.token_lang(std::max(0, lang_id_from_str(language))));
  const int sot_len = (int)toks.size();
  toks.push_back(v.not_);
  for (int s = i_segment; s < i_segment + n_segments; ++s)
    for (auto& t : result_all[s].tokens)
      if (t.id < v.eot) toks.push_back(t.id);
  toks.push_back(v.eot);
  const int N = (int)toks.size();
  // validated before anything is registered: a job that is never issued would block every later
  // wait on it (positions past n_text_ctx have no embedding, the DTW buffers hold RMAX rows)
  WDR_CHECK(N >= 1 && N <= RMAX, "DTW re-forward: token count out of range");
  Impl::DtwJob job;
  job.i0 = i_segment;
  job.n = n_segments;
  if (m.blk_pool.empty() || m.ev_pool.empty()) {
    // other chain threads may be capturing graphs: a pinned allocation outside the process-wide
    // allocation mutex would invalidate their capture (whisper_ctx.cpp top, ROCm 7.2)
    std::lock_guard<std::recursive_mutex> g(hip_alloc_mutex());
    if (m.blk_pool.empty()) {
      int* blk = nullptr;
      WDR_HIP(hipHostMalloc((void**)&blk, (3 * RMAX + RMAX + 8) * 4, hipHostMallocDefault));
      m.blk_pool.push_back(blk);
    }
    if (m.ev_pool.empty()) {
      hipEvent_t e;
      WDR_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      m.ev_pool.push_back(e);
    }
  }
  job.blk = m.blk_pool.back();
  m.blk_pool.pop_back();
  job.done = m.ev_pool.back();
  m.ev_pool.pop_back();
  Impl::DtwSet& D = m.dset;
  if (batched && dtw_queue_on()) {
    // multi-chain run: the re-forward goes to the context's DTW queue, batched with the other
    // chains' off the decode chain's critical path; the slot keeps a handle (reused only after
    // the pass has read it).  Registered only once the queue has accepted it: a job that is
    // never issued must not be waited on.
    WDR_HIP(hipStreamSynchronize(s_));   // the window's cross-K/V (on-demand encodes) in place
    auto q = std::make_shared<DtwQJob>();
    q->toks = toks;
    q->seq = chain * NSLOT + DTW_SEQ;
    q->xkv = m.xkv();
    q->sot_len = sot_len;
    q->seek = seek;
    q->n_audio = n_frames / 2;
    q->blk = job.blk;
    q->done = job.done;
    DtwQueue& dq = ctx_.dtw_queue();
    dq.submit(q);
    job.q = q;
    m.jobs.push_back(job);
    if (m.xsel >= 0) m.alt_dtw = q;
    else m.slots[m.cur].dtw = q;
    // passes already run no longer write the DTW sequence
    m.qlive.erase(std::remove_if(m.qlive.begin(), m.qlive.end(),
                                 [&](const std::shared_ptr<DtwQJob>& x) {
                                   return dq.is_issued(x) && hipEventQuery(x->fwd) == hipSuccess;
                                 }),
                  m.qlive.end());
    m.qlive.push_back(q);
    return;
  }
  m.jobs.push_back(job);
  if (batched) {
    // multi-chain run (WDR_DTW_QUEUE=0): the re-forward's rows ride in the chain's next batched
    // request (its next prompt prefill, or a request of their own: flush_dtw); the DTW kernels
    // follow on the DTW stream (dtw_after_step)
    WDR_CHECK(!m.pend.on, "DTW re-forward already pending");
    WDR_HIP(hipStreamSynchronize(s_));   // the window's cross-K/V (on-demand encodes) in place
    m.pend.on = true;
    m.pend.toks = toks;
    m.pend.xkv = m.xkv();
    m.pend.slot = -1;
    m.pend.sot_len = sot_len;
    m.pend.seek = seek;
    m.pend.n_audio = n_frames / 2;
    m.pend.blk = job.blk;
    m.pend.done = job.done;
    return;
  } else {
    // queued re-forwards of an earlier batched run write the same DTW sequence: after them
    dtw_queue_fence(m.sd);
    // the window's cross-K/V (encoded ahead, or on demand on the decode stream) must be in place
    WDR_HIP(hipEventRecord(m.ev_sync, s_));
    WDR_HIP(hipStreamWaitEvent(m.sd, m.ev_sync, 0));
    prefill_on(toks.data(), N, DTW_SEQ, false, true, true, m.sd, m.xkv());
  }
  const int n_audio = n_frames / 2;
  launch_dtw(D.cap.as<float>(), (int)ctx_.aheads.size(), N, 1500, n_audio, sot_len, seek, D.nrm.as<float>(),
             D.xdtw.as<float>(), D.times.as<int>(), D.times.as<int>() + RMAX + 4, m.sd);
  WDR_HIP(wdr_memcpy_async(job.blk + 3 * RMAX, D.times.p, (RMAX + 8) * 4, hipMemcpyDeviceToHost, m.sd));
  WDR_HIP(hipEventRecord(job.done, m.sd));
  WDR_HIP(hipEventRecord(m.ev_dtw, m.sd));
}

// the pending DTW re-forward's rows into a batcher request (capture into this state's DTW
// buffer, which the previous job's DTW kernels must have finished reading)
void State::dtw_attach(StepBatcher::Req& q) {
  Impl& m = *m_;
  if (!m.pend.on) return;
  WDR_HIP(hipEventSynchronize(m.ev_dtw));
  q.dn = (int)m.pend.toks.size();
  q.dtok = m.pend.toks.data();
  q.dseq = chain * NSLOT + DTW_SEQ;
  q.dxkv = m.pend.xkv;
  q.dcap = m.dset.cap.as<float>();
  q.dl_end = capture_l_end(ctx_);
}

// after the batched request that carried the pending re-forward: the DTW kernels on the DTW
// stream, the times back to the job's pinned block, and the slot (if its release waited)
void State::dtw_after_step() {
  Impl& m = *m_;
  if (!m.pend.on) return;
  Impl::DtwSet& D = m.dset;
  const int N = (int)m.pend.toks.size();
  launch_dtw(D.cap.as<float>(), (int)ctx_.aheads.size(), N, 1500, m.pend.n_audio, m.pend.sot_len, m.pend.seek,
             D.nrm.as<float>(), D.xdtw.as<float>(), D.times.as<int>(), D.times.as<int>() + RMAX + 4, m.sd);
  WDR_HIP(wdr_memcpy_async(m.pend.blk + 3 * RMAX, D.times.p, (RMAX + 8) * 4, hipMemcpyDeviceToHost, m.sd));
  WDR_HIP(hipEventRecord(m.pend.done, m.sd));
  WDR_HIP(hipEventRecord(m.ev_dtw, m.sd));
  if (m.pend.slot >= 0) WDR_HIP(hipEventRecord(m.slots[m.pend.slot].freed, m.sd));
  m.pend.on = false;
  m.pend.slot = -1;
}

// the pending re-forward as a batcher request of its own (before anything that overwrites its
// slot, and before its result is read)
void State::flush_dtw() {
  Impl& m = *m_;
  if (!m.pend.on) return;
  StepBatcher& b = ctx_.step_batcher(chain);
  StepBatcher::Req q;
  q.n = 0;
  q.vids = m.vids;
  dtw_attach(q);
  b.enter();
  try {
    b.step(q);
  } catch (...) {
    b.leave();
    throw;
  }
  b.leave();
  dtw_after_step();
}

std::vector<DtwTicket> State::take_dtw_jobs() {
  Impl& m = *m_;
  std::vector<DtwTicket> out;
  for (auto& j : m.jobs) out.push_back(DtwTicket{j.i0, j.n, j.blk, (void*)j.done, j.q});
  m.jobs.clear();
  return out;
}

void State::resolve_dtw(DtwTicket& t, std::vector<ResultSeg>& segs) {
  Impl& m = *m_;
  const Vocab& v = ctx_.vocab;
  if (m.pend.on && m.pend.done == (hipEvent_t)t.event) flush_dtw();
  if (t.q) ctx_.dtw_queue().wait_issued(t.q);
  WDR_HIP(hipEventSynchronize((hipEvent_t)t.event));
  t.q.reset();
  const int* times = t.blk + 3 * RMAX;
  const int nt = times[RMAX + 4];
  int k = 0;
  for (int s = t.i0; s < t.i0 + t.n && s < (int)segs.size() && k < nt; ++s)
    for (auto& tok : segs[s].tokens) {
      if (k >= nt) break;
      if (tok.id < v.eot) tok.t_dtw = times[k++];
    }
  m.blk_pool.push_back(t.blk);
  m.ev_pool.push_back((hipEvent_t)t.event);
  t.blk = nullptr;
  t.event = nullptr;
}

// ------------------------------------------------------------------ whisper_full
static int c_round(double x) { return x >= 0 ? (int)std::floor(x + 0.5) : -(int)std::floor(-x + 0.5); }

struct Seq {
  std::vector<TokenData> tokens;
  int result_len = 0, seek_delta = 3000;
  bool has_ts = false, failed = false, completed = false;
  double sum_logprobs = -INFINITY, avg_logprobs = -INFINITY, entropy = 0.0, score = -INFINITY;
  float no_speech_prob = 0.f;
};

static void score_sequence(Seq& s, const FullParams& p) {
  if (s.result_len == 0) return;
  double res = 0.0;
  for (int i = 0; i < s.result_len; ++i) res += s.tokens[i].plog;
  s.sum_logprobs = res;
  s.avg_logprobs = res / s.result_len;
  double pen = s.result_len;
  if (p.length_penalty > 0.0f) pen = std::pow((5.0 + pen) / 6.0, p.length_penalty);
  s.score = res / pen;
  std::map<int, int> cnt;
  int tot = 0;
  for (int i = std::max(0, s.result_len - 32); i < s.result_len; ++i) {
    cnt[s.tokens[i].id]++;
    tot++;
  }
  double ent = 0.0;
  for (auto& kv : cnt) {
    const double pr = kv.second / (double)tot;
    ent -= pr * std::log(pr);
  }
  s.entropy = ent;
}

// whisper.cpp's beam search at t = 0 (WHISPER_SAMPLING_BEAM_SEARCH, patience -1): K decoders
// share the prompt; every step each live decoder proposes its top-K tokens, the candidates are
// ordered by cumulative log-probability (stable: decoder, then rank), duplicate sequences
// are dropped, and live decoders take the best candidates in order (wrapping around when
// there are fewer), their KV caches following their new parents.  Mirrors
// oracle/whisper_full.py WhisperState.decode_beam.
Seq State::decode_beam(const std::vector<int>& prompt, const FullParams& params, float t_cur, int seek, int seek_end,
                       int Lf, int window, float* nosp, bool pre_batched) {
  const Vocab& v = ctx_.vocab;
  const int K = std::max(1, std::min(params.beam_size, std::min(NSEQ, BEAM_KMAX)));
  const int n_max = ctx_.model.hp.n_text_ctx / 2 - 4;
  const int P = (int)prompt.size();
  const int delta_min = 10;
  std::vector<Seq> dec(K);
  std::vector<double> sum_all(K, 0.0);
  // the prompt is in sequence 0 (prefilled by full(), or below in the first batched step): every
  // decoder starts from a copy of it
  auto share_prompt = [&]() {
    std::vector<std::pair<int, int>> share;
    for (int j = 1; j < K; ++j) share.push_back({0, j});
    kv_reorder(share, P);
  };
  if (!pre_batched) share_prompt();
  std::vector<BeamCand> bc((size_t)NSEQ * K);
  std::vector<TokenData> td(NSEQ);
  // multi-chain run: from the second token on, the live beams join the batched step
  struct Seat {
    StepBatcher* b = nullptr;
    ~Seat() {
      if (b) b->leave();
    }
  } seat;
  for (int i = 0; i < n_max; ++i) {
    std::vector<int> act;
    for (int j = 0; j < K; ++j)
      if (!dec[j].completed && !dec[j].failed) act.push_back(j);
    if (act.empty()) break;
    std::vector<LogitsCtl> ctl(act.size());
    for (size_t r = 0; r < act.size(); ++r) {
      const Seq& d = dec[act[r]];
      LogitsCtl& c = ctl[r];
      c = LogitsCtl{};
      c.n_tokens = (int)d.tokens.size();
      c.last_ts = !d.tokens.empty() && d.tokens.back().id >= v.beg;
      c.pen_ts = d.tokens.size() < 2 || d.tokens[d.tokens.size() - 2].id >= v.beg;
      c.has_ts = d.has_ts;
      c.seek_delta = d.seek_delta;
      c.temperature = t_cur;
      if (Lf) {
        if (i == 0) { c.force_kind = 1; c.force_tok = v.beg; }
        else if (i < Lf - 2) c.force_kind = 2;
        else if (i == Lf - 2) { c.force_kind = 1; c.force_tok = v.beg + std::min(1500, std::max(1, (window - delta_min - 1) / 2)); }
        else { c.force_kind = 1; c.force_tok = v.eot; }
      }
    }
    if (i == 0 && pre_batched) {
      // multi-chain run: the prompt prefill rides in the other chains' batched step; its last
      // row's logits give the rules' pick and the top-K candidates, replicated below
      if (!seat.b) {
        seat.b = &ctx_.step_batcher(chain);
        seat.b->enter();
      }
      StepBatcher::Req rq;
      rq.n = 0;
      rq.pn = P;
      rq.ptok = prompt.data();
      rq.pseq = chain * NSLOT + 0;
      rq.pxkv = m_->xkv();
      rq.pctl = ctl[0];
      rq.vids = m_->vids;
      rq.K = K;
      dtw_attach(rq);   // the previous window's re-forward rides along
      const bool lr = m_->lang_ride && m_->lang_ride(rq);
      seat.b->step(rq);
      dtw_after_step();
      if (lr) m_->lang_after(rq);
      times.prefills++;
      td[0] = rq.pout;
      *nosp = rq.pnosp;
      for (int k = 0; k < K; ++k) bc[k] = rq.pcand[k];
      share_prompt();
      for (size_t r = 1; r < act.size(); ++r) {
        td[r] = td[0];
        for (int k = 0; k < K; ++k) bc[r * K + k] = bc[k];
      }
    } else if (i == 0) {
      // every decoder holds the prompt's logits: process once, replicate
      float ns = 0.f;
      run_logits(1, ctl.data(), td.data(), &ns);
      *nosp = ns;
      logits_topk(1, K, bc.data());
      for (size_t r = 1; r < act.size(); ++r) {
        td[r] = td[0];
        for (int k = 0; k < K; ++k) bc[r * K + k] = bc[k];
      }
    } else {
      std::vector<int> toks(act.size()), seqs(act.size()), pos(act.size(), P + i - 1);
      for (size_t r = 0; r < act.size(); ++r) {
        toks[r] = dec[act[r]].tokens.back().id;
        seqs[r] = act[r];
      }
      if (batched) {
        if (!seat.b) {
          seat.b = &ctx_.step_batcher(chain);
          seat.b->enter();
        }
        StepBatcher::Req q;
        q.n = (int)act.size();
        for (int r = 0; r < q.n; ++r) {
          q.tok[r] = toks[r];
          q.seq[r] = chain * NSLOT + seqs[r];
          q.pos[r] = pos[r];
          q.ctl[r] = ctl[r];
        }
        q.xkv = m_->xkv();
        q.vids = m_->vids;
        q.K = K;
        const bool lr = m_->lang_ride && m_->lang_ride(q);   // the next segment's detection row
        seat.b->step(q);
        if (lr) m_->lang_after(q);
        for (int r = 0; r < q.n; ++r) {
          td[r] = q.out[r];
          for (int k = 0; k < K; ++k) bc[(size_t)r * K + k] = q.cand[r * K + k];
        }
        times.decode_steps++;
      } else {
        step_and_sample(toks.data(), seqs.data(), pos.data(), ctl.data(), (int)act.size(), td.data(), K, bc.data());
      }
    }
    struct Cand {
      int j;
      double sum;
      TokenData tok;
    };
    std::vector<Cand> cs;
    for (size_t r = 0; r < act.size(); ++r)
      for (int k = 0; k < K; ++k) {
        const BeamCand& b = bc[r * K + k];
        if (b.id < 0) continue;
        TokenData t;
        t.id = b.id;
        t.tid = td[r].tid;
        t.p = b.p;
        t.plog = b.plog;
        t.pt = td[r].pt;
        t.ptsum = td[r].ptsum;
        if (t.id >= v.beg) {
          t.tid = t.id;
          t.pt = t.p;
        }
        cs.push_back({act[r], sum_all[act[r]] + (double)t.plog, t});
      }
    std::stable_sort(cs.begin(), cs.end(), [](const Cand& a, const Cand& b) { return a.sum > b.sum; });
    std::vector<Cand> uniq;
    for (const Cand& c : cs) {
      bool dup = false;
      for (const Cand& u : uniq) {
        if (u.tok.id != c.tok.id || dec[u.j].tokens.size() != dec[c.j].tokens.size()) continue;
        bool same = true;
        for (size_t q = 0; q < dec[c.j].tokens.size() && same; ++q) same = dec[u.j].tokens[q].id == dec[c.j].tokens[q].id;
        if (same) { dup = true; break; }
      }
      if (!dup) uniq.push_back(c);
    }
    WDR_CHECK(!uniq.empty(), "beam search: no finite candidate");
    std::vector<Seq> nd = dec;
    std::vector<double> ns = sum_all;
    std::vector<std::pair<int, int>> moves;
    size_t cur = 0;
    for (int j : act) {
      if (cur >= uniq.size()) cur = 0;
      const Cand& c = uniq[cur++];
      nd[j] = dec[c.j];
      nd[j].tokens.push_back(c.tok);
      ns[j] = c.sum;
      if (c.j != j) moves.push_back({c.j, j});
    }
    dec.swap(nd);
    sum_all.swap(ns);
    kv_reorder(moves, P + i);
    for (int j : act) {
      Seq& d = dec[j];
      const TokenData& tok = d.tokens.back();
      if (tok.id > v.beg) {
        const int sdn = 2 * (tok.id - v.beg);
        if (d.has_ts && d.seek_delta > sdn && d.result_len < i) {
          d.failed = true;
          continue;
        }
        d.seek_delta = sdn;
        d.result_len = i + 1;
        d.has_ts = true;
      }
      if (tok.id == v.eot || (params.max_tokens > 0 && i >= params.max_tokens) ||
          (d.has_ts && seek + d.seek_delta + delta_min >= seek_end)) {
        if (d.result_len == 0) {
          if (seek + d.seek_delta + delta_min >= seek_end) {
            d.result_len = i + 1;
          } else {
            d.failed = true;
            continue;
          }
        }
        if (params.single_segment) {
          d.result_len = i + 1;
          d.seek_delta = 3000;
        }
        d.completed = true;
        continue;
      }
      if (i == n_max - 1 && (d.result_len == 0 || d.seek_delta < 3000 / 2)) d.failed = true;
    }
  }
  int best = 0;
  double best_score = -INFINITY;
  for (int j = 0; j < K; ++j) {
    Seq& d = dec[j];
    if (d.failed) continue;
    d.tokens.resize(std::min((int)d.tokens.size(), d.result_len));
    score_sequence(d, params);
    if (d.result_len > 32 && d.entropy < params.entropy_thold) {
      d.failed = true;
      continue;
    }
    if (best_score < d.score) {
      best_score = d.score;
      best = j;
    }
  }
  Seq out = dec[best];
  out.tokens.resize(std::min((int)out.tokens.size(), out.result_len));
  score_sequence(out, params);
  return out;
}

// temperature fallback (t > 0): best_of decoders share the prompt and each draws its tokens
// with std::discrete_distribution over the processed probabilities and its own std::mt19937
// (whisper_sample_token with best = false); ranking as in beam search.  Mirrors
// oracle/whisper_full.py WhisperState.decode_sample.
Seq State::decode_sample(const std::vector<int>& prompt, const FullParams& params, float t_cur, int seek, int seek_end,
                         int Lf, int window, float* nosp) {
  Impl& m = *m_;
  sampled = true;
  const Vocab& v = ctx_.vocab;
  const int K = std::max(1, std::min(params.best_of, NSEQ));
  const int n_max = ctx_.model.hp.n_text_ctx / 2 - 4;
  const int P = (int)prompt.size();
  const int delta_min = 10;
  const int V = m.V;
  std::vector<Seq> dec(K);
  {
    std::vector<std::pair<int, int>> share;
    for (int j = 1; j < K; ++j) share.push_back({0, j});
    kv_reorder(share, P);
  }
  m.hp_probs.resize((size_t)NSEQ * V);
  m.hp_logp.resize((size_t)NSEQ * V);
  std::vector<TokenData> td(NSEQ);
  for (int i = 0; i < n_max; ++i) {
    std::vector<int> act;
    for (int j = 0; j < K; ++j)
      if (!dec[j].completed && !dec[j].failed) act.push_back(j);
    if (act.empty()) break;
    std::vector<LogitsCtl> ctl(act.size());
    for (size_t r = 0; r < act.size(); ++r) {
      const Seq& d = dec[act[r]];
      LogitsCtl& c = ctl[r];
      c = LogitsCtl{};
      c.n_tokens = (int)d.tokens.size();
      c.last_ts = !d.tokens.empty() && d.tokens.back().id >= v.beg;
      c.pen_ts = d.tokens.size() < 2 || d.tokens[d.tokens.size() - 2].id >= v.beg;
      c.has_ts = d.has_ts;
      c.seek_delta = d.seek_delta;
      c.temperature = t_cur;
      if (Lf) {
        if (i == 0) { c.force_kind = 1; c.force_tok = v.beg; }
        else if (i < Lf - 2) c.force_kind = 2;
        else if (i == Lf - 2) { c.force_kind = 1; c.force_tok = v.beg + std::min(1500, std::max(1, (window - delta_min - 1) / 2)); }
        else { c.force_kind = 1; c.force_tok = v.eot; }
      }
    }
    int R = (int)act.size();
    if (i == 0) {
      float ns = 0.f;
      run_logits(1, ctl.data(), td.data(), &ns);
      *nosp = ns;
      R = 1;
    } else {
      std::vector<int> toks(act.size()), seqs(act.size()), pos(act.size(), P + i - 1);
      for (size_t r = 0; r < act.size(); ++r) {
        toks[r] = dec[act[r]].tokens.back().id;
        seqs[r] = act[r];
      }
      decoder_step(toks.data(), seqs.data(), pos.data(), R);
      run_logits(R, ctl.data(), td.data(), nullptr);
    }
    launch_logits_probs(m.mb.logits.as<float>(), m.V, m.ctl.as<LogitsCtl>(), m.vids, R, m.work.as<float>(),
                        m.sprobs.as<float>(), m.slogp.as<float>(), s_);
    WDR_HIP(wdr_memcpy_async(m.hp_probs.data(), m.sprobs.p, (size_t)R * V * 4, hipMemcpyDeviceToHost, s_));
    WDR_HIP(wdr_memcpy_async(m.hp_logp.data(), m.slogp.p, (size_t)R * V * 4, hipMemcpyDeviceToHost, s_));
    WDR_HIP(hipStreamSynchronize(s_));
    for (size_t a = 0; a < act.size(); ++a) {
      const int j = act[a];
      const int r = i == 0 ? 0 : (int)a;   // at i == 0 every decoder holds the prompt's distribution
      const float* pr = m.hp_probs.data() + (size_t)r * V;
      std::discrete_distribution<> dist(pr, pr + V);
      TokenData t;
      {   // timestamp statistics exactly as whisper_sample_token (sequential double sums)
        double sum_ts = 0.0, max_ts = 0.0;
        int tid = 0;
        for (int q = v.beg; q < V; ++q) {
          sum_ts += pr[q];
          if (max_ts < pr[q]) {
            max_ts = pr[q];
            tid = q;
          }
        }
        t.tid = tid;
        t.pt = (float)(max_ts / (sum_ts + 1e-10));
        t.ptsum = (float)sum_ts;
      }
      t.id = dist(m.rng[j]);
      t.p = pr[t.id];
      t.plog = m.hp_logp[(size_t)r * V + t.id];
      if (t.id >= v.beg) {
        t.tid = t.id;
        t.pt = t.p;
      }
      dec[j].tokens.push_back(t);
    }
    for (int j : act) {
      Seq& d = dec[j];
      const TokenData& tok = d.tokens.back();
      if (tok.id > v.beg) {
        const int sdn = 2 * (tok.id - v.beg);
        if (d.has_ts && d.seek_delta > sdn && d.result_len < i) {
          d.failed = true;
          continue;
        }
        d.seek_delta = sdn;
        d.result_len = i + 1;
        d.has_ts = true;
      }
      if (tok.id == v.eot || (params.max_tokens > 0 && i >= params.max_tokens) ||
          (d.has_ts && seek + d.seek_delta + delta_min >= seek_end)) {
        if (d.result_len == 0) {
          if (seek + d.seek_delta + delta_min >= seek_end) {
            d.result_len = i + 1;
          } else {
            d.failed = true;
            continue;
          }
        }
        if (params.single_segment) {
          d.result_len = i + 1;
          d.seek_delta = 3000;
        }
        d.completed = true;
        continue;
      }
      if (i == n_max - 1 && (d.result_len == 0 || d.seek_delta < 3000 / 2)) d.failed = true;
    }
  }
  int best = 0;
  double best_score = -INFINITY;
  for (int j = 0; j < K; ++j) {
    Seq& d = dec[j];
    if (d.failed) continue;
    d.tokens.resize(std::min((int)d.tokens.size(), d.result_len));
    score_sequence(d, params);
    if (d.result_len > 32 && d.entropy < params.entropy_thold) {
      d.failed = true;
      continue;
    }
    if (best_score < d.score) {
      best_score = d.score;
      best = j;
    }
  }
  Seq out = dec[best];
  out.tokens.resize(std::min((int)out.tokens.size(), out.result_len));
  score_sequence(out, params);
  return out;
}

int State::full(const FullParams& params, const float* samples, int n, int job, bool async_dtw) {
  WDR_HIP(hipSetDevice(ctx_.cp.gpu_device));
  Impl& m = *m_;
  const Vocab& v = ctx_.vocab;
  const HParams& hp = ctx_.model.hp;
  result_all.clear();
  {   // jobs a previous caller never collected: drain them
    std::vector<DtwTicket> stale = take_dtw_jobs();
    std::vector<ResultSeg> none;
    for (auto& t : stale) resolve_dtw(t, none);
  }
  for (int j = 1; j < NSEQ; ++j) m.rng[j] = std::mt19937(0);   // WHISPER_DECODER_INIT, every call
  sampled = false;
  double t_start = now_s();
  const bool planned = job >= 0 && job < (int)m.plan.pcm.size();
  // the slot goes back to the encode-ahead ring once this segment's last kernel has run
  // the slot goes back to the encode-ahead ring once the decode stream AND the DTW stream
  // (this segment's re-forwards read the slot's cross-K/V) are past it
  struct Release {
    Impl& m;
    hipStream_t s;
    bool on;
    ~Release() {
      if (!on) return;
      (void)hipEventRecord(m.ev_sync, s);
      (void)hipStreamWaitEvent(m.sd, m.ev_sync, 0);
      (void)hipEventRecord(m.slots[m.cur].freed, m.sd);
    }
  } release{m, s_, planned};
  int encoded_seek = -1;
  m.xsel = -1;   // window 0 reads the segment's own slot
  // WDR_CHAIN_LOG=<file>: one line per full() call -- chain, job, wall at entry and exit (s), top_up ms,
  // ready-wait ms, energy ms, decode ms (windows' decode loops), post ms (results, heuristic
  // timestamps, DTW submit) -- where a chain spends the time between its batched steps
  static FILE* clog = getenv("WDR_CHAIN_LOG") ? fopen(getenv("WDR_CHAIN_LOG"), "w") : nullptr;
  static std::mutex clog_mu;
  double c_top = 0, c_ready = 0, c_energy = 0, c_dec = 0, c_post = 0;
  const double c_t0 = now_s();
  m.t_fence = 0;
  m.t_enc_launch = 0;
  if (planned) {
    top_up(job);
    c_top = now_s() - c_t0;
    {
      std::lock_guard<std::mutex> g(m.enc_mu);
      WDR_CHECK((int)m.plan.next_enq > job, "encode-ahead plan out of order");
    }
    m.cur = job % m.S;
    n = m.plan.n[job];
    wait_event_polled(m.slots[m.cur].ready);
    times.encode += now_s() - t_start;   // time the decoder waited on the encode-ahead stream
    c_ready = now_s() - c_t0 - c_top;
    t_start = now_s();
    encoded_seek = 0;
  } else {
    compute_mel(samples, n);
  }
  if (params.token_timestamps) {
    t_beg = t_last = tid_last = 0;
    energy.assign(n, 0.f);
    if (n > 0 && planned && m.slots[m.cur].energy_n == n) {
      // computed on the encode-ahead stream before `ready` (top_up)
      memcpy(energy.data(), m.slots[m.cur].h_energy, (size_t)n * 4);
    } else if (n > 0) {
      if (n > m.energy_cap) {
        m.energy_d = DevMem((size_t)n * 4);
        m.energy_cap = n;
      }
      launch_energy(m.slots[m.cur].x.as<float>(), n, m.energy_d.as<float>(), s_);
      WDR_HIP(wdr_memcpy_async(energy.data(), m.energy_d.p, (size_t)n * 4, hipMemcpyDeviceToHost, s_));
    }
  }
  WDR_HIP(hipStreamSynchronize(s_));
  times.mel += now_s() - t_start;
  c_energy = now_s() - t_start;
  const int seek_start = 0;
  const int seek_end = 1 + (int)((n + 200 - 400) / 160);
  const int delta_min = 10;
  if (seek_end < seek_start + delta_min) return 0;

  std::vector<int> prompt_past;
  if (params.has_initial_prompt && !params.initial_prompt.empty()) prompt_past = v.tokenize(params.initial_prompt);

  auto encode = [&](int seek) {
    if (encoded_seek != seek) {
      const double t = now_s();
      // a later window of the segment: into the other of (slot, spare) when the DTW queue runs
      // the re-forwards -- the one the previous window's queued pass is still reading stays
      // untouched, so the encode does not wait for that pass (configs[2]'s long VAD segments:
      // every later window did)
      if (encoded_seek >= 0 && batched && dtw_queue_on() && odm_alt()) m.xsel = m.xsel < 0 ? 0 : -1;
      flush_dtw();   // a pending re-forward reads the slot this encode overwrites
      stream_fence(s_, m.ev_dtw, host_fence());   // a DTW job may still read this slot
      if (m.xsel >= 0) alt_dtw_fence();   // ... or a queued pass
      else slot_dtw_fence(m.cur, s_);
      WDR_HIP(hipStreamSynchronize(encode_window(seek)));
      times.encode += now_s() - t;
      times.windows++;
      encoded_seek = seek;
    }
  };

  // (before the language detection: its row may ride in a batched step, which applies batch[0]'s
  // vocabulary rules to every row)
  if (params.max_initial_ts > 0.0f) {
    const float precision = 30.0f / hp.n_audio_ctx;
    m.vids.max_initial_tid = (int)std::round(params.max_initial_ts / precision);
  } else {
    m.vids.max_initial_tid = -1;
  }
  m.vids.suppress_blank = params.suppress_blank ? 1 : 0;

  std::string language = params.language;
  if (language.empty() || language == "auto") {
    encode(seek_start);
    const double t = now_s();
    std::vector<float> ll(100);
    if (lang_hint >= 0 && lang_hint < 100) {
      // the engine's fix-up re-decode of a segment whose window 0 was already detected: the
      // detection depends on nothing but that window, so its argmax stands (lang_hint)
      ll.assign(100, 0.f);
      ll[lang_hint] = 1.f;
    } else if (planned && m.plan.detect_lang && m.lang_src[m.cur] == job) {
      // computed on the encode stream before `ready`, or by a detection row of an earlier batched step
      memcpy(ll.data(), m.h_lang + (size_t)m.cur * 100, 100 * 4);
    } else if (planned && batched && m.plan.detect_lang && lang_piggyback()) {
      // not detected yet (a plan's segment 0, or its window was encoded only after the segment
      // before had decoded): the detection row alone in a batched step, beside the other chains'
      StepBatcher& b = ctx_.step_batcher(chain);
      b.enter();
      struct Leave {
        StepBatcher* b;
        ~Leave() { b->leave(); }
      } leave_b{&b};
      StepBatcher::Req rq;
      rq.n = 0;
      rq.ln = 1;
      rq.lseq = chain * NSLOT + LANG_SEQ;
      rq.lxkv = m.xkv();
      rq.vids = m.vids;
      b.step(rq);
      memcpy(ll.data(), rq.lout, 100 * 4);
    } else {
      const int sot = v.sot;
      decoder_prefill(&sot, 1, 0, true, false);
      times.lang_passes++;
      times.lang_rows++;
      WDR_HIP(wdr_memcpy_async(ll.data(), m.mb.logits.as<float>() + v.sot + 1, 100 * 4, hipMemcpyDeviceToHost, s_));
      WDR_HIP(hipStreamSynchronize(s_));
    }
    int best = 0;
    for (int i = 1; i < 100; ++i)
      if (ll[i] > ll[best]) best = i;
    lang_id = best;
    language = kLangs[best];
    times.decode += now_s() - t;
    times.lang += now_s() - t;
  }
  std::vector<int> prompt_init = {v.sot};
  if (v.multilingual) {
    lang_id = std::max(0, lang_id_from_str(language));
    prompt_init.push_back(v.token_lang(lang_id));
    prompt_init.push_back(params.translate ? v.translate : v.transcribe);
  }
  std::vector<float> temps;
  if (params.temperature_inc > 0.0f) {
    for (float t = params.temperature; t < 1.0f + 1e-6f; t += params.temperature_inc) temps.push_back(t);
  } else {
    temps.push_back(params.temperature);
  }

  // lang_piggyback: the next plan segment's detection row rides in one of this segment's batched
  // steps once its window is encoded (its slot's `ready` has passed); at most one per segment
  const int lang_nx = job + 1;
  const bool lang_want = planned && batched && m.plan.detect_lang && lang_piggyback() &&
                         lang_nx < (int)m.plan.n.size();
  bool lang_done = !lang_want;
  auto lang_ride = [&](StepBatcher::Req& rq) {
    if (lang_done) return false;
    {
      std::lock_guard<std::mutex> g(m.enc_mu);   // lang_src of the segment is written before next_enq
      if ((int)m.plan.next_enq <= lang_nx) return false;
    }
    const int sl = lang_nx % m.S;
    if (m.lang_src[sl] == lang_nx) {   // the encode-ahead batch's own pass (a plan's first batch)
      lang_done = true;
      return false;
    }
    if (hipEventQuery(m.slots[sl].ready) != hipSuccess) return false;
    rq.ln = 1;
    rq.lseq = chain * NSLOT + LANG_SEQ;
    rq.lxkv = m.xkv_ring.as<f16>() + (size_t)sl * m.xkv_slot_elems;
    return true;
  };
  auto lang_after = [&](const StepBatcher::Req& rq) {
    const int sl = lang_nx % m.S;
    memcpy(m.h_lang + (size_t)sl * 100, rq.lout, 100 * 4);
    m.lang_src[sl] = lang_nx;   // (its row and slot read are counted with the batched step's)
    lang_done = true;
  };
  m.lang_ride = lang_ride;   // for decode_beam's batched steps, cleared when this call ends
  m.lang_after = lang_after;
  struct LangClear {
    Impl& m;
    ~LangClear() {
      m.lang_ride = nullptr;
      m.lang_after = nullptr;
    }
  } lang_clear{m};

  int seek = seek_start;
  const int n_text_ctx = hp.n_text_ctx;
  std::vector<int> prompt;
  while (true) {
    if (seek + 100 >= seek_end) break;
    bool prompt_timed = false;
    encode(seek);
    if (seek > seek_start && seek + 500 >= seek_end) prompt_past.clear();
    Seq best;
    const double t_dec = now_s();
    for (size_t it = 0; it < temps.size(); ++it) {
      const float t_cur = temps[it];
      prompt.clear();
      if (!prompt_past.empty() && t_cur < 0.5f && params.n_max_text_ctx > 0) {
        const int n_take = std::min(std::min(params.n_max_text_ctx, n_text_ctx / 2), (int)prompt_past.size());
        prompt.push_back(v.prev);
        prompt.insert(prompt.end(), prompt_past.end() - n_take, prompt_past.end());
      }
      prompt.insert(prompt.end(), prompt_init.begin(), prompt_init.end());
      const bool single = params.greedy && t_cur <= 0.f;
      // multi-chain greedy run: the prompt prefill rides in the batched step (its last row's
      // logits give the first token), so the chain never leaves the batch
      const bool pre_batched = batched && single;
      // multi-chain beam search at t = 0: its prompt prefill rides in a batched step too, with the
      // prompt's top-K candidates (decode_beam)
      // (WDR_BEAM_PREFILL=0: on the chain's own stream as before, A/B; read once)
      static const bool beam_pre_on = !(getenv("WDR_BEAM_PREFILL") && atoi(getenv("WDR_BEAM_PREFILL")) == 0);
      const bool beam_pre = beam_pre_on && batched && !params.greedy && t_cur <= 0.f;
      if (!pre_batched && !beam_pre) {
        flush_dtw();
        WDR_HIP(hipEventRecord(m.ev_p0, s_));
        decoder_prefill(prompt.data(), (int)prompt.size(), 0, true, false);
        WDR_HIP(hipEventRecord(m.ev_p1, s_));
        prompt_timed = true;
      }
      const int window = std::min(seek_end - seek, 3000);
      int Lf = 0;
      if (params.force_len_rate > 0.f) Lf = std::max(3, c_round(params.force_len_rate * window / 100.0) + 3);
      Seq sq;
      const int n_max = n_text_ctx / 2 - 4;
      float nosp = 0.f;
      if (t_cur > 0.f) {
        sq = decode_sample(prompt, params, t_cur, seek, seek_end, Lf, window, &nosp);
      } else if (!params.greedy) {
        sq = decode_beam(prompt, params, t_cur, seek, seek_end, Lf, window, &nosp, beam_pre);
      }
      // multi-chain run: from the second token on, this chain's row joins the batched step
      struct Lockstep {
        StepBatcher* b = nullptr;
        ~Lockstep() {
          if (b) b->leave();
        }
      } lockstep;
      for (int i = 0; i < n_max && single; ++i) {
        LogitsCtl c{};
        c.n_tokens = (int)sq.tokens.size();
        c.last_ts = !sq.tokens.empty() && sq.tokens.back().id >= v.beg;
        c.pen_ts = sq.tokens.size() < 2 || sq.tokens[sq.tokens.size() - 2].id >= v.beg;
        c.has_ts = sq.has_ts;
        c.seek_delta = sq.seek_delta;
        c.temperature = t_cur;
        if (Lf) {
          if (i == 0) { c.force_kind = 1; c.force_tok = v.beg; }
          else if (i < Lf - 2) c.force_kind = 2;
          else if (i == Lf - 2) { c.force_kind = 1; c.force_tok = v.beg + std::min(1500, std::max(1, (window - delta_min - 1) / 2)); }
          else { c.force_kind = 1; c.force_tok = v.eot; }
        }
        TokenData tok;
        float ns = 0.f;
        if (i == 0 && pre_batched) {
          // the prompt prefill rides in the other chains' batched step (WDR_PREFILL_SPLIT=1: on a
          // prefill batcher of its own, A/B)
          StepBatcher* pb = nullptr;
          if (ctx_.prefill_split) {
            pb = &ctx_.prefill_batcher();
            pb->enter();
          } else if (!lockstep.b) {
            lockstep.b = &ctx_.step_batcher(chain);
            lockstep.b->enter();
          }
          struct Leave {
            StepBatcher* b;
            ~Leave() {
              if (b) b->leave();
            }
          } leave_pb{pb};
          StepBatcher::Req rq;
          rq.n = 0;
          rq.pn = (int)prompt.size();
          rq.ptok = prompt.data();
          rq.pseq = chain * NSLOT + 0;
          rq.pxkv = m.xkv();
          rq.pctl = c;
          rq.vids = m.vids;
          dtw_attach(rq);   // the previous window's re-forward rides along
          const bool lr = lang_ride(rq);
          (pb ? pb : lockstep.b)->step(rq);
          dtw_after_step();
          if (lr) lang_after(rq);
          tok = rq.pout;
          nosp = rq.pnosp;
          times.prefills++;
        } else if (i == 0) {
          run_logits(1, &c, &tok, &ns);
          nosp = ns;
        } else {
          const int pos = (int)prompt.size() + i - 1;
          const int seq0 = 0;
          const int prev_id = sq.tokens.back().id;
          if (batched) {
            if (!lockstep.b) {
              lockstep.b = &ctx_.step_batcher(chain);
              lockstep.b->enter();
            }
            StepBatcher::Req rq = row_req(prev_id, chain * NSLOT + seq0, pos, m.xkv(), c, m.vids);
            const bool lr = lang_ride(rq);
            lockstep.b->step(rq);
            if (lr) lang_after(rq);
            tok = rq.out[0];
            times.decode_steps++;
          } else {
            step_and_sample(&prev_id, &seq0, &pos, &c, 1, &tok);
          }
        }
        sq.tokens.push_back(tok);
        if (tok.id > v.beg) {
          const int sdn = 2 * (tok.id - v.beg);
          if (sq.has_ts && sq.seek_delta > sdn && sq.result_len < i) {
            sq.failed = true;
            break;
          }
          sq.seek_delta = sdn;
          sq.result_len = i + 1;
          sq.has_ts = true;
        }
        if (tok.id == v.eot || (params.max_tokens > 0 && i >= params.max_tokens) ||
            (sq.has_ts && seek + sq.seek_delta + delta_min >= seek_end)) {
          if (sq.result_len == 0) {
            if (seek + sq.seek_delta + delta_min >= seek_end) {
              sq.result_len = i + 1;
            } else {
              sq.failed = true;
              break;
            }
          }
          if (params.single_segment) {
            sq.result_len = i + 1;
            sq.seek_delta = 3000;
          }
          sq.completed = true;
          break;
        }
        if (i == n_max - 1 && (sq.result_len == 0 || sq.seek_delta < 3000 / 2)) {
          sq.failed = true;
          break;
        }
      }
      if (single) {
        sq.tokens.resize(std::min((int)sq.tokens.size(), sq.result_len));
        score_sequence(sq, params);
        if (!sq.failed && sq.result_len > 32 && sq.entropy < params.entropy_thold) sq.failed = true;
      }
      sq.no_speech_prob = nosp;
      best = sq;
      bool success = true;
      if (it != temps.size() - 1) {
        if (sq.failed || (sq.avg_logprobs < params.logprob_thold && sq.no_speech_prob < params.no_speech_thold))
          success = false;
      }
      if (success) break;
    }
    times.decode += now_s() - t_dec;
    c_dec += now_s() - t_dec;
    const double t_post = now_s();
    struct PostT {
      double t0;
      double& acc;
      ~PostT() { acc += now_s() - t0; }
    } post_t{t_post, c_post};
    if (prompt_timed) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, m.ev_p0, m.ev_p1) == hipSuccess) times.prompt_gpu += ms * 1e-3;
    }
    int seek_delta = best.seek_delta;
    const int result_len = best.result_len;
    auto& tokens_cur = best.tokens;
    const size_t n_before = result_all.size();
    const bool is_no_speech = best.no_speech_prob > params.no_speech_thold && best.avg_logprobs < params.logprob_thold;
    std::vector<int> new_past;
    if (!prompt.empty() && prompt.front() == v.prev)
      new_past.insert(new_past.end(), prompt.begin() + 1, prompt.end() - prompt_init.size());
    for (int i = 0; i < result_len && !is_no_speech; ++i) new_past.push_back(tokens_cur[i].id);
    prompt_past = new_past;
    if (!tokens_cur.empty() && !is_no_speech) {
      const long long t0 = seek + 2LL * (tokens_cur.front().tid - v.beg);
      std::string text;
      for (auto& t : tokens_cur)
        if (t.id < v.eot) text += v.id_to_token[t.id];
      if (!text.empty()) {
        const long long t1 = seek + seek_delta;
        result_all.push_back({t0, t1, text, tokens_cur});
        if (params.token_timestamps) heuristic_timestamps((int)result_all.size() - 1, params);
      }
    }
    const int n_new = (int)(result_all.size() - n_before);
    if (!ctx_.aheads.empty() && n_new) {
      const double t = now_s();
      const int n_frames = std::min(std::min(3000, seek_delta), seek_end - seek);
      dtw_timestamps((int)n_before, n_new, seek, n_frames, language);
      times.dtw += now_s() - t;
    }
    if (tokens_cur.size() > 1 && tokens_cur[tokens_cur.size() - 2].id < v.beg && tokens_cur.back().id > v.beg)
      seek_delta = std::min(seek_end - seek, 3000);
    seek += seek_delta;
  }
  if (clog) {
    std::lock_guard<std::mutex> g(clog_mu);
    fprintf(clog, "%d %d %.6f %.6f %.3f %.3f %.3f %.3f %.3f %.3f %.3f\n", chain, job, c_t0, now_s(), c_top * 1e3,
            c_ready * 1e3, c_energy * 1e3, c_dec * 1e3, c_post * 1e3, m.t_fence.load() * 1e-6,
            m.t_enc_launch.load() * 1e-6);
    fflush(clog);
  }
  // the last window's pending re-forward (WDR_DTW_QUEUE=0) runs before the slot is released:
  // deferring the release into the next segment's first request let an encode-ahead batch wait
  // on the slot's previous `freed` record and overwrite the cross-K/V the re-forward still reads
  flush_dtw();
  if (!async_dtw) {
    std::vector<DtwTicket> tk = take_dtw_jobs();
    for (auto& t : tk) resolve_dtw(t, result_all);
  }
  return 0;
}

}  // namespace wdr

// ------------------------------------------------------------------ multi-chain step batcher
namespace wdr {

// rows of one batched launch: decode rows, prompt prefills and DTW re-forwards of every chain
// of the context (a prefill <= 228 rows, a DTW re-forward <= 229; 16384 rows cover 32 chains'
// typical mixes, above that 470 per chain), logit rows: 8 beams + a prefill's last row per chain
static int rows_cap(const Context& c) { return std::max(16384, c.max_chains * 470); }
static int logit_cap(const Context& c) { return std::max(320, c.max_chains * 10); }

struct StepBatcher::Impl {
  std::mutex mu;
  std::condition_variable cv;
  int active = 0;                 // chains inside the batcher
  std::vector<Req*> pend;         // requests of the batch being collected
  bool running = false;           // a batch is on the GPU (new requests collect for the next)
  // a batch launches when every chain inside has submitted, or WDR_BATCH_WAIT_US after the GPU
  // became free with at least one request waiting: a chain busy on the host (a segment's end,
  // its DTW submission, the next prompt) joins the following batch instead of holding the other
  // chains' rows back -- exact, since a row's result does not depend on its batch (rows.h)
  double t_free = 0;              // when the last batch's results were handed out
  double t_first = 0;             // when the oldest pending request arrived
  // WDR_BATCH_WAIT_US (read when the batcher is made): how long a batch may wait for stragglers
  // once the GPU is free (default 1000 us: at 40 chains 300 / 600 / 1000 us gave 744 / 755 / 758
  // xRT, profiles/r04/ab_wait40.txt; negative: wait for every chain, the round-3 rule)
  double wait_s = 1000e-6;
  hipStream_t s = nullptr;
  int d = 0, V = 0, H = 0;
  int RB = 0, LB = 0;             // row / logit-row capacity of one launch
  RowsBufs bufs;
  std::unique_ptr<RowBatch> tb;
  DevMem work, tokout, ctl, beamc;
  LogitsCtl* h_ctl = nullptr;     // [LB]
  TokOut* h_tok = nullptr;        // [LB]
  BeamCand* h_beam = nullptr;     // [LB][BEAM_KMAX]
  float* h_lang = nullptr;        // [LB][100]: language logits of the batch's detection rows
  struct G {
    hipGraphExec_t exec = nullptr;
    VocabIds vids{};
    void drop() {
      if (exec) (void)hipGraphExecDestroy(exec);
      exec = nullptr;
    }
  };
  std::map<long long, G> graphs;  // decode-only batches, by (K, group kind, groups, rows)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;   // a launch's GPU span (WDR_BATCH_LOG)
};

StepBatcher::StepBatcher(Context& ctx) : ctx_(ctx), m_(new Impl) {
  WDR_HIP(hipSetDevice(ctx.cp.gpu_device));
  Impl& m = *m_;
  const HParams& hp = ctx.model.hp;
  m.d = hp.n_text_state;
  m.V = hp.n_vocab;
  m.H = hp.n_text_head;
  int lo = 0, hi = 0;
  WDR_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
  m.s = dedicated_stream("WDR_BATCH_HWQ", false, hi);
  if (const char* e = getenv("WDR_BATCH_WAIT_US")) m.wait_s = atof(e) * 1e-6;
  const int RB = rows_cap(ctx), LB = logit_cap(ctx);
  m.RB = RB;
  m.LB = LB;
  m.bufs.alloc(RB, LB, m.d, m.H, m.V);
  m.tb = std::make_unique<RowBatch>(RB, LB, RB);
  m.work = DevMem((size_t)LB * m.V * 4);
  m.tokout = DevMem(LB * sizeof(TokOut));
  m.ctl = DevMem(LB * sizeof(LogitsCtl));
  m.beamc = DevMem((size_t)LB * BEAM_KMAX * sizeof(BeamCand));
  WDR_HIP(hipHostMalloc((void**)&m.h_beam, (size_t)LB * BEAM_KMAX * sizeof(BeamCand), hipHostMallocDefault));
  WDR_HIP(hipHostMalloc((void**)&m.h_ctl, LB * sizeof(LogitsCtl), hipHostMallocDefault));
  WDR_HIP(hipHostMalloc((void**)&m.h_tok, LB * sizeof(TokOut), hipHostMallocDefault));
  WDR_HIP(hipHostMalloc((void**)&m.h_lang, (size_t)LB * 100 * 4, hipHostMallocDefault));
  WDR_HIP(hipEventCreate(&m.ev0));
  WDR_HIP(hipEventCreate(&m.ev1));
}

StepBatcher::~StepBatcher() {
  if (!m_) return;
  if (m_->s) (void)hipStreamSynchronize(m_->s);
  for (auto& g : m_->graphs) g.second.drop();
  if (m_->s) {
    (void)hipStreamSynchronize(m_->s);
    (void)hipStreamDestroy(m_->s);
  }
  (void)hipHostFree(m_->h_ctl);
  (void)hipHostFree(m_->h_tok);
  (void)hipHostFree(m_->h_beam);
  (void)hipHostFree(m_->h_lang);
  if (m_->ev0) (void)hipEventDestroy(m_->ev0);
  if (m_->ev1) (void)hipEventDestroy(m_->ev1);
}

StepBatcher& Context::step_batcher(int chain) {
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  if (batchers.empty()) batchers.resize(std::max(1, n_batchers));
  auto& b = batchers[(size_t)std::max(0, chain) % batchers.size()];
  if (!b) b = std::make_unique<StepBatcher>(*this);
  return *b;
}

StepBatcher& Context::prefill_batcher() {
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  if (!prefill_b) prefill_b = std::make_unique<StepBatcher>(*this);
  return *prefill_b;
}

Context::BatchStats Context::batcher_stats() {
  BatchStats o;
  for (int i = 0; i < std::max(1, n_batchers) + (prefill_b ? 1 : 0); ++i) {
    StepBatcher& sb = i < std::max(1, n_batchers) ? step_batcher(i) : *prefill_b;
    o.launches += sb.launches;
    o.rows += sb.rows;
    o.prefill_rows += sb.prefill_rows;
    o.dtw_rows += sb.dtw_rows;
    o.prefills += sb.prefills;
    o.dtws += sb.dtws;
    o.mixed += sb.mixed;
    o.vgroups += sb.vgroups;
    o.tiles += sb.tiles;
    o.step_s = std::max(o.step_s, sb.step_s);
  }
  if (dtwq) {
    o.dq_passes = dtwq->passes;
    o.dq_rows = dtwq->rows;
    o.dq_jobs = dtwq->jobs;
  }
  return o;
}

void StepBatcher::enter() {
  std::lock_guard<std::mutex> g(m_->mu);
  m_->active++;
}

void StepBatcher::leave() {
  std::lock_guard<std::mutex> g(m_->mu);
  m_->active--;
  m_->cv.notify_all();   // a waiter may now hold the last missing request
}

void StepBatcher::step(Req& r) {
  Impl& m = *m_;
  std::unique_lock<std::mutex> lk(m.mu);
  r.done = false;
  r.err = nullptr;
  if (m.pend.empty()) m.t_first = now_s();
  m.pend.push_back(&r);
  const double wait = m.wait_s;
  while (!r.done) {
    if (!m.running && !m.pend.empty()) {
      const bool all = (int)m.pend.size() >= m.active;
      const double t_go = std::max(m.t_free, m.t_first) + wait;
      if (all || (wait >= 0 && now_s() >= t_go)) {
        std::vector<Req*> batch;
        batch.swap(m.pend);
        m.running = true;
        lk.unlock();
        std::exception_ptr e;
        try {
          launch(batch);
        } catch (...) {
          e = std::current_exception();
        }
        lk.lock();
        for (Req* q : batch) {
          q->err = e;
          q->done = true;
        }
        m.running = false;
        m.t_free = now_s();
        m.cv.notify_all();
        continue;
      }
      if (wait >= 0) {
        m.cv.wait_for(lk, std::chrono::duration<double>(std::max(t_go - now_s(), 1e-6)));
        continue;
      }
    }
    m.cv.wait(lk);
  }
  if (r.err) std::rethrow_exception(r.err);
}

// one batch: every request's DTW rows, decode rows and prefill rows as ONE rows forward (rows.h),
// then the logit rules + greedy pick of every logit row, and the top-K candidates when a request
// asks for them.  Decode-only batches replay a graph captured per shape; batches holding a
// prefill or a DTW re-forward (shapes vary with the prompt) launch eagerly.
void StepBatcher::launch(std::vector<Req*>& batch) {
  Impl& m = *m_;
  RowBatch& tb = *m.tb;
  tb.clear();
  int K = 0, n_pre = 0, n_dtw = 0, n_lang = 0;
  std::vector<int> lidx(batch.size(), -1), lpre(batch.size(), -1), llang(batch.size(), -1);
  for (size_t i = 0; i < batch.size(); ++i) {
    Req* q = batch[i];
    WDR_CHECK(q->n >= 0 && q->n <= kRows && q->K >= 0 && q->K <= BEAM_KMAX && q->pn >= 0 && q->dn >= 0 &&
                  (q->ln == 0 || (q->ln == 1 && q->lxkv)) && q->n + q->pn + q->dn + q->ln > 0,
              "step batcher: bad request");
    if (q->dn > 0) {
      RowGroupDesc g;
      g.n = q->dn;
      g.tok = q->dtok;
      g.seq0 = q->dseq;
      g.xkv = q->dxkv;
      g.cap = q->dcap;
      g.l_end = q->dl_end;
      tb.add(g);
      n_dtw += q->dn;
      dtws++;
    }
    if (q->n > 0) {
      RowGroupDesc g;
      g.n = q->n;
      g.tok = q->tok;
      g.seq = q->seq;
      g.pos = q->pos;
      g.xkv = q->xkv;
      g.logits = 2;
      lidx[i] = tb.add(g);
      for (int j = 0; j < q->n; ++j) m.h_ctl[lidx[i] + j] = q->ctl[j];
    }
    if (q->n > 0 || q->pn > 0) K = std::max(K, q->K);
    if (q->pn > 0) {
      RowGroupDesc g;
      g.n = q->pn;
      g.tok = q->ptok;
      g.seq0 = q->pseq;
      g.xkv = q->pxkv;
      g.logits = 1;
      lpre[i] = tb.add(g);
      m.h_ctl[lpre[i]] = q->pctl;
      n_pre += q->pn;
      prefills++;
    }
    if (q->ln > 0) {   // language detection row: SOT at position 0 (whisper.cpp's detection pass)
      RowGroupDesc g;
      g.n = 1;
      g.tok = &q->vids.sot;
      g.seq0 = q->lseq;
      g.xkv = q->lxkv;
      g.logits = 1;
      llang[i] = tb.add(g);
      m.h_ctl[llang[i]] = LogitsCtl{};   // its pick runs and is ignored: the language logits are read raw
      n_lang++;
    }
  }
  const int R = tb.R, NL = tb.n_logit;
  const VocabIds& vids = batch[0]->vids;
  WDR_HIP(hipSetDevice(ctx_.cp.gpu_device));
  RowsIO io = m.bufs.io(ctx_, m.V);
  auto tail = [&]() {   // logit rules, greedy pick and top-K of the logit rows (after the forward)
    if (NL == 0) return;
    WDR_HIP(wdr_memcpy_async(m.ctl.p, m.h_ctl, NL * sizeof(LogitsCtl), hipMemcpyHostToDevice, m.s));
    launch_logits_process(m.bufs.logits.as<float>(), m.V, m.ctl.as<LogitsCtl>(), vids, NL, m.work.as<float>(),
                          m.tokout.as<TokOut>(), m.s);
    WDR_HIP(wdr_memcpy_async(m.h_tok, m.tokout.p, NL * sizeof(TokOut), hipMemcpyDeviceToHost, m.s));
    for (size_t i = 0; i < batch.size(); ++i)
      if (llang[i] >= 0)
        WDR_HIP(wdr_memcpy_async(m.h_lang + (size_t)llang[i] * 100,
                                 m.bufs.logits.as<float>() + (size_t)llang[i] * m.V + vids.sot + 1, 100 * 4,
                                 hipMemcpyDeviceToHost, m.s));
    if (K > 0) {
      launch_logits_topk(m.bufs.logits.as<float>(), m.V, m.ctl.as<LogitsCtl>(), vids, NL, K, m.work.as<float>(),
                         m.beamc.as<BeamCand>(), m.s);
      WDR_HIP(wdr_memcpy_async(m.h_beam, m.beamc.p, (size_t)NL * K * sizeof(BeamCand), hipMemcpyDeviceToHost, m.s));
    }
  };
  const double t_step = now_s();
  const bool decode_only = n_pre == 0 && n_dtw == 0 && n_lang == 0;
  // only a batch that would replay a graph draws an eager sampled run (prof.h): mixed batches
  // always run eagerly and are sampled at the base rate
  const bool sampled = decode_only && !no_graph() && prof_step();
  static FILE* blog = getenv("WDR_BATCH_LOG") ? fopen(getenv("WDR_BATCH_LOG"), "w") : nullptr;
  if (blog) WDR_HIP(hipEventRecord(m.ev0, m.s));
  if (sampled || no_graph() || !decode_only) {
    // sampled step for live kernel timing (prof.h: its launches run eagerly, 1 in 2 of them
    // clocked), graphs disabled, or a mixed batch
    prof_in_step(sampled);
    try {
      tb.upload(io, m.s, true, false);
      rows_forward(ctx_, io, R, m.s);
      tail();
    } catch (...) {
      prof_in_step(false);
      throw;
    }
    prof_in_step(false);
  } else {
    // the cross-attention grid has one workgroup row per group: the group count is in the key
    const bool grouped = tb.vgrp_max > 1;
    Impl::G& g = m.graphs[((long long)K << 40) + (grouped ? 1ll << 39 : 0ll) + ((long long)tb.n_vgrp << 16) + R];
    if (g.exec && memcmp(&g.vids, &vids, sizeof(VocabIds)) != 0) g.drop();
    if (!g.exec) {
      std::lock_guard<std::recursive_mutex> cap_lock(hip_alloc_mutex());   // no allocation meanwhile
      hipGraph_t graph;
      prof_capture(true);
      WDR_HIP(hipStreamBeginCapture(m.s, hipStreamCaptureModeRelaxed));
      tb.upload(io, m.s, true, false);
      rows_forward(ctx_, io, R, m.s);
      tail();
      prof_capture(false);
      WDR_HIP(hipStreamEndCapture(m.s, &graph));
      WDR_HIP(hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0));
      WDR_HIP(hipGraphDestroy(graph));
      g.vids = vids;
    } else {
      tb.upload(io, m.s, false, false);   // the captured copy node reads the staging
    }
    {
      std::mutex* mu = launch_lock();   // WDR_LAUNCH_LOCK (prof.h)
      if (mu) mu->lock();
      const hipError_t ge = hipGraphLaunch(g.exec, m.s);
      if (mu) mu->unlock();
      WDR_HIP(ge);
    }
  }
  if (blog) WDR_HIP(hipEventRecord(m.ev1, m.s));
  const double t_enq = now_s();   // host side of the launch done (eager: every kernel enqueued)
  WDR_HIP(hipStreamSynchronize(m.s));
  auto tok_of = [&](int i) {
    const TokOut& o = m.h_tok[i];
    TokenData t{};
    t.id = o.id;
    t.tid = o.tid;
    t.p = o.p;
    t.plog = o.plog;
    t.pt = o.pt;
    t.ptsum = o.ptsum;
    return t;
  };
  for (size_t i = 0; i < batch.size(); ++i) {
    Req* q = batch[i];
    if (lidx[i] >= 0)
      for (int j = 0; j < q->n; ++j) {
        q->out[j] = tok_of(lidx[i] + j);
        if (q->K > 0)
          for (int k = 0; k < q->K; ++k) q->cand[j * q->K + k] = m.h_beam[(size_t)(lidx[i] + j) * K + k];
      }
    if (llang[i] >= 0) memcpy(q->lout, m.h_lang + (size_t)llang[i] * 100, 100 * 4);
    if (lpre[i] >= 0) {
      q->pout = tok_of(lpre[i]);
      q->pnosp = m.h_tok[lpre[i]].nosp_prob;
      for (int k = 0; k < q->K; ++k) q->pcand[k] = m.h_beam[(size_t)lpre[i] * K + k];
    }
  }
  launches++;
  rows += R;
  vgroups += tb.n_vgrp;
  tiles += tb.n_tiles;
  prefill_rows += n_pre;
  dtw_rows += n_dtw;
  if (!decode_only) mixed++;
  const double t_end = now_s();
  step_s += t_end - t_step;
  // WDR_BATCH_LOG=<file>: one line per launch (start s, rows, wall ms, prefill rows, DTW rows,
  // GPU ms: the launch's span on its stream, first command to last, host enqueue ms)
  if (blog) {
    float gms = 0.f;
    (void)hipEventElapsedTime(&gms, m.ev0, m.ev1);
    fprintf(blog, "%.6f %d %.3f %d %d %.3f %.3f\n", t_step, R, (t_end - t_step) * 1e3, n_pre, n_dtw, gms,
            (t_enq - t_step) * 1e3);
    fflush(blog);
  }
}

}  // namespace wdr

// ------------------------------------------------------------------ DTW queue
namespace wdr {

DtwQJob::DtwQJob() { WDR_HIP(hipEventCreateWithFlags(&fwd, hipEventDisableTiming)); }
DtwQJob::~DtwQJob() {
  if (fwd) (void)hipEventDestroy(fwd);
}

struct DtwQueue::Impl {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::shared_ptr<DtwQJob>> pend;
  int pend_rows = 0;
  int urgent = 0;
  bool stop = false;
  std::exception_ptr err;
  std::thread th;
  hipStream_t s = nullptr;
  int RB = 0, A = 1, l_end = 1, min_rows = 256;
  double max_age = 0.05;
  RowsBufs bufs;
  std::unique_ptr<RowBatch> tb;
  DevMem cap, nrm, xdtw, times;
};

DtwQueue& Context::dtw_queue() {
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  if (!dtwq) dtwq = std::make_unique<DtwQueue>(*this);
  return *dtwq;
}

DtwQueue::DtwQueue(Context& ctx) : m_(new Impl), ctx_(ctx) {
  WDR_HIP(hipSetDevice(ctx.cp.gpu_device));
  Impl& m = *m_;
  const HParams& hp = ctx.model.hp;
  m.A = std::max<int>(1, (int)ctx.aheads.size());
  m.l_end = capture_l_end(ctx);
  m.RB = 1024;   // rows of one pass (a DTW re-forward is <= RMAX + 1 rows)
  if (const char* e = getenv("WDR_DTW_MIN_ROWS")) m.min_rows = std::max(1, atoi(e));
  if (const char* e = getenv("WDR_DTW_AGE_MS")) m.max_age = std::max(0.0, atof(e)) * 1e-3;
  int lo = 0, hi = 0;
  WDR_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
  m.s = dedicated_stream("WDR_DTWQ_HWQ", false, lo);
  m.bufs.alloc(m.RB, 1, hp.n_text_state, hp.n_text_head, hp.n_vocab);
  m.tb = std::make_unique<RowBatch>(m.RB, 1, m.RB);
  m.cap = DevMem((size_t)m.A * m.RB * 1500 * 4);
  m.nrm = DevMem((size_t)m.A * RMAX * 1500 * 4);
  m.xdtw = DevMem((size_t)RMAX * 1500 * 4);
  m.times = DevMem((RMAX + 8) * 4);
  m.th = std::thread([this] {
    pthread_setname_np(pthread_self(), "wdr-dtwq");
    run();
  });
}

DtwQueue::~DtwQueue() {
  {
    std::lock_guard<std::mutex> g(m_->mu);
    m_->stop = true;
  }
  m_->cv.notify_all();
  if (m_->th.joinable()) m_->th.join();
  if (m_->s) {
    (void)hipStreamSynchronize(m_->s);
    (void)hipStreamDestroy(m_->s);
  }
}

void DtwQueue::submit(const std::shared_ptr<DtwQJob>& j) {
  WDR_CHECK((int)j->toks.size() >= 1 && (int)j->toks.size() <= RMAX && j->xkv && j->blk && j->done,
            "DTW queue: bad job");
  {
    std::lock_guard<std::mutex> g(m_->mu);
    j->t_submit = now_s();
    m_->pend.push_back(j);
    m_->pend_rows += (int)j->toks.size();
    jobs++;
  }
  m_->cv.notify_all();
}

bool DtwQueue::is_issued(const std::shared_ptr<DtwQJob>& j) {
  std::lock_guard<std::mutex> g(m_->mu);
  return j->issued;
}

void DtwQueue::wait_issued(const std::shared_ptr<DtwQJob>& j) {
  Impl& m = *m_;
  std::unique_lock<std::mutex> lk(m.mu);
  if (!j->issued) {
    m.urgent++;
    m.cv.notify_all();
    m.cv.wait(lk, [&] { return j->issued; });
    m.urgent--;
  }
  // only the failure of the pass that carried this job (or of the worker's start) reaches it
  if (j->err) std::rethrow_exception(j->err);
  if (m.err) std::rethrow_exception(m.err);
}

void DtwQueue::run() {
  Impl& m = *m_;
  try {
    WDR_HIP(hipSetDevice(ctx_.cp.gpu_device));
  } catch (...) {
    std::lock_guard<std::mutex> g(m.mu);
    m.err = std::current_exception();
  }
  std::unique_lock<std::mutex> lk(m.mu);
  while (true) {
    auto ready = [&] {
      return !m.pend.empty() && (m.stop || m.urgent > 0 || m.pend_rows >= m.min_rows ||
                                 now_s() - m.pend.front()->t_submit >= m.max_age);
    };
    m.cv.wait_for(lk, std::chrono::milliseconds(2), [&] { return ready() || (m.stop && m.pend.empty()); });
    if (m.pend.empty()) {
      if (m.stop) break;
      continue;
    }
    if (!ready()) continue;
    // oldest first, one job per DTW sequence (chain), within the pass's row capacity
    std::vector<std::shared_ptr<DtwQJob>> batch;
    std::set<int> seqs;
    int rows = 0;
    for (auto it = m.pend.begin(); it != m.pend.end();) {
      const int n = (int)(*it)->toks.size();
      if (seqs.count((*it)->seq) || rows + n > m.RB) {
        ++it;
        continue;
      }
      seqs.insert((*it)->seq);
      rows += n;
      batch.push_back(*it);
      it = m.pend.erase(it);
    }
    m.pend_rows -= rows;
    lk.unlock();
    std::exception_ptr e = m.err;
    if (!e) {
      try {
        issue(batch);
      } catch (...) {
        e = std::current_exception();
      }
    }
    lk.lock();
    for (auto& j : batch) {
      j->err = e;   // scoped to this pass: later passes (and later runs) start clean
      j->issued = true;
    }
    m.cv.notify_all();
  }
}

void DtwQueue::issue(std::vector<std::shared_ptr<DtwQJob>>& batch) {
  Impl& m = *m_;
  RowBatch& tb = *m.tb;
  tb.clear();
  size_t off = 0;
  for (auto& j : batch) {
    RowGroupDesc g;
    g.n = (int)j->toks.size();
    g.tok = j->toks.data();
    g.seq0 = j->seq;
    g.xkv = j->xkv;
    g.cap = m.cap.as<float>() + off;
    g.l_end = m.l_end;
    tb.add(g);
    j->cap_off = off;
    off += (size_t)m.A * g.n * 1500;
  }
  RowsIO io = m.bufs.io(ctx_, ctx_.model.hp.n_vocab);
  tb.upload(io, m.s, true, true);
  dtw_rows_forward(ctx_, io, tb.R, m.l_end, m.s);
  for (auto& j : batch) WDR_HIP(hipEventRecord(j->fwd, m.s));
  for (auto& j : batch) {
    launch_dtw(m.cap.as<float>() + j->cap_off, m.A, (int)j->toks.size(), 1500, j->n_audio, j->sot_len, j->seek,
               m.nrm.as<float>(), m.xdtw.as<float>(), m.times.as<int>(), m.times.as<int>() + RMAX + 4, m.s);
    WDR_HIP(wdr_memcpy_async(j->blk + 3 * RMAX, m.times.p, (RMAX + 8) * 4, hipMemcpyDeviceToHost, m.s));
    WDR_HIP(hipEventRecord(j->done, m.s));
  }
  passes++;
  rows += tb.R;
}

}  // namespace wdr
