// libwdr C ABI (include/wdr.h): Engine, the seam calls, and the reference crate's own
// Rust glue restated in C++:
//   src/audio.rs:4-24            read_wav (hound checks, verbatim messages)
//   src/vad.rs:33-84             cs -> s mask, sort, merge gaps < 200 ms, sample slicing
//   src/transcribe.rs:20-87      setup_params
//   src/transcribe.rs:171-320    token text cleanup + DTW-midpoint word bounds
//   src/transcribe.rs:323-535    run_transcription_pipeline (prompt chain, offsets, clipping,
//                                callbacks in reference order)
//   src/engine.rs:65-200         transcribe_audio (segmentation choice, context, pipeline)
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <sys/stat.h>
#include <dirent.h>
#include <condition_variable>
#include <exception>
#include <mutex>
#include <set>
#include <pthread.h>
#include <thread>
#include <vector>

#include "../../include/wdr.h"
#include "diarize.h"
#include "formatting.h"
#include "vad.h"
#include "whisper.h"
#include "ggml_file.h"
#include "model_files.h"
#include "prof.h"

using namespace wdr;

static thread_local std::string g_err;

static int fail(const std::string& m) {
  g_err = m;
  return -1;
}

#define WDR_GUARD(...)                          \
  try {                                         \
    __VA_ARGS__                                 \
  } catch (const std::exception& ex) {          \
    return fail(ex.what());                     \
  } catch (...) {                               \
    return fail("unknown error");               \
  }

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ------------------------------------------------------------------ text helpers (Rust semantics)
// Rust char::is_whitespace over UTF-8: ASCII whitespace + the Unicode White_Space code points.
static size_t ws_len(const std::string& s, size_t i) {
  const unsigned char c = s[i];
  if (c == ' ' || (c >= 0x09 && c <= 0x0D)) return 1;
  if (c == 0xC2 && i + 1 < s.size() && ((unsigned char)s[i + 1] == 0x85 || (unsigned char)s[i + 1] == 0xA0)) return 2;
  if (c == 0xE1 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x9A && (unsigned char)s[i + 2] == 0x80) return 3;
  if (c == 0xE2 && i + 2 < s.size()) {
    const unsigned char b = s[i + 1], d = s[i + 2];
    if (b == 0x80 && ((d >= 0x80 && d <= 0x8A) || d == 0xA8 || d == 0xA9 || d == 0xAF)) return 3;
    if (b == 0x81 && d == 0x9F) return 3;
  }
  if (c == 0xE3 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 && (unsigned char)s[i + 2] == 0x80) return 3;
  return 0;
}
static size_t utf8_len(unsigned char c) { return c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : 4; }

static std::string trim_start(const std::string& s) {
  size_t i = 0;
  while (i < s.size()) {
    const size_t w = ws_len(s, i);
    if (!w) break;
    i += w;
  }
  return s.substr(i);
}
static bool is_ws_end(const std::string& s, size_t end, size_t* w) {   // whitespace code point ending at `end`
  for (size_t k = 1; k <= 3 && k <= end; ++k) {
    const size_t st = end - k;
    if (utf8_len((unsigned char)s[st]) == k || (k == 1 && (unsigned char)s[st] < 0x80)) {
      if (ws_len(s, st) == k) { *w = k; return true; }
    }
  }
  return false;
}
static std::string trim(const std::string& s) {
  std::string t = trim_start(s);
  size_t e = t.size(), w;
  while (e > 0 && is_ws_end(t, e, &w)) e -= w;
  return t.substr(0, e);
}
static std::string trim_nul_then_ws(const std::string& s) {   // s.trim_matches('\0').trim()
  size_t a = 0, b = s.size();
  while (a < b && s[a] == '\0') ++a;
  while (b > a && s[b - 1] == '\0') --b;
  return trim(s.substr(a, b - a));
}

// src/transcribe.rs:205-212
static bool is_whole_control_token(const std::string& s) {
  const std::string t = trim_nul_then_ws(s);
  if (!(t.size() >= 2 && t.compare(0, 2, "[_") == 0 && t.back() == ']')) return false;
  if (t.size() < 3) return false;
  const std::string inner = t.substr(2, t.size() - 3);
  if (inner.empty()) return false;
  for (unsigned char c : inner)
    if (!((c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_')) return false;
  return true;
}

// src/transcribe.rs:215-240
static std::string strip_embedded_control_markers(const std::string& s) {
  std::string r;
  size_t i = 0;
  while (i < s.size()) {
    if (i + 1 < s.size() && s[i] == '[' && s[i + 1] == '_') {
      size_t j = i + 2;
      while (j < s.size() && s[j] != ']') ++j;
      if (j < s.size() && is_whole_control_token(s.substr(i, j - i + 1))) {
        i = j + 1;
        continue;
      }
    }
    r.push_back(s[i]);
    ++i;
  }
  return r;
}

struct Word {
  std::string text;
  double start, end;
  bool has_p;
  float p;
};
struct Seg {
  double start, end;
  std::string text;
  std::vector<Word> words;
  bool has_words = false;
  bool has_speaker = false;
  std::string speaker;
  int64_t src = -1;   // input SpeechSegment index (run_pipeline)
};

static double cs_to_s(long long cs) { return (double)cs * 0.01; }

// src/transcribe.rs:242-320
static std::vector<Word> get_token_timestamps(const ResultSeg& seg, const Vocab& v) {
  struct Tok {
    std::string text;
    float p;
    double t0, t1;
    bool has_a;
    double a;
  };
  std::vector<Tok> toks;
  for (const auto& t : seg.tokens) {
    const std::string& raw = v.id_to_token[t.id];
    if (is_whole_control_token(raw)) continue;
    std::string clean = strip_embedded_control_markers(raw);
    if (trim_nul_then_ws(clean).empty()) continue;
    toks.push_back({clean, t.p, cs_to_s(t.t0), cs_to_s(t.t1), t.t_dtw >= 0, t.t_dtw >= 0 ? cs_to_s(t.t_dtw) : 0.0});
  }
  std::vector<Word> out;
  for (size_t i = 0; i < toks.size(); ++i) {
    const bool hp = i > 0 && toks[i - 1].has_a, hh = toks[i].has_a, hn = i + 1 < toks.size() && toks[i + 1].has_a;
    const double start = (hp && hh) ? 0.5 * (toks[i - 1].a + toks[i].a) : toks[i].t0;
    const double end = (hh && hn) ? 0.5 * (toks[i].a + toks[i + 1].a) : toks[i].t1;
    out.push_back({toks[i].text, start, end, true, toks[i].p});
  }
  return out;
}

// src/transcribe.rs:171-203 (alphanumeric count: ASCII alnum + every non-ASCII code point)
static std::vector<Word> interpolate_word_timestamps(const std::string& line, double start, double end) {
  std::vector<Word> out;
  const double dur = std::max(end - start, 0.0);
  if (dur <= 0.0) return out;
  std::vector<std::string> toks;
  size_t i = 0;
  while (i < line.size()) {
    size_t w = ws_len(line, i);
    if (w) { i += w; continue; }
    size_t j = i;
    while (j < line.size() && !ws_len(line, j)) j += utf8_len((unsigned char)line[j]);
    std::string t = line.substr(i, j - i);
    if (!trim_nul_then_ws(t).empty()) toks.push_back(t);
    i = j;
  }
  if (toks.empty()) return out;
  std::vector<size_t> wts;
  size_t tot = 0;
  for (auto& t : toks) {
    size_t c = 0;
    for (size_t k = 0; k < t.size(); k += utf8_len((unsigned char)t[k])) {
      const unsigned char ch = t[k];
      if (ch >= 0x80 || std::isalnum(ch)) ++c;
    }
    wts.push_back(std::max<size_t>(c, 1));
    tot += wts.back();
  }
  size_t acc = 0;
  for (size_t k = 0; k < toks.size(); ++k) {
    const double t0 = start + ((double)acc / tot) * dur;
    const double t1 = k + 1 == toks.size() ? end : start + ((double)(acc + wts[k]) / tot) * dur;
    acc += wts[k];
    out.push_back({toks[k], t0, t1, false, 0.f});
  }
  return out;
}

// ------------------------------------------------------------------ ABI objects
struct wdr_context {
  std::unique_ptr<Context> ctx;
  std::unique_ptr<State> st;
  // gpu_device None (src/engine.rs:14): every visible GPU.  peers[g - 1] is the
  // model on device devices[g]; decode chain k runs on GPU k % G (chain k / G of its pool)
  std::vector<int> devices;
  std::vector<std::unique_ptr<Context>> peers;
  std::map<int, std::unique_ptr<State>> chain_st; // decode chains 1.. (multi-chain pipeline)
  int chains = 1;                                 // decode chains per GPU and run_pipeline call
  // early prompt fix-up: 0 off, 1 when the predecessor chain has already finished, 2 always (a
  // chain waits for its predecessor to finish: test seam), 3 from the prompt the predecessor's
  // speculative pass left (a chain waits for that pass, not for the predecessor's own fix-up; the
  // default: WDR_EARLY_FIXUP=0..3 picks another)
  int early_fixup = -1;
  struct ChainStats {
    long long chains = 1, launches = 0, rows = 0, fixups = 0, replays = 0, early = 0;
    long long prefill_rows = 0, dtw_rows = 0, prefills = 0, dtws = 0, mixed = 0, vgroups = 0, tiles = 0;
    long long dq_passes = 0, dq_rows = 0, dq_jobs = 0;   // DTW queue
    double spec_s = 0, fixup_s = 0, step_s = 0;
  } cs;                                           // the last run_pipeline's multi-chain figures
  hipStream_t low_dummy = nullptr;  // WDR_LOWQ_AT_PIPE (A/B, run_pipeline)
  std::unique_ptr<CamModel> cam;   // EmbeddingExtractor, created on the first diarized run
  std::string cam_path;            // ... from this embedding model file ("" = synthetic weights)
  double load_s = 0;
  double embed_s = 0;              // wall time the decode chain waited on speaker embeddings
  ~wdr_context() {
    if (low_dummy) (void)hipStreamDestroy(low_dummy);
  }
};

// Speaker embeddings of every speech segment, computed in segment order on a host worker
// thread that drives CamModel's own low-priority stream, concurrently with the decode chain
// (an embedding depends on the segment's PCM only, src/transcribe.rs:466).  finalize() of
// segment i blocks until embedding i is done; errors surface there.
class EmbedAhead {
 public:
  EmbedAhead(CamModel& cam, const std::vector<wdr_speech_segment>& segs)
      : emb_(segs.size() * 512), ok_(segs.size(), 0) {
    th_ = std::thread([this, &cam, &segs] {
      pthread_setname_np(pthread_self(), "wdr-embed");
      try {
        // batches of consecutive segments (CamModel::embed_batch: one forward over all their
        // frames); the first batch is small so that segment 0's embedding is ready early
        size_t i = 0;
        long long cap = 2000;
        while (i < segs.size() && !stop_) {
          std::vector<const int16_t*> p;
          std::vector<size_t> n;
          long long frames = 0;
          for (size_t j = i; j < segs.size() && (p.empty() || (frames < cap && p.size() < 64)); ++j) {
            p.push_back(segs[j].samples);
            n.push_back(segs[j].n_samples);
            frames += (long long)segs[j].n_samples / 160;
          }
          const int B = (int)p.size();
          std::vector<char> ok(B);
          cam.embed_batch(p.data(), n.data(), B, emb_.data() + i * 512, ok.data());
          std::lock_guard<std::mutex> g(mu_);
          for (int b = 0; b < B; ++b) ok_[i + b] = ok[b];
          i += B;
          done_ = i;
          cv_.notify_all();
          cap = 16000;
        }
      } catch (...) {
        std::lock_guard<std::mutex> g(mu_);
        err_ = std::current_exception();
        cv_.notify_all();
      }
    });
  }
  ~EmbedAhead() {
    stop_ = true;
    if (th_.joinable()) th_.join();
  }
  // embedding of segment i (nullptr where the reference's ORT call fails -> speaker "?")
  const float* get(size_t i) {
    std::unique_lock<std::mutex> g(mu_);
    cv_.wait(g, [&] { return done_ > i || err_; });
    if (done_ <= i && err_) std::rethrow_exception(err_);
    return ok_[i] ? emb_.data() + i * 512 : nullptr;
  }

 private:
  std::vector<float> emb_;
  std::vector<char> ok_;
  std::mutex mu_;
  std::condition_variable cv_;
  size_t done_ = 0;
  std::exception_ptr err_;
  std::atomic<bool> stop_{false};
  std::thread th_;
};

struct SynCfg {
  double weight_std = 0.02, emb_std = 0.02;
  float force_len_rate = 0.f;
  bool disable_fallback = false;
};
static SynCfg syn_of(const wdr_synthetic* s) {
  SynCfg c;
  if (s) {
    if (s->weight_std > 0) c.weight_std = s->weight_std;
    if (s->emb_std > 0) c.emb_std = s->emb_std;
    c.force_len_rate = s->force_len_rate;
    c.disable_fallback = s->disable_fallback != 0;
  }
  return c;
}

struct wdr_vad {
  std::unique_ptr<VadModel> m;
};

struct wdr_diarizer {
  int device = 0;
  std::string seg_path, emb_path;   // "" = synthetic seeded weights
  std::unique_ptr<SegModel> seg;
  std::unique_ptr<CamModel> cam;
  SegModel& S() {
    if (!seg) seg = std::make_unique<SegModel>(device, seg_path);
    return *seg;
  }
  CamModel& E() {
    if (!cam) cam = std::make_unique<CamModel>(device, emb_path);
    return *cam;
  }
};

struct wdr_speakers {
  std::unique_ptr<SpeakerManager> m;
};

// DiarizeOptions as Engine::transcribe_audio builds it (src/engine.rs:101-111): threshold
// default 0.5, max_speakers None / Some(0) -> usize::MAX
static wdr_diarize_options diarize_options(const wdr_transcribe_options* o, const char* seg_path,
                                           const char* emb_path) {
  wdr_diarize_options d{};
  d.segment_model_path = seg_path;
  d.embedding_model_path = emb_path;
  d.threshold = (o && o->advanced && o->advanced->has_diarize_threshold) ? o->advanced->diarize_threshold : 0.5f;
  d.max_speakers = (o && o->has_max_speakers && o->max_speakers != 0) ? o->max_speakers : UINT64_MAX;
  return d;
}

struct wdr_engine {
  wdr_engine_config cfg{};
  std::string cache_dir, vad_path, seg_path, emb_path;
  SynCfg syn;
  bool syn_set = false;   // wdr_engine_set_synthetic: models missing on disk run on seeded weights
  std::map<std::string, std::unique_ptr<wdr_context>> contexts;
  std::unique_ptr<VadModel> vad;
  std::string vad_loaded;   // model file the VAD was made from ("" = synthetic)
  std::unique_ptr<SegModel> seg;
  std::string seg_loaded;
};

// src/vad.rs:6-85 on top of the GPU VAD: probabilities -> whisper.cpp segments (cs) -> the
// crate's own merge/slice (same code as wdr_vad_merge).  Segments borrow `pcm`.
static void vad_get_segments(VadModel& vm, const int16_t* pcm, size_t n, std::vector<std::pair<double, double>>* mask,
                             std::vector<wdr_speech_segment>* segs) {
  const std::vector<float> pr = vm.probs(pcm, n);
  const std::vector<std::pair<float, float>> cs = vad_segments_from_probs(pr, VadParams());
  mask->clear();
  for (auto& c : cs) {
    const double a = (double)c.first / 100.0, b = (double)c.second / 100.0;
    if (b > a) mask->push_back({a, b});
  }
  std::stable_sort(mask->begin(), mask->end(), [](auto& x, auto& y) { return x.first < y.first; });
  std::vector<std::pair<double, double>> merged;
  for (auto& m : *mask) {
    if (!merged.empty() && m.first - merged.back().second < 0.200) merged.back().second = std::max(m.second, merged.back().second);
    else merged.push_back(m);
  }
  const float SR = 16000.0f, nf = (float)n;
  segs->clear();
  for (auto& m : merged) {
    const size_t si = (size_t)std::min(std::max(std::round((float)m.first * SR), 0.0f), nf);
    const size_t ei = (size_t)std::min(std::max(std::round((float)m.second * SR), 0.0f), nf);
    if (!(m.second > m.first) || !(ei > si)) continue;
    segs->push_back({m.first, m.second, pcm + si, ei - si});
  }
}

// src/transcribe.rs:20-87
static FullParams setup_params(const wdr_transcribe_options* o, const SynCfg& syn) {
  FullParams p;
  const wdr_advanced* a = o ? o->advanced : nullptr;
  int n = 5;
  if (a && a->has_best_of_or_beam_size) n = a->best_of_or_beam_size;
  n = std::max(1, n);
  p.greedy = a && a->sampling_strategy && std::string(a->sampling_strategy) == "greedy";
  p.best_of = n;
  p.beam_size = n;
  p.suppress_blank = true;
  p.token_timestamps = true;
  p.single_segment = true;
  if (o && o->lang) p.language = o->lang;
  if (o && o->whisper_to_english == 1) p.translate = true;
  if (a) {
    if (a->has_temperature) p.temperature = a->temperature;
    if (a->has_max_text_ctx) p.n_max_text_ctx = a->max_text_ctx;
    if (a->init_prompt) {
      p.initial_prompt = a->init_prompt;
      p.has_initial_prompt = true;
    }
  }
  p.force_len_rate = syn.force_len_rate;
  if (syn.disable_fallback) {
    p.logprob_thold = -INFINITY;
    p.entropy_thold = -1.f;
  }
  return p;
}

static bool file_exists(const char* p) {
  struct stat st;
  return p && stat(p, &st) == 0;
}

// A cached model file under the engine's cache dir, without network: <cache>/<file>, or the
// hf-hub layout the reference's model manager uses, <cache>/models--<owner>--<repo>/snapshots/
// <rev>/<file> (src/model_manager.rs:661-681).  Empty when absent.
static std::string find_cached_file(const std::string& cache_dir, const std::string& hub_dir, const std::string& file) {
  if (cache_dir.empty()) return std::string();
  const std::string direct = cache_dir + "/" + file;
  if (file_exists(direct.c_str())) return direct;
  const std::string snaps = cache_dir + "/" + hub_dir + "/snapshots";
  std::string found;
  if (DIR* d = opendir(snaps.c_str())) {
    std::vector<std::string> revs;
    while (dirent* ent = readdir(d))
      if (ent->d_name[0] != '.') revs.push_back(ent->d_name);
    closedir(d);
    std::sort(revs.begin(), revs.end());
    for (const std::string& r : revs) {
      const std::string c = snaps + "/" + r + "/" + file;
      if (file_exists(c.c_str())) {
        found = c;
        break;
      }
    }
  }
  return found;
}
// ggml-<model>.bin from ggerganov/whisper.cpp (src/model_manager.rs:148-162)
static std::string find_model_file(const std::string& cache_dir, const std::string& model) {
  return find_cached_file(cache_dir, "models--ggerganov--whisper.cpp", "ggml-" + model + ".bin");
}

// src/transcribe.rs:89-166.  model_path: a whisper.cpp ggml file (hparams, mel filters, vocabulary and weights from it;
// model_name then only selects the DTW alignment-head preset, src/transcribe.rs:117-129);
// empty: the named configuration with synthetic seeded weights
static std::unique_ptr<wdr_context> make_context(const std::string& model_name, bool has_dev, int dev, int8_t use_gpu,
                                                 int8_t enable_dtw, const SynCfg& syn,
                                                 const std::string& model_path = std::string()) {
  HParams hp;
  std::unique_ptr<GgmlFile> gf;
  if (!model_path.empty()) {
    gf = std::make_unique<GgmlFile>(model_path);
    const int32_t* h = gf->hp;
    hp.n_vocab = h[0]; hp.n_audio_ctx = h[1]; hp.n_audio_state = h[2]; hp.n_audio_head = h[3];
    hp.n_audio_layer = h[4]; hp.n_text_ctx = h[5]; hp.n_text_state = h[6]; hp.n_text_head = h[7];
    hp.n_text_layer = h[8]; hp.n_mels = h[9];
  } else if (!hparams_for(model_name, &hp)) {
    throw std::runtime_error("failed to open model: unknown model '" + model_name + "'");
  }
  ContextParams cp;
  if (use_gpu == 0) cp.use_gpu = false;
  if (has_dev) cp.gpu_device = dev;
  cp.dtw = enable_dtw == 1;
  cp.flash_attn = false;
  cp.weight_std = syn.weight_std;
  cp.emb_std = syn.emb_std;
  auto c = std::make_unique<wdr_context>();
  // the GPUs: the one named, or (None) every visible one -- WDR_DEVICES="0,0" lists them
  // explicitly (two models on one GPU exercise the multi-GPU path on a one-GPU machine)
  if (has_dev) {
    c->devices = {dev};
  } else if (const char* e = getenv("WDR_DEVICES")) {
    // validated here, not later as HIP errors: ordinals of visible GPUs, at most 8 entries
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) throw std::runtime_error("WDR_DEVICES: no visible GPU");
    for (const char* q = e; *q;) {
      char* end = nullptr;
      const long g = strtol(q, &end, 10);
      if (end == q || g < 0 || g >= n || (*end && *end != ','))
        throw std::runtime_error(std::string("WDR_DEVICES: bad device list '") + e + "' (" + std::to_string(n) +
                                 " visible GPUs)");
      if (c->devices.size() >= 8) throw std::runtime_error("WDR_DEVICES: at most 8 devices");
      c->devices.push_back((int)g);
      q = *end == ',' ? end + 1 : end;
    }
  } else {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) n = 1;
    for (int g = 0; g < std::min(n, 8); ++g) c->devices.push_back(g);
  }
  WDR_CHECK(!c->devices.empty(), "no GPU device");
  cp.gpu_device = c->devices[0];
  const double t = now_s();
  try {
    c->ctx = std::make_unique<Context>(model_name, hp, cp, gf.get());
    c->st = std::make_unique<State>(*c->ctx);
    for (size_t g = 1; g < c->devices.size(); ++g) {
      ContextParams pc = cp;
      pc.gpu_device = c->devices[g];
      c->peers.push_back(std::make_unique<Context>(model_name, hp, pc, gf.get()));
    }
    c->chains = c->ctx->max_chains;   // WDR_DECODE_CHAINS (default 40), wdr_context_set_chains
  } catch (const std::exception& ex) {
    throw std::runtime_error(std::string("create whisper context crash: ") + ex.what());
  }
  c->load_s = now_s() - t;
  return c;
}

struct CallbackCtx {
  const wdr_callbacks* cb;
};

// ---- formatting glue (src/engine.rs:192-199)
static void apply_overrides(PostProcessConfig& c, const wdr_formatting_overrides* ov) {
  if (!ov) return;
  if (ov->has_max_chars_per_line) c.max_chars_per_line = ov->max_chars_per_line;
  if (ov->has_max_lines) c.max_lines = ov->max_lines;
  if (ov->has_cps_cap) c.cps_cap = ov->cps_cap;
  if (ov->has_split_gap_sec) c.split_gap_sec = ov->split_gap_sec;
  if (ov->has_comma_min_chars_before_allow) c.comma_min_chars_before_allow = ov->comma_min_chars_before_allow;
  if (ov->has_min_word_dur) c.min_word_dur = ov->min_word_dur;
  if (ov->has_min_sub_dur) c.min_sub_dur = ov->min_sub_dur;
  if (ov->has_max_sub_dur) c.max_sub_dur = ov->max_sub_dur;
  if (ov->has_soft_max_words_per_line) c.soft_max_words_per_line = ov->soft_max_words_per_line;
  if (ov->insert_interword_space >= 0) c.insert_interword_space = ov->insert_interword_space != 0;
  if (ov->use_grapheme_len >= 0) c.use_grapheme_len = ov->use_grapheme_len != 0;
  if (ov->enforce_kinsoku >= 0) c.enforce_kinsoku = ov->enforce_kinsoku != 0;
  if (ov->allow_comma_split >= 0) c.allow_comma_split = ov->allow_comma_split != 0;
}

static std::vector<FmtSeg> to_fmt(const std::vector<Seg>& in) {
  std::vector<FmtSeg> out;
  for (const Seg& s : in) {
    FmtSeg f;
    f.start = s.start;
    f.end = s.end;
    f.text = s.text;
    f.has_words = s.has_words;
    for (const Word& w : s.words) f.words.push_back({w.text, w.start, w.end, w.has_p, w.p});
    f.has_speaker = s.has_speaker;
    f.speaker = s.speaker;
    out.push_back(std::move(f));
  }
  return out;
}

static std::vector<Seg> from_fmt(const std::vector<FmtSeg>& in) {
  std::vector<Seg> out;
  for (const FmtSeg& f : in) {
    Seg s;
    s.start = f.start;
    s.end = f.end;
    s.text = f.text;
    s.has_words = f.has_words;
    for (const FmtWord& w : f.words) {
      Word x;
      x.text = w.text;
      x.start = w.start;
      x.end = w.end;
      x.has_p = w.has_p;
      x.p = w.p;
      s.words.push_back(std::move(x));
    }
    s.has_speaker = f.has_speaker;
    s.speaker = f.speaker;
    out.push_back(std::move(s));
  }
  return out;
}

static wdr_segment_list* to_list(const std::vector<Seg>& segs, const std::string* lang) {
  auto* l = (wdr_segment_list*)calloc(1, sizeof(wdr_segment_list));
  l->n_segments = segs.size();
  l->segments = (wdr_segment*)calloc(std::max<size_t>(1, segs.size()), sizeof(wdr_segment));
  for (size_t i = 0; i < segs.size(); ++i) {
    wdr_segment& o = l->segments[i];
    o.start = segs[i].start;
    o.end = segs[i].end;
    o.text = strdup(segs[i].text.c_str());
    if (segs[i].has_words) {
      auto* w = (wdr_word*)calloc(std::max<size_t>(1, segs[i].words.size()), sizeof(wdr_word));
      for (size_t k = 0; k < segs[i].words.size(); ++k) {
        w[k].text = strdup(segs[i].words[k].text.c_str());
        w[k].start = segs[i].words[k].start;
        w[k].end = segs[i].words[k].end;
        w[k].has_probability = segs[i].words[k].has_p;
        w[k].probability = segs[i].words[k].p;
      }
      o.words = w;
      o.n_words = segs[i].words.size();
    }
    o.speaker_id = segs[i].has_speaker ? strdup(segs[i].speaker.c_str()) : nullptr;
  }
  l->detected_lang = lang ? strdup(lang->c_str()) : nullptr;
  if (!segs.empty() && segs[0].src >= 0) {
    auto* ix = (int64_t*)calloc(segs.size(), sizeof(int64_t));
    for (size_t i = 0; i < segs.size(); ++i) ix[i] = segs[i].src;
    l->speech_index = ix;
  }
  return l;
}

static void emit_segment(const wdr_callbacks* cb, const Seg& s) {
  if (!cb || !cb->new_segment) return;
  std::vector<wdr_word> w(s.words.size());
  for (size_t k = 0; k < s.words.size(); ++k)
    w[k] = {s.words[k].text.c_str(), s.words[k].start, s.words[k].end, (int8_t)s.words[k].has_p, s.words[k].p};
  wdr_segment o{s.start, s.end, s.text.c_str(), s.has_words ? w.data() : nullptr, s.has_words ? w.size() : 0,
                s.has_speaker ? s.speaker.c_str() : nullptr};
  cb->new_segment(cb->user, &o);
}

// ------------------------------------------------------------------ multi-chain decoding
// One segment's decode output (DTW resolved), and the prompt state of the reference's segment
// loop (src/transcribe.rs:384-386, 502): the prompt entering segment i+1 is the text of segment
// i's last result when that is non-empty, else the prompt segment i used.
struct SegOut {
  std::vector<ResultSeg> res;
  int lang_id = 0;
  bool lang_known = false;         // lang_id detected by the speculative pass (lang "auto")
  bool sampled = false;            // a t > 0 decoder drew random numbers
  bool rng_clean = true;           // decoded from decoder 0's initial RNG state (nothing drew before it)
  std::string rng_after;           // decoder 0's RNG right after this segment (when sampled)
};
struct Prompt {
  bool has = false;
  std::string text;
  bool operator==(const Prompt& o) const { return has == o.has && (!has || text == o.text); }
  bool operator!=(const Prompt& o) const { return !(*this == o); }
};
static Prompt next_prompt(const Prompt& e, const std::vector<ResultSeg>& res) {
  if (!res.empty()) {
    const std::string t = trim_start(res.back().text);
    if (!trim(t).empty()) return {true, t};
  }
  return e;
}
static FullParams with_prompt(const FullParams& base, const Prompt& e) {
  FullParams p = base;
  p.has_initial_prompt = e.has;
  p.initial_prompt = e.has ? e.text : std::string();
  return p;
}
static std::vector<float> seg_f32(const wdr_speech_segment& s) {
  std::vector<float> x(s.n_samples);
  for (size_t k = 0; k < s.n_samples; ++k) x[k] = (float)s.samples[k] / 32768.0f;
  return x;
}

// Decode every speech segment with C chains.  Chain c decodes the contiguous block
// [a_c, b_c) on its own State and host thread, speculatively from the pipeline's initial
// prompt; its greedy steps are batched with the other chains' (StepBatcher).  Then, in chain
// order, chain c's block is re-decoded segment by segment from the true incoming prompt
// until the prompt entering the next segment equals the speculative run's; from there on
// the speculative results ARE the sequential ones.  Random draws (t > 0 decoders) make a
// result depend on every earlier draw (decoder 0's RNG lives in the state): from the first
// segment that drew, the rest of the file is re-decoded sequentially from that segment's RNG
// state.  The output equals the single-chain loop's exactly.
// rng0: decoder 0's RNG entering the first segment (the fresh state's, or the state a previous
// block of the same file left, multi-GPU one-file path); "clean" below means "equal to rng0".
static std::vector<SegOut> decode_chains(wdr_context* c, const std::vector<wdr_speech_segment>& segs,
                                         const wdr_transcribe_options* o, const FullParams& params, int C,
                                         const wdr_callbacks* cb, const std::string& rng0) {
  const size_t N = segs.size();
  const int G = (int)c->devices.size();
  // chain k: GPU k % G, chain k / G of that GPU's KV pool (a fixed mapping, so states persist)
  auto ctx_of = [&](int k) -> Context& { return k % G == 0 ? *c->ctx : *c->peers[k % G - 1]; };
  for (int k = 1; k < C; ++k)
    if (!c->chain_st.count(k)) {
      WDR_HIP(hipSetDevice(c->devices[k % G]));
      c->chain_st[k] = std::make_unique<State>(ctx_of(k), k / G);
    }
  auto state = [&](int k) -> State& { return k == 0 ? *c->st : *c->chain_st.at(k); };
  auto on_gpu = [&](int k) { WDR_HIP(hipSetDevice(c->devices[k % G])); };
  const bool auto_lang = !o || !o->lang || std::string(o->lang).empty() || std::string(o->lang) == "auto";
  // contiguous blocks balanced by estimated decode cost (each chain at least one segment):
  // tokens grow with the segment's duration, plus a per-segment overhead (prompt prefill,
  // the SOT / timestamp / EOT steps, DTW re-forward) worth WDR_BALANCE_SEG_S seconds of audio
  // WDR_BALANCE_SKEW = s (default 0.08): chain k's share of the cost scaled by 1 + s (1 - 2k /
  // (C - 1)) -- the first encode batches are issued in chain order (below), so chain k starts
  // decoding about k batch-times after chain 0 (1-h bench: 0.03 ... 0.69 s over 40 chains) and,
  // one token per batched step like every chain, would end that much later on an equal share
  // (profiles/r05/ab_balance_skew.txt: 805.6 vs 790.0 (no skew) vs 775.7 xRT (neither) mean of 3;
  // with the skew the chains' ends show no trend in k)
  std::vector<size_t> cut(C + 1, 0);
  {
    static const double seg_s = getenv("WDR_BALANCE_SEG_S") ? atof(getenv("WDR_BALANCE_SEG_S")) : 0.0;
    static const double skew = getenv("WDR_BALANCE_SKEW") ? atof(getenv("WDR_BALANCE_SKEW")) : 0.08;
    std::vector<double> P(N + 1, 0.0);
    for (size_t i = 0; i < N; ++i) P[i + 1] = P[i] + (double)segs[i].n_samples + seg_s * 16000.0;
    std::vector<double> F(C + 1, 0.0);   // cumulative share of chains 0 .. k-1
    for (int k = 0; k < C; ++k) F[k + 1] = F[k] + 1.0 + (C > 1 ? skew * (1.0 - 2.0 * k / (C - 1)) : 0.0);
    for (int k = 1; k < C; ++k) {
      const double t = P[N] * F[k] / F[C];
      size_t x = std::lower_bound(P.begin(), P.end(), t) - P.begin();
      if (x > 0 && t - P[x - 1] <= P[std::min(x, N)] - t) --x;
      cut[k] = std::min(std::max(x, cut[k - 1] + 1), N - (size_t)(C - k));
    }
    cut[C] = N;
  }
  std::vector<SegOut> out(N);
  // spec_out[i]: the prompt leaving segment i in its chain's speculative run (every block
  // starts from the pipeline's initial prompt e0)
  std::vector<Prompt> spec_out(N);
  const Prompt e0{params.has_initial_prompt, params.initial_prompt};
  std::atomic<bool> stop{false};
  std::vector<std::exception_ptr> errs(C);
  c->cs.chains = C;
  auto batch_stats = [&]() {
    Context::BatchStats o;
    for (int g = 0; g < std::min(G, C); ++g) {
      const Context::BatchStats b = (g == 0 ? *c->ctx : *c->peers[g - 1]).batcher_stats();
      o.launches += b.launches;
      o.rows += b.rows;
      o.prefill_rows += b.prefill_rows;
      o.dtw_rows += b.dtw_rows;
      o.prefills += b.prefills;
      o.dtws += b.dtws;
      o.mixed += b.mixed;
      o.vgroups += b.vgroups;
      o.tiles += b.tiles;
      o.step_s = std::max(o.step_s, b.step_s);
      o.dq_passes += b.dq_passes;
      o.dq_rows += b.dq_rows;
      o.dq_jobs += b.dq_jobs;
    }
    return o;
  };
  const Context::BatchStats b0 = batch_stats();
  const double t_spec = now_s();
  // dec_in[k]: the prompt chain k's first segment was last decoded from
  std::vector<Prompt> dec_in(C, e0);
  std::atomic<long long> fixups{0}, early_n{0};
  // re-decode block k from prompt e, segment by segment, until the prompt leaving a segment
  // equals the one its successor was decoded from (used by the early and the round fix-ups)
  auto redo_block = [&](int k, const Prompt& e_in, bool batched, std::atomic<long long>* count) {
    on_gpu(k);
    State& st = state(k);
    const size_t a = cut[k], b = cut[k + 1];
    st.batched = batched;
    struct Guard {
      State& st;
      ~Guard() { st.batched = false; }
    } guard{st};
    Prompt e = e_in;
    struct Hint {
      State& st;
      ~Hint() { st.lang_hint = -1; }
    } hint{st};
    for (size_t j = a; j < b && !stop; ++j) {
      const std::vector<float> x = seg_f32(segs[j]);
      st.set_rng_state(rng0);
      // the speculative pass detected this segment's language from its window 0 alone: the
      // re-decode keeps it instead of a detection pass of its own
      // (WDR_LANG_HINT=0: detect again, A/B)
      static const bool hint_on = !(getenv("WDR_LANG_HINT") && atoi(getenv("WDR_LANG_HINT")) == 0);
      st.lang_hint = hint_on && out[j].lang_known ? out[j].lang_id : -1;
      if (st.full(with_prompt(params, e), x.data(), (int)x.size(), -1, false) != 0)
        throw std::runtime_error("failed to transcribe");
      out[j].res = st.result_all;
      out[j].lang_id = st.lang_id;
      out[j].sampled = st.sampled;
      out[j].rng_clean = true;   // rng0 above
      out[j].rng_after = st.sampled ? st.rng_state() : std::string();
      e = next_prompt(e, out[j].res);
      const bool converged = e == spec_out[j];
      spec_out[j] = e;
      (*count)++;
      if (converged) break;
    }
  };
  // planned[k]: chain k issued its first encode batch (st.plan).  The chains of one device issue
  // theirs in chain order -- chain k after chain k - G, its predecessor on the same GPU, whose
  // encode streams it shares (chain k runs on GPU k % G); chains on other devices do not wait
  std::unique_ptr<std::atomic<int>[]> planned(new std::atomic<int>[C]);
  for (int k = 0; k < C; ++k) planned[k] = 0;
  // done[k]: chain k finished its speculative block (and its early fix-up); spec_done[k]: its
  // speculative pass ended, spec_last[k] the prompt leaving the block then (under spec_mu: the
  // chain's own early fix-up may rewrite spec_out of its block meanwhile)
  std::unique_ptr<std::atomic<int>[]> done(new std::atomic<int>[C]);
  std::unique_ptr<std::atomic<int>[]> spec_done(new std::atomic<int>[C]);
  for (int k = 0; k < C; ++k) done[k] = spec_done[k] = 0;
  std::vector<Prompt> spec_last(C, e0);
  std::mutex spec_mu;
  auto worker = [&](int k) {
    State& st = state(k);
    try {
      on_gpu(k);
      const size_t a = cut[k], b = cut[k + 1];
      st.times = StageTimes{};
      st.set_rng_state(rng0);
      st.batched = C > 1;
      std::vector<const int16_t*> pcm;
      std::vector<int> ns;
      for (size_t i = a; i < b; ++i) {
        pcm.push_back(segs[i].samples);
        ns.push_back((int)segs[i].n_samples);
      }
      {
        // the first encode batches in chain order: the shared encode streams run them first-in
        // first-out, so chain k starts decoding about k batch-times in (WDR_BALANCE_SKEW)
        struct Turn {
          std::atomic<int>& t;
          ~Turn() { t.store(1); }
        } turn{planned[k]};
        while (k >= G && !planned[k - G].load() && !stop) std::this_thread::sleep_for(std::chrono::microseconds(20));
        st.plan(pcm.data(), ns.data(), (int)(b - a), auto_lang);
      }
      struct Guard {
        State& st;
        ~Guard() {
          st.batched = false;
          try {
            st.unplan();
          } catch (...) {
          }
        }
      } guard{st};
      Prompt e = e0;
      // the block's DTW tickets, resolved after its last segment: the re-forwards run batched
      // with the other chains' (DtwQueue) and nothing on the chain waits for them before that
      std::vector<std::pair<size_t, std::vector<DtwTicket>>> tks;
      struct Resolve {   // on an error too: return the tickets' blocks / events to the state
        State& st;
        std::vector<std::pair<size_t, std::vector<DtwTicket>>>& tks;
        std::vector<SegOut>& out;
        ~Resolve() {
          for (auto& p : tks)
            for (auto& t : p.second)
              if (t.blk) {
                try {
                  st.resolve_dtw(t, out[p.first].res);
                } catch (...) {
                }
              }
        }
      } resolve_guard{st, tks, out};
      bool drew = false;   // a segment of this block drew before: decoder 0's RNG is no longer initial
      for (size_t i = a; i < b && !stop; ++i) {
        if (st.full(with_prompt(params, e), nullptr, 0, (int)(i - a), true) != 0)
          throw std::runtime_error("failed to transcribe");
        out[i].res = st.result_all;
        out[i].lang_id = st.lang_id;
        out[i].lang_known = auto_lang;
        out[i].sampled = st.sampled;
        out[i].rng_clean = !drew;
        drew = drew || st.sampled;
        if (st.sampled) out[i].rng_after = st.rng_state();
        tks.emplace_back(i, st.take_dtw_jobs());
        e = next_prompt(e, out[i].res);
        spec_out[i] = e;
      }
      for (auto& p : tks)
        for (auto& t : p.second) st.resolve_dtw(t, out[p.first].res);
      std::lock_guard<std::mutex> g(spec_mu);
      spec_last[k] = e;
    } catch (...) {
      errs[k] = std::current_exception();
      stop = true;
    }
    spec_done[k] = 1;
    // early fix-up: if chain k-1 has already finished, the prompt leaving its block is known
    // now (as it stands) -- redo block k from it while the other chains' steps are still
    // running, its rows joining their batches instead of a fix-up round after them.  The
    // rounds below re-check it against the final prompt, so the result stays exact.
    // Mode 3 (default): a chain that finishes before its predecessor's speculative pass waits for
    // it (nothing else is left for it to do) and redoes from the prompt that pass left, instead of
    // idling until the rounds -- which start only after every chain is done and then run the
    // redone blocks as small batches at the end.  If the predecessor's own early fix-up later
    // changes that prompt, the rounds redo this block again: exact either way.
    try {
      static const int env_mode = getenv("WDR_EARLY_FIXUP") ? atoi(getenv("WDR_EARLY_FIXUP")) : 3;
      const int mode = c->early_fixup >= 0 ? c->early_fixup : env_mode;
      if (mode == 2 && k > 0)
        while (!done[k - 1].load() && !stop) std::this_thread::sleep_for(std::chrono::microseconds(200));
      if (mode == 3 && k > 0)
        while (!spec_done[k - 1].load() && !stop) std::this_thread::sleep_for(std::chrono::microseconds(200));
      if (mode > 0 && !errs[k] && !stop && k > 0 && (mode == 3 ? spec_done[k - 1].load() : done[k - 1].load())) {
        Prompt et;
        if (done[k - 1].load()) {
          et = spec_out[cut[k] - 1];   // the predecessor finished: its block no longer changes
        } else {
          std::lock_guard<std::mutex> g(spec_mu);
          et = spec_last[k - 1];
        }
        if (et != dec_in[k]) {
          redo_block(k, et, C > 1, &early_n);
          dec_in[k] = et;
        }
      }
    } catch (...) {
      errs[k] = std::current_exception();
      stop = true;
    }
    done[k] = 1;
  };
  {
    std::atomic<int> live{C};
    std::vector<std::thread> th;
    for (int k = 0; k < C; ++k)
      th.emplace_back([&, k] {
        pthread_setname_np(pthread_self(), "wdr-chain");
        worker(k);
        live--;
      });
    // cancellation is polled here: callbacks fire on the calling thread only
    while (live > 0) {
      if (!stop && cb && cb->is_cancelled && cb->is_cancelled(cb->user)) stop = true;
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
    for (auto& t : th) t.join();
    for (auto& e : errs)
      if (e) std::rethrow_exception(e);
    if (stop) throw std::runtime_error("failed to transcribe");
  }
  c->cs.spec_s = now_s() - t_spec;
  const double t_fix = now_s();
  // Fix-up rounds.  dec_in[k] is the prompt chain k's first segment was decoded from (e0 in
  // the speculative run); the true one is the prompt leaving block k-1 as it now stands.  Every
  // chain whose two differ re-decodes its block from the true prompt -- all such chains at once,
  // their greedy steps batched as in the speculative phase -- segment by segment until the
  // prompt leaving a segment equals the one its successor was decoded from.  A chain that ran
  // through its whole block changes its successor's true prompt: the next round redoes that
  // one.  Chain 0 is always exact, so every round fixes at least one more chain.  Each redone
  // segment starts from decoder 0's initial RNG state: no segment before it drew (or the
  // sampled tail below redoes it anyway).
  for (;;) {
    std::vector<int> redo;
    std::vector<Prompt> e_true(C);
    for (int k = 1; k < C; ++k) {
      e_true[k] = spec_out[cut[k] - 1];
      if (e_true[k] != dec_in[k]) redo.push_back(k);
    }
    if (redo.empty()) break;
    const bool batch = redo.size() > 1;
    auto fix = [&](int k) {
      try {
        redo_block(k, e_true[k], batch, &fixups);
      } catch (...) {
        errs[k] = std::current_exception();
        stop = true;
      }
    };
    std::atomic<int> live{(int)redo.size()};
    std::vector<std::thread> th;
    for (int k : redo)
      th.emplace_back([&, k] {
        pthread_setname_np(pthread_self(), "wdr-fixup");
        fix(k);
        live--;
      });
    while (live > 0) {
      if (!stop && cb && cb->is_cancelled && cb->is_cancelled(cb->user)) stop = true;
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    for (auto& t : th) t.join();
    for (auto& e : errs)
      if (e) std::rethrow_exception(e);
    if (stop) throw std::runtime_error("failed to transcribe");
    for (int k : redo) dec_in[k] = e_true[k];
  }
  c->cs.fixups = fixups + early_n;
  c->cs.early = early_n;
  // random draws: no segment before the first one (file order) that drew did draw, so in the
  // sequential loop it starts from decoder 0's initial RNG.  If its kept result was decoded from
  // that state it is exact and the re-decode starts after it (from its RNG state); if not (a
  // speculative segment before it in its block drew, and the fix-up stopped before redoing it),
  // the re-decode starts at it, from the initial state.  Every later segment is re-decoded in order.
  size_t f = N;
  for (size_t i = 0; i < N; ++i)
    if (out[i].sampled) {
      f = i;
      break;
    }
  const size_t rs = (f < N && !out[f].rng_clean) ? f : f + 1;
  if (rs < N) {
    on_gpu(0);
    State& st = *c->st;
    Prompt e = e0;
    for (size_t i = 0; i < rs; ++i) e = next_prompt(e, out[i].res);
    if (rs == f) st.set_rng_state(rng0);
    else st.set_rng_state(out[f].rng_after);
    for (size_t i = rs; i < N; ++i) {
      if (cb && cb->is_cancelled && cb->is_cancelled(cb->user)) throw std::runtime_error("failed to transcribe");
      const std::vector<float> x = seg_f32(segs[i]);
      c->cs.replays++;
      if (st.full(with_prompt(params, e), x.data(), (int)x.size(), -1, false) != 0)
        throw std::runtime_error("failed to transcribe");
      out[i].res = st.result_all;
      out[i].lang_id = st.lang_id;
      out[i].sampled = st.sampled;
      out[i].rng_after = st.sampled ? st.rng_state() : std::string();
      e = next_prompt(e, out[i].res);
    }
  }
  c->cs.fixup_s = now_s() - t_fix;
  {
    const Context::BatchStats b1 = batch_stats();
    c->cs.launches = b1.launches - b0.launches;
    c->cs.rows = b1.rows - b0.rows;
    c->cs.prefill_rows = b1.prefill_rows - b0.prefill_rows;
    c->cs.dtw_rows = b1.dtw_rows - b0.dtw_rows;
    c->cs.prefills = b1.prefills - b0.prefills;
    c->cs.dtws = b1.dtws - b0.dtws;
    c->cs.mixed = b1.mixed - b0.mixed;
    c->cs.vgroups = b1.vgroups - b0.vgroups;
    c->cs.tiles = b1.tiles - b0.tiles;
    c->cs.step_s = b1.step_s - b0.step_s;
    c->cs.dq_passes = b1.dq_passes - b0.dq_passes;
    c->cs.dq_rows = b1.dq_rows - b0.dq_rows;
    c->cs.dq_jobs = b1.dq_jobs - b0.dq_jobs;
  }
  // stage accounting: chains' times summed into the context's state
  for (int k = 1; k < C; ++k) {
    const StageTimes& t = state(k).times;
    StageTimes& m = c->st->times;
    m.mel += t.mel; m.encode += t.encode; m.decode += t.decode; m.dtw += t.dtw;
    m.windows += t.windows; m.decode_steps += t.decode_steps; m.prefills += t.prefills;
    m.lang += t.lang; m.prompt_gpu += t.prompt_gpu;
    m.lang_passes += t.lang_passes; m.lang_rows += t.lang_rows;
  }
  return out;
}

// src/transcribe.rs:323-535
// raw: per-segment results only (no overlap clip against the next segment, no speakers): the
// multi-GPU path (wdr/distributed.py) merges several GPUs' raw blocks and applies both in order.
// dopts: DiarizeOptions (src/transcribe.rs:327, 339-345); its presence switches speakers on.
// RNG carry (multi-GPU one-file path, wdr_run_pipeline_block): rng_in = decoder 0's RNG entering
// the first segment (null: the fresh state's, src/transcribe.rs:335); rng_out = its state after
// the last one; sampled[i] = segment i drew random numbers (t > 0 decoders)
struct RngCarry {
  const std::string* rng_in = nullptr;
  std::string rng_out;
  std::vector<char> sampled;
};
static std::vector<Seg> run_pipeline(wdr_context* c, const std::vector<wdr_speech_segment>& segs,
                                     const wdr_transcribe_options* o, const wdr_diarize_options* dopts,
                                     const SynCfg& syn, const wdr_callbacks* cb, std::string* detected_lang,
                                     bool* has_lang, bool raw = false, RngCarry* carry = nullptr) {
  const bool diarize = dopts != nullptr && !raw;
  const float dthr = dopts ? dopts->threshold : 0.5f;
  SpeakerManager speakers(dopts ? dopts->max_speakers : UINT64_MAX);
  if (diarize) {
    // EmbeddingExtractor::new(&diarize_options.embedding_model_path) (src/transcribe.rs:343)
    const std::string path = dopts->embedding_model_path ? dopts->embedding_model_path : "";
    if (!path.empty() && !file_exists(path.c_str())) throw std::runtime_error("embedding model file doesn't exist: " + path);
    if (!c->cam || c->cam_path != path) {
      c->cam.reset();
      c->cam = std::make_unique<CamModel>(c->ctx->cp.gpu_device, path);
      c->cam_path = path;
    }
  }
  static const bool lowq_at_pipe = !(getenv("WDR_LOWQ_AT_PIPE") && atoi(getenv("WDR_LOWQ_AT_PIPE")) == 0);
  if (!diarize && !c->low_dummy && lowq_at_pipe) {
    // WDR_LOWQ_AT_PIPE (default 1): an un-diarized pipeline gets a lowest-priority stream where the
    // embedding model's would be (before the decode chains' states on the first call), its
    // hardware queue instantiated by one memset.  It changes how the runtime spreads the states'
    // lowest-priority DTW streams over its 4 low queues; measured: configs[2]'s VAD line 632 ->
    // 737-740 xRT, the diarized line unaffected (it never takes this branch);
    // profiles/r06/ab_lines_hwq.txt, DESIGN.md §5 "Hardware queues, round 6"
    int lo = 0, hi = 0;
    WDR_HIP(hipSetDevice(c->devices[0]));
    WDR_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    WDR_HIP(hipStreamCreateWithPriority(&c->low_dummy, hipStreamNonBlocking, lo));
    DevMem one(16);
    WDR_HIP(hipMemsetAsync(one.p, 0, 16, c->low_dummy));
    WDR_HIP(hipStreamSynchronize(c->low_dummy));
  }
  std::unique_ptr<EmbedAhead> embeds;
  if (diarize) embeds = std::make_unique<EmbedAhead>(*c->cam, segs);
  // WDR_HOST_SPIN=N (diagnostic, A/B): N host threads spin for the duration of the call (does
  // keeping host cores awake change the batched steps' pace?)
  struct Spin {
    std::atomic<bool> stop{false};
    std::vector<std::thread> th;
    ~Spin() {
      stop = true;
      for (auto& t : th) t.join();
    }
  } spin;
  if (const char* e = getenv("WDR_HOST_SPIN"))
    for (int i = 0; i < std::max(0, std::min(8, atoi(e))); ++i)
      spin.th.emplace_back([&spin] {
        while (!spin.stop.load(std::memory_order_relaxed)) __builtin_ia32_pause();
      });
  FullParams params = setup_params(o, syn);
  const Vocab& v = c->ctx->vocab;
  const double user_offset = (o && o->has_offset) ? o->offset : 0.0;
  std::vector<Seg> out;
  bool have_prev = false;
  std::string previous_text;
  *has_lang = false;
  if (o && o->lang && std::string(o->lang) != "auto") {
    *detected_lang = o->lang;
    *has_lang = true;
  }
  const bool translated = o && o->whisper_to_english == 1;
  // decode chains: greedy and beam search at t = 0 (their steps batch across chains; t > 0
  // decoders from the first window on keep one chain)
  const int C = (params.temperature <= 0.f)
                    ? std::max(1, std::min({c->chains * (int)c->devices.size(),
                                            c->ctx->max_chains * (int)c->devices.size(), (int)segs.size()}))
                    : 1;
  WDR_HIP(hipSetDevice(c->devices[0]));
  // every segment's PCM goes to the encode-ahead ring up front (int16 -> f32 on the GPU,
  // the same x / 32768 as src/transcribe.rs's conversion); multi-chain: per chain block
  // the reference creates a fresh whisper state per pipeline call (src/transcribe.rs:335):
  // decoder 0's RNG starts from its initial seed (or from the state carried in)
  c->st->reset_rng();
  if (carry && carry->rng_in) c->st->set_rng_state(*carry->rng_in);
  const std::string rng0 = c->st->rng_state();
  if (carry) carry->sampled.assign(segs.size(), 0);
  if (C == 1) {
    std::vector<const int16_t*> pcm(segs.size());
    std::vector<int> ns(segs.size());
    for (size_t i = 0; i < segs.size(); ++i) {
      WDR_CHECK(segs[i].n_samples < (size_t)INT32_MAX, "speech segment too long");
      pcm[i] = segs[i].samples;
      ns[i] = (int)segs[i].n_samples;
    }
    const bool auto_lang = !o || !o->lang || std::string(o->lang).empty() || std::string(o->lang) == "auto";
    c->st->plan(pcm.data(), ns.data(), (int)segs.size(), auto_lang);
  }
  struct Unplan {
    State& st;
    ~Unplan() {
      try {
        st.unplan();
      } catch (...) {
      }
    }
  } unplan_guard{*c->st};
  // One-segment lag: segment i's DTW re-forwards run on the DTW stream while segment i+1
  // decodes; segment i is then finished (word times, speakers, callbacks in order).  The
  // prompt chain only needs segment i's text, which full() returns at once.
  struct Pending {
    size_t i = 0;
    std::vector<ResultSeg> res;
    std::vector<DtwTicket> tk;
  };
  std::vector<Pending> pend;
  struct Drain {   // on an error, return any in-flight DTW jobs to the state's pools
    wdr_context* c;
    std::vector<Pending>& p;
    ~Drain() {
      for (auto& q : p)
        for (auto& t : q.tk)
          if (t.blk) {
            try {
              c->st->resolve_dtw(t, q.res);
            } catch (...) {
            }
          }
    }
  } drain{c, pend};
  auto finalize = [&](Pending& P) {
    for (auto& t : P.tk) c->st->resolve_dtw(t, P.res);
    P.tk.clear();
    const size_t i = P.i;
    const wdr_speech_segment& ss = segs[i];
    const double base_offset = ss.start + user_offset;
    const float* emb = nullptr;
    bool have_emb = false;
    for (const ResultSeg& r : P.res) {
      std::string text = trim_start(r.text);
      const double approx_start = base_offset + cs_to_s(r.t0);
      const double approx_end = base_offset + cs_to_s(r.t1);
      std::vector<Word> words;
      if (translated) {
        words = interpolate_word_timestamps(text, approx_start, approx_end);
      } else {
        words = get_token_timestamps(r, v);
        for (auto& w : words) {
          w.start += base_offset;
          w.end += base_offset;
        }
      }
      const double seg_start = words.empty() ? approx_start : words.front().start;
      const double seg_end = words.empty() ? approx_end : words.back().end;
      if (!out.empty() && !raw) {
        Seg& last = out.back();
        if (last.end > seg_start) last.end = seg_start;
        if (last.has_words && !last.words.empty() && last.words.back().end > last.end) last.words.back().end = last.end;
      }
      Seg s;
      s.start = seg_start;
      s.end = seg_end;
      s.text = text;
      s.has_words = !words.empty();
      s.words = std::move(words);
      s.src = (int64_t)i;
      if (diarize) {
        // src/transcribe.rs:461-497: embed the whole speech segment (recomputed per whisper
        // segment in the reference; identical input -> computed once here), then assign
        if (!have_emb) {
          const double te = now_s();
          emb = embeds->get(i);
          c->embed_s += now_s() - te;
          have_emb = true;
        }
        s.has_speaker = true;
        s.speaker = speakers.assign(emb, 512, dthr);
      }
      emit_segment(cb, s);
      if (cb && cb->progress) {
        const int pct = (int)((double)(i + 1) / (double)segs.size() * 100.0);
        cb->progress(cb->user, pct, 1, "Transcribing audio");
      }
      out.push_back(std::move(s));
    }
  };
  if (C > 1) {
    // multi-chain: C States decode C contiguous blocks concurrently (batched greedy steps),
    // then the exact prompt fix-up; results come back DTW-resolved, finished here in order
    std::vector<SegOut> res = decode_chains(c, segs, o, params, C, cb, rng0);
    if (carry) {
      carry->rng_out = rng0;
      for (size_t i = 0; i < segs.size(); ++i) {
        carry->sampled[i] = res[i].sampled;
        if (res[i].sampled) carry->rng_out = res[i].rng_after;
      }
    }
    for (size_t i = 0; i < segs.size(); ++i) {
      if (i == 0 && !*has_lang) {
        *detected_lang = kLangs[std::max(0, std::min(99, res[0].lang_id))];
        *has_lang = true;
      }
      Pending P;
      P.i = i;
      P.res = std::move(res[i].res);
      finalize(P);
    }
    return out;
  }
  for (size_t i = 0; i < segs.size(); ++i) {
    if (have_prev) {
      params.initial_prompt = previous_text;
      params.has_initial_prompt = true;
    }
    if (cb && cb->is_cancelled && cb->is_cancelled(cb->user)) throw std::runtime_error("failed to transcribe");
    int rc;
    try {
      rc = c->st->full(params, nullptr, 0, (int)i, /*async_dtw=*/true);
    } catch (const std::exception& ex) {
      throw std::runtime_error(std::string("failed to transcribe: ") + ex.what());
    }
    if (rc != 0) throw std::runtime_error("failed to transcribe");
    if (carry) carry->sampled[i] = c->st->sampled;
    if (!*has_lang) {
      *detected_lang = kLangs[std::max(0, std::min(99, c->st->lang_id))];
      *has_lang = true;
    }
    Pending cur;
    cur.i = i;
    cur.res = c->st->result_all;
    cur.tk = c->st->take_dtw_jobs();
    for (const ResultSeg& r : cur.res) {   // src/transcribe.rs:502 prompt chain
      const std::string text = trim_start(r.text);
      have_prev = !trim(text).empty();
      if (have_prev) previous_text = text;
    }
    if (!pend.empty()) {
      finalize(pend[0]);
      pend.clear();
    }
    pend.push_back(std::move(cur));
  }
  if (!pend.empty()) {
    finalize(pend[0]);
    pend.clear();
  }
  if (carry) carry->rng_out = c->st->rng_state();
  return out;
}

// ------------------------------------------------------------------ read_wav (src/audio.rs:4-24)
static std::vector<int16_t> read_wav_impl(const char* path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("failed to read file");
  std::vector<char> data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  auto u32 = [&](size_t o) { uint32_t v; memcpy(&v, &data[o], 4); return v; };
  auto u16 = [&](size_t o) { uint16_t v; memcpy(&v, &data[o], 2); return v; };
  if (data.size() < 12 || memcmp(&data[0], "RIFF", 4) || memcmp(&data[8], "WAVE", 4))
    throw std::runtime_error("failed to read file");
  size_t pos = 12;
  bool have_fmt = false, have_data = false;
  uint16_t tag = 0, ch = 0, bits = 0;
  uint32_t rate = 0;
  size_t dpos = 0, dlen = 0;
  while (pos + 8 <= data.size()) {
    const uint32_t sz = u32(pos + 4);
    if (!memcmp(&data[pos], "fmt ", 4) && pos + 8 + 16 <= data.size()) {
      tag = u16(pos + 8); ch = u16(pos + 10); rate = u32(pos + 12); bits = u16(pos + 22);
      have_fmt = true;
    } else if (!memcmp(&data[pos], "data", 4)) {
      dpos = pos + 8;
      dlen = std::min<size_t>(sz, data.size() - dpos);
      have_data = true;
    }
    pos += 8 + (size_t)sz + (sz & 1);
  }
  if (!have_fmt || !have_data) throw std::runtime_error("failed to read file");
  if (ch != 1) throw std::runtime_error("expected mono audio file and found " + std::to_string(ch) + " channels!");
  if (!(tag == 1 || tag == 0xFFFE)) throw std::runtime_error("expected integer sample format");
  if (rate != 16000) throw std::runtime_error("expected 16KHz sample rate");
  if (bits != 16) throw std::runtime_error("expected 16 bits per sample");
  std::vector<int16_t> out(dlen / 2);
  if (!out.empty()) memcpy(out.data(), &data[dpos], out.size() * 2);
  return out;
}

// ------------------------------------------------------------------ ABI
static int diar_segments_out(const std::vector<DiarSegment>& ds, const int16_t* samples, size_t n,
                             wdr_speech_segment** segs_out, size_t* n_segs) {
  {
    size_t tot = 0;
    for (auto& x : ds) tot += x.end_idx - x.start_idx;
    // one allocation: the segment array followed by copies of their (zero-padded) samples
    const size_t head = std::max<size_t>(1, ds.size()) * sizeof(wdr_speech_segment);
    char* blk = (char*)malloc(head + std::max<size_t>(1, tot) * 2);
    wdr_speech_segment* sg = (wdr_speech_segment*)blk;
    int16_t* dst = (int16_t*)(blk + head);
    for (size_t i = 0; i < ds.size(); ++i) {
      const size_t len = ds[i].end_idx - ds[i].start_idx;
      for (size_t k = 0; k < len; ++k) {
        const size_t src = ds[i].start_idx + k;
        dst[k] = src < n ? samples[src] : 0;
      }
      sg[i] = {ds[i].start, ds[i].end, dst, len};
      dst += len;
    }
    *segs_out = sg;
    *n_segs = ds.size();
    return 0;
  }
}

// ------------------------------------------------------------------ live handles and teardown
// Every handle libwdr hands out is registered until it is freed, so that wdr_shutdown (and the
// process-exit hook below) can release what the host left alive -- contexts with their worker
// threads (DTW queue, encode-ahead, step batchers), streams, device memory -- while the HIP
// runtime is still up.  A free of a handle that is no longer registered (freed already, or
// released by wdr_shutdown) does nothing.
// Calls in flight: every entry point that takes a handle holds it (InUse) for the call's
// duration; wdr_shutdown releases only handles no call holds -- a host thread still inside
// wdr_run_pipeline when exit() runs the hook keeps its context -- and releases a handle by
// destroying its contents in place without returning the allocation, so a later handle can never
// reuse the address of a released one and a stale free of it stays a no-op.
namespace {
struct Live {
  std::mutex mu;
  std::set<void*> eng, ctx, vad, dia, spk;
  std::map<const void*, int> busy;   // handle -> entry-point calls in flight
};
Live& live() {
  static Live* l = new Live();   // never destroyed: the exit hook and late frees may run after statics
  return *l;
}
// an entry point's hold on a handle; a handle that is not (or no longer) registered is an error
struct InUse {
  const void* p = nullptr;
  InUse(std::set<void*> Live::*set, const void* h) {
    if (!h) throw std::runtime_error("null handle");
    std::lock_guard<std::mutex> g(live().mu);
    if (!(live().*set).count(const_cast<void*>(h))) throw std::runtime_error("handle was freed or released by wdr_shutdown");
    ++live().busy[h];
    p = h;
  }
  ~InUse() {
    if (!p) return;
    std::lock_guard<std::mutex> g(live().mu);
    auto it = live().busy.find(p);
    if (it != live().busy.end() && --it->second == 0) live().busy.erase(it);
  }
  InUse(const InUse&) = delete;
  InUse& operator=(const InUse&) = delete;
};
#define WDR_USE(SET, H) InUse wdr_in_use_(&Live::SET, (H))
void wdr_exit_hook() { wdr_shutdown(); }
template <typename T>
T* track(std::set<void*> Live::*set, T* p) {
  static std::once_flag once;
  // registered after the HIP runtime has initialised (its first handle needs it): exit runs this
  // hook before the runtime's own teardown (handlers run in reverse order of registration)
  std::call_once(once, [] { std::atexit(wdr_exit_hook); });
  std::lock_guard<std::mutex> g(live().mu);
  (live().*set).insert(p);
  return p;
}
template <typename T>
bool untrack(std::set<void*> Live::*set, T* p) {
  if (!p) return false;
  std::lock_guard<std::mutex> g(live().mu);
  return (live().*set).erase(p) > 0;
}
}  // namespace

extern "C" {

void wdr_shutdown(void) {
  std::set<void*> eng, ctx, vad, dia, spk;
  bool any_busy = false;
  {
    std::lock_guard<std::mutex> g(live().mu);
    Live& L = live();
    // take the handles no call holds; a held one stays registered (its owner frees it later)
    auto take = [&](std::set<void*>& from, std::set<void*>& to) {
      for (auto it = from.begin(); it != from.end();) {
        if (L.busy.count(*it)) {
          any_busy = true;
          ++it;
        } else {
          to.insert(*it);
          it = from.erase(it);
        }
      }
    };
    take(L.eng, eng);
    take(L.ctx, ctx);
    take(L.vad, vad);
    take(L.dia, dia);
    take(L.spk, spk);
  }
  // engines own their cached contexts; contexts join their threads and free their device memory.
  // Destroyed in place, the allocation kept: no later handle reuses a released address.
  for (void* p : eng) ((wdr_engine*)p)->~wdr_engine();
  for (void* p : ctx) ((wdr_context*)p)->~wdr_context();
  for (void* p : vad) ((wdr_vad*)p)->~wdr_vad();
  for (void* p : dia) ((wdr_diarizer*)p)->~wdr_diarizer();
  for (void* p : spk) ((wdr_speakers*)p)->~wdr_speakers();
  if (any_busy) return;   // the stream pools / profiler serve the calls still running
  destroy_stream_pools();
  prof_shutdown();
}

const char* wdr_last_error(void) { return g_err.c_str(); }
int wdr_abi_version(void) { return WDR_ABI_VERSION; }
int wdr_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
void wdr_free(void* p) { free(p); }

int wdr_engine_new(const wdr_engine_config* cfg, wdr_engine** out) {
  WDR_GUARD({
    auto* e = new wdr_engine();
    if (cfg) {
      e->cfg = *cfg;
      if (cfg->cache_dir) e->cache_dir = cfg->cache_dir;
      if (cfg->vad_model_path) e->vad_path = cfg->vad_model_path;
      if (cfg->diarize_segment_model_path) e->seg_path = cfg->diarize_segment_model_path;
      if (cfg->diarize_embedding_model_path) e->emb_path = cfg->diarize_embedding_model_path;
    } else {
      e->cfg.enable_dtw = 1;
      e->cfg.enable_flash_attn = 0;
      e->cfg.use_gpu = 1;
      e->cache_dir = "./cache";
    }
    *out = track(&Live::eng, e);
    return 0;
  })
}

void wdr_engine_free(wdr_engine* e) {
  if (untrack(&Live::eng, e)) delete e;
}

int wdr_engine_set_synthetic(wdr_engine* e, const wdr_synthetic* syn) {
  WDR_GUARD({
    WDR_USE(eng, e);
    e->syn = syn_of(syn);
    e->syn_set = true;
    e->contexts.clear();
    return 0;
  })
}

int wdr_transcribe_audio(wdr_engine* e, const char* audio_path, const wdr_transcribe_options* o,
                         const wdr_formatting_overrides* fmt, const wdr_callbacks* cb, wdr_segment_list** out) {
  WDR_GUARD({
    WDR_USE(eng, e);
    if (!audio_path || !file_exists(audio_path)) return fail("audio file doesn't exist");
    const std::string model = (o && o->model) ? o->model : "base";
    // ModelManager::ensure_whisper_model (src/engine.rs:78-81): the cached ggml file, offline.
    // No file: the reference's create_context fails "whisper file doesn't exist"
    // (src/transcribe.rs:99-101) unless synthetic weights were asked for explicitly.
    auto it = e->contexts.find(model);
    std::string model_path;
    if (it == e->contexts.end()) {
      model_path = find_model_file(e->cache_dir, model);
      if (model_path.empty() && !e->syn_set) return fail("whisper file doesn't exist");
    }
    if (o && o->translate_target && !(o->whisper_to_english == 1))
      return fail("translate_target: network translation is out of scope for libwdr");
    std::vector<int16_t> pcm = read_wav_impl(audio_path);
    std::vector<wdr_speech_segment> segs;
    std::vector<int16_t> dpad;   // owns the samples of pyannote segments (they index the padded buffer)
    std::vector<std::pair<double, double>> vad_mask;   // VadMaskOracle input (VAD branch only)
    bool have_mask = false;
    const bool vad = !o || o->enable_vad == 1;   // `if let Some(true) = options.enable_vad` (src/engine.rs:123)
    const int dev = e->cfg.has_gpu_device ? e->cfg.gpu_device : 0;
    // a model file from the config, else the cache; absent -> synthetic (opt-in) or an error
    auto resolve = [&](const std::string& cfg_path, const std::string& hub, const std::string& file,
                       const char* what) -> std::string {
      if (!cfg_path.empty()) {
        if (!file_exists(cfg_path.c_str())) throw std::runtime_error(std::string(what) + " file doesn't exist: " + cfg_path);
        return cfg_path;
      }
      const std::string f = find_cached_file(e->cache_dir, hub, file);
      if (f.empty() && !e->syn_set) throw std::runtime_error(std::string(what) + " file doesn't exist");
      return f;
    };
    bool diarize = false;
    std::string seg_path, emb_path;
    if (o && o->enable_diarize == 1) {
      // src/engine.rs:89-122: model paths from the config (both given) or the cache, then
      // pyannote segmentation -> SpeechSegments
      diarize = true;
      const bool both = !e->seg_path.empty() && !e->emb_path.empty();
      seg_path = resolve(both ? e->seg_path : "", "", "segmentation-3.0.onnx", "segmentation model");
      emb_path = resolve(both ? e->emb_path : "", "", "wespeaker_en_voxceleb_CAM++.onnx", "embedding model");
      if (!e->seg || e->seg_loaded != seg_path) {
        e->seg.reset();
        e->seg = std::make_unique<SegModel>(dev, seg_path);
        e->seg_loaded = seg_path;
      }
      const std::vector<DiarSegment> ds = e->seg->get_segments(pcm.data(), pcm.size());
      dpad.assign(pcm.begin(), pcm.end());
      dpad.resize(pcm.size() + (160000 - pcm.size() % 160000), 0);
      for (const DiarSegment& d : ds) segs.push_back({d.start, d.end, dpad.data() + d.start_idx, d.end_idx - d.start_idx});
    } else if (vad) {
      // src/engine.rs:123-139: cfg.vad_model_path, else ggml-silero-v5.1.2.bin from
      // ggml-org/whisper-vad (src/model_manager.rs:303-319)
      const std::string vp = resolve(e->vad_path, "models--ggml-org--whisper-vad", "ggml-silero-v5.1.2.bin", "VAD model");
      if (!e->vad || e->vad_loaded != vp) {
        e->vad.reset();
        e->vad = std::make_unique<VadModel>(dev, vp);
        e->vad_loaded = vp;
      }
      vad_get_segments(*e->vad, pcm.data(), pcm.size(), &vad_mask, &segs);
      have_mask = true;
    } else {
      // whole file as one segment (src/engine.rs:141-147)
      segs.push_back({0.0, (double)pcm.size() / 16000.0, pcm.data(), pcm.size()});
    }
    if (it == e->contexts.end())
      it = e->contexts.emplace(model, make_context(model, e->cfg.has_gpu_device, e->cfg.gpu_device, e->cfg.use_gpu,
                                                   e->cfg.enable_dtw, e->syn, model_path))
               .first;
    const wdr_diarize_options dopts = diarize_options(o, seg_path.c_str(), emb_path.c_str());
    std::string lang;
    bool has_lang = false;
    std::vector<Seg> res =
        run_pipeline(it->second.get(), segs, o, diarize ? &dopts : nullptr, e->syn, cb, &lang, &has_lang);
    // src/engine.rs:179-199: preset of the detected (else requested) language + overrides,
    // then process_segments with the VAD mask oracle when VAD produced the segments
    const std::string eff = has_lang ? lang : ((o && o->lang) ? std::string(o->lang) : std::string("auto"));
    PostProcessConfig pcfg = config_for_language(eff);
    apply_overrides(pcfg, fmt);
    res = from_fmt(process_segments(to_fmt(res), pcfg, have_mask ? &vad_mask : nullptr));
    *out = to_list(res, has_lang ? &lang : nullptr);
    return 0;
  })
}

int wdr_vad_create(const char* model_path, int8_t has_gpu_device, int32_t gpu_device, wdr_vad** out) {
  WDR_GUARD({
    if (model_path && !file_exists(model_path)) return fail(std::string("VAD model file doesn't exist: ") + model_path);
    auto v = std::make_unique<wdr_vad>();
    v->m = std::make_unique<VadModel>(has_gpu_device ? gpu_device : 0, model_path ? model_path : "");
    *out = track(&Live::vad, v.release());
    return 0;
  })
}

void wdr_vad_free(wdr_vad* v) {
  if (untrack(&Live::vad, v)) delete v;
}

int wdr_vad_probs(wdr_vad* v, const int16_t* samples, size_t n, float* probs_out, double* us_per_step) {
  WDR_GUARD({
    WDR_USE(vad, v);
    const std::vector<float> p = v->m->probs(samples, n);
    if (!p.empty()) memcpy(probs_out, p.data(), p.size() * 4);
    if (us_per_step) *us_per_step = v->m->last_scan_us_per_step;
    return 0;
  })
}

int wdr_vad_stats(wdr_vad* v, double* us_per_chunk) {
  WDR_GUARD({
    WDR_USE(vad, v);
    *us_per_chunk = v->m->last_scan_us_per_step;
    return 0;
  })
}

int wdr_vad_segments_from_probs(const float* probs, size_t n_probs, float* cs_out, size_t* n_out) {
  WDR_GUARD({
    const std::vector<std::pair<float, float>> cs =
        vad_segments_from_probs(std::vector<float>(probs, probs + n_probs), VadParams());
    for (size_t i = 0; i < cs.size(); ++i) {
      cs_out[2 * i] = cs[i].first;
      cs_out[2 * i + 1] = cs[i].second;
    }
    *n_out = cs.size();
    return 0;
  })
}

int wdr_vad_get_segments(wdr_vad* v, const int16_t* samples, size_t n, double** mask_out, size_t* n_mask,
                         wdr_speech_segment** segs_out, size_t* n_segs) {
  WDR_GUARD({
    WDR_USE(vad, v);
    std::vector<std::pair<double, double>> mask;
    std::vector<wdr_speech_segment> segs;
    vad_get_segments(*v->m, samples, n, &mask, &segs);
    *mask_out = (double*)malloc(std::max<size_t>(1, mask.size()) * 2 * sizeof(double));
    for (size_t i = 0; i < mask.size(); ++i) {
      (*mask_out)[2 * i] = mask[i].first;
      (*mask_out)[2 * i + 1] = mask[i].second;
    }
    *n_mask = mask.size();
    *segs_out = (wdr_speech_segment*)malloc(std::max<size_t>(1, segs.size()) * sizeof(wdr_speech_segment));
    if (!segs.empty()) memcpy(*segs_out, segs.data(), segs.size() * sizeof(wdr_speech_segment));
    *n_segs = segs.size();
    return 0;
  })
}

int wdr_diarizer_create(const char* segment_model_path, const char* embedding_model_path, int8_t has_gpu_device,
                        int32_t gpu_device, wdr_diarizer** out) {
  WDR_GUARD({
    for (const char* p : {segment_model_path, embedding_model_path})
      if (p && !file_exists(p)) return fail(std::string("diarization model file doesn't exist: ") + p);
    auto d = std::make_unique<wdr_diarizer>();
    d->device = has_gpu_device ? gpu_device : 0;
    d->seg_path = segment_model_path ? segment_model_path : "";
    d->emb_path = embedding_model_path ? embedding_model_path : "";
    // load eagerly: a bad file fails here, as ORT session creation does in the reference
    if (!d->seg_path.empty()) d->S();
    if (!d->emb_path.empty()) d->E();
    *out = track(&Live::dia, d.release());
    return 0;
  })
}

void wdr_diarizer_free(wdr_diarizer* d) {
  if (untrack(&Live::dia, d)) delete d;
}

int wdr_diarize_frame_classes(wdr_diarizer* d, const int16_t* samples, size_t n, int32_t* cls_out, float* logprobs_out) {
  WDR_GUARD({
    WDR_USE(dia, d);
    std::vector<float> lp;
    const std::vector<int> cls = d->S().frame_classes(samples, n, logprobs_out ? &lp : nullptr);
    for (size_t i = 0; i < cls.size(); ++i) cls_out[i] = cls[i];
    if (logprobs_out && !lp.empty()) memcpy(logprobs_out, lp.data(), lp.size() * 4);
    return 0;
  })
}

int wdr_diarize_get_segments(wdr_diarizer* d, const int16_t* samples, size_t n, wdr_speech_segment** segs_out,
                             size_t* n_segs) {
  WDR_GUARD({
    WDR_USE(dia, d);
    return diar_segments_out(d->S().get_segments(samples, n), samples, n, segs_out, n_segs);
  })
}

int wdr_diarize_segments_from_classes(const int32_t* cls, size_t n_windows, const int16_t* samples, size_t n,
                                      wdr_speech_segment** segs_out, size_t* n_segs) {
  WDR_GUARD({
    if (n_windows != n / 160000 + 1) return fail("frame classes: expected n / 160000 + 1 windows");
    std::vector<int> c(cls, cls + n_windows * 589);
    return diar_segments_out(diar_stitch(c, n), samples, n, segs_out, n_segs);
  })
}

int wdr_diarize_fbank(wdr_diarizer* d, const int16_t* samples, size_t n, float* feats_out, size_t* n_frames) {
  WDR_GUARD({
    WDR_USE(dia, d);
    const std::vector<float> f = d->E().feats(samples, n);
    if (!f.empty()) memcpy(feats_out, f.data(), f.size() * 4);
    *n_frames = f.size() / 80;
    return 0;
  })
}

int wdr_diarize_embedding(wdr_diarizer* d, const int16_t* samples, size_t n, float* emb_out, int8_t* ok) {
  WDR_GUARD({
    WDR_USE(dia, d);
    *ok = d->E().embed(samples, n, emb_out) ? 1 : 0;
    return 0;
  })
}

int wdr_diarize_embedding_batch(wdr_diarizer* d, const int16_t* const* samples, const size_t* n, int32_t B,
                                float* emb_out, int8_t* ok) {
  WDR_GUARD({
    WDR_USE(dia, d);
    if (B < 0) return fail("embedding batch: negative count");
    std::vector<char> k(B);
    if (B) d->E().embed_batch(samples, n, B, emb_out, k.data());
    for (int b = 0; b < B; ++b) ok[b] = k[b];
    return 0;
  })
}

int wdr_diarize_stats(wdr_diarizer* d, double* seg_ms, double* emb_ms) {
  WDR_GUARD({
    WDR_USE(dia, d);
    *seg_ms = d->seg ? d->seg->last_ms : 0.0;
    *emb_ms = d->cam ? d->cam->last_ms : 0.0;
    return 0;
  })
}

int wdr_speakers_new(int8_t has_max_speakers, uint64_t max_speakers, wdr_speakers** out) {
  WDR_GUARD({
    auto m = std::make_unique<wdr_speakers>();
    m->m = std::make_unique<SpeakerManager>((has_max_speakers && max_speakers != 0) ? max_speakers : UINT64_MAX);
    *out = track(&Live::spk, m.release());
    return 0;
  })
}

void wdr_speakers_free(wdr_speakers* m) {
  if (untrack(&Live::spk, m)) delete m;
}

int wdr_speakers_assign(wdr_speakers* m, const float* emb, int32_t dim, float threshold, char* id_out, size_t cap) {
  WDR_GUARD({
    WDR_USE(spk, m);
    const std::string id = m->m->assign(emb, dim, threshold);
    WDR_CHECK(cap > id.size(), "speaker id buffer too small");
    memcpy(id_out, id.c_str(), id.size() + 1);
    return 0;
  })
}

// host seam: libstdc++ std::discrete_distribution over f32 weights driven by std::mt19937(seed)
// (the draw whisper_sample_token makes at t > 0), to pin the oracle's restatement
int wdr_dbg_discrete(const float* w, size_t n, uint32_t seed, int32_t n_draws, int32_t* out) {
  WDR_GUARD({
    std::mt19937 g(seed);
    std::discrete_distribution<> d(w, w + n);
    for (int i = 0; i < n_draws; ++i) out[i] = d(g);
    return 0;
  })
}

int wdr_process_segments(const wdr_segment* segs, size_t n_segs, const char* lang, const wdr_formatting_overrides* ov,
                         int8_t has_mask, const double* vad_mask, size_t n_mask, wdr_segment_list** out) {
  WDR_GUARD({
    std::vector<Seg> in;
    for (size_t i = 0; i < n_segs; ++i) {
      Seg s;
      s.start = segs[i].start;
      s.end = segs[i].end;
      s.text = segs[i].text ? segs[i].text : "";
      s.has_words = segs[i].words != nullptr;
      for (size_t k = 0; s.has_words && k < segs[i].n_words; ++k) {
        Word w;
        w.text = segs[i].words[k].text ? segs[i].words[k].text : "";
        w.start = segs[i].words[k].start;
        w.end = segs[i].words[k].end;
        w.has_p = segs[i].words[k].has_probability != 0;
        w.p = segs[i].words[k].probability;
        s.words.push_back(std::move(w));
      }
      s.has_speaker = segs[i].speaker_id != nullptr;
      if (s.has_speaker) s.speaker = segs[i].speaker_id;
      in.push_back(std::move(s));
    }
    PostProcessConfig cfg = config_for_language(lang ? lang : "auto");
    apply_overrides(cfg, ov);
    std::vector<std::pair<double, double>> mask;
    for (size_t i = 0; has_mask && i < n_mask; ++i) mask.push_back({vad_mask[2 * i], vad_mask[2 * i + 1]});
    const std::vector<Seg> res = from_fmt(process_segments(to_fmt(in), cfg, has_mask ? &mask : nullptr));
    *out = to_list(res, nullptr);
    return 0;
  })
}

int wdr_dbg_model_file(int32_t kind, const char* path, char** names_out, float** data_out, size_t* n_values) {
  WDR_GUARD({
    if (!path || !file_exists(path)) return fail("model file doesn't exist");
    TensorMap tm;
    if (kind == 0) tm = load_silero_ggml(path);
    else if (kind == 1) tm = load_segmentation_onnx(path);
    else if (kind == 2) tm = load_campplus_onnx(path);
    else return fail("model file kind: 0 Silero ggml, 1 segmentation ONNX, 2 CAM++ ONNX");
    std::string names;
    size_t tot = 0;
    for (auto& kv : tm) {
      names += kv.first + ":" + std::to_string(kv.second.size()) + "\n";
      tot += kv.second.size();
    }
    *names_out = strdup(names.c_str());
    *data_out = (float*)malloc(std::max<size_t>(1, tot) * 4);
    size_t o = 0;
    for (auto& kv : tm) {
      if (!kv.second.empty()) memcpy(*data_out + o, kv.second.data(), kv.second.size() * 4);
      o += kv.second.size();
    }
    *n_values = tot;
    return 0;
  })
}

int wdr_read_wav(const char* path, int16_t** samples, size_t* n) {
  WDR_GUARD({
    std::vector<int16_t> v = read_wav_impl(path);
    *samples = (int16_t*)malloc(std::max<size_t>(1, v.size()) * 2);
    if (!v.empty()) memcpy(*samples, v.data(), v.size() * 2);
    *n = v.size();
    return 0;
  })
}

// src/vad.rs:33-84: input = whisper.cpp VAD segments in centiseconds
int wdr_vad_merge(const double* st_cs, const double* en_cs, size_t n_segs, const int16_t* samples, size_t n_samples,
                  double* mask_out, size_t* n_mask, double* merged_out, int64_t* merged_idx, size_t* n_merged) {
  (void)samples;
  WDR_GUARD({
    std::vector<std::pair<double, double>> mask;
    for (size_t i = 0; i < n_segs; ++i) {
      const double a = (double)(float)st_cs[i] / 100.0, b = (double)(float)en_cs[i] / 100.0;
      if (b > a) mask.push_back({a, b});
    }
    std::stable_sort(mask.begin(), mask.end(), [](auto& x, auto& y) { return x.first < y.first; });
    std::vector<std::pair<double, double>> merged;
    for (auto& m : mask) {
      if (!merged.empty() && m.first - merged.back().second < 0.200) merged.back().second = std::max(m.second, merged.back().second);
      else merged.push_back(m);
    }
    const float SR = 16000.0f, nf = (float)n_samples;
    size_t k = 0;
    for (auto& m : merged) {
      const size_t si = (size_t)std::min(std::max(std::round((float)m.first * SR), 0.0f), nf);
      const size_t ei = (size_t)std::min(std::max(std::round((float)m.second * SR), 0.0f), nf);
      if (!(m.second > m.first) || !(ei > si)) continue;
      merged_out[2 * k] = m.first;
      merged_out[2 * k + 1] = m.second;
      merged_idx[2 * k] = (int64_t)si;
      merged_idx[2 * k + 1] = (int64_t)ei;
      ++k;
    }
    for (size_t i = 0; i < mask.size(); ++i) {
      mask_out[2 * i] = mask[i].first;
      mask_out[2 * i + 1] = mask[i].second;
    }
    *n_mask = mask.size();
    *n_merged = k;
    return 0;
  })
}

int wdr_context_create(const char* model_path, const char* model_name, int8_t has_gpu_device, int32_t gpu_device,
                       int8_t use_gpu, int8_t enable_dtw, int8_t enable_flash_attn, int8_t has_num_samples,
                       uint64_t num_samples, const wdr_synthetic* syn, wdr_context** out) {
  (void)enable_flash_attn;
  (void)has_num_samples;
  (void)num_samples;
  WDR_GUARD({
    if (model_path && *model_path && !file_exists(model_path)) return fail("whisper file doesn't exist");
    if ((!model_path || !*model_path) && !syn) return fail("whisper file doesn't exist");
    *out = track(&Live::ctx, make_context(model_name ? model_name : "base", has_gpu_device == 1, gpu_device, use_gpu,
                                          enable_dtw, syn_of(syn), model_path ? std::string(model_path) : std::string())
                                 .release());
    return 0;
  })
}

void wdr_context_free(wdr_context* c) {
  if (untrack(&Live::ctx, c)) delete c;
}

int wdr_ggml_info(const char* path, int32_t* hparams, int64_t* n_tensors, int64_t* n_vocab_tokens) {
  WDR_GUARD({
    if (!path || !file_exists(path)) return fail("whisper file doesn't exist");
    const GgmlFile f(path);
    memcpy(hparams, f.hp, sizeof f.hp);
    *n_tensors = (int64_t)f.tensors.size();
    *n_vocab_tokens = (int64_t)f.vocab.size();
    return 0;
  })
}

int wdr_run_pipeline(wdr_context* c, const wdr_speech_segment* segs, size_t n_segs, const wdr_transcribe_options* o,
                     const wdr_diarize_options* dopts, const wdr_synthetic* syn, const wdr_callbacks* cb,
                     wdr_segment_list** out) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    std::vector<wdr_speech_segment> v(segs, segs + n_segs);
    std::string lang;
    bool has_lang = false;
    const double t = now_s();
    c->st->times = StageTimes{};
    c->cs = wdr_context::ChainStats{};
    std::vector<Seg> res = run_pipeline(c, v, o, dopts, syn_of(syn), cb, &lang, &has_lang);
    c->st->times.glue = now_s() - t;   // total wall for this pipeline call
    *out = to_list(res, has_lang ? &lang : nullptr);
    return 0;
  })
}

int wdr_run_pipeline_raw(wdr_context* c, const wdr_speech_segment* segs, size_t n_segs,
                         const wdr_transcribe_options* o, const wdr_synthetic* syn, wdr_segment_list** out) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    std::vector<wdr_speech_segment> v(segs, segs + n_segs);
    std::string lang;
    bool has_lang = false;
    const double t = now_s();
    c->st->times = StageTimes{};
    c->cs = wdr_context::ChainStats{};
    std::vector<Seg> res = run_pipeline(c, v, o, nullptr, syn_of(syn), nullptr, &lang, &has_lang, true);
    c->st->times.glue = now_s() - t;
    *out = to_list(res, has_lang ? &lang : nullptr);
    if (!(*out)->speech_index && !res.empty()) return fail("raw pipeline: missing speech index");
    return 0;
  })
}

int wdr_run_pipeline_block(wdr_context* c, const wdr_speech_segment* segs, size_t n_segs,
                           const wdr_transcribe_options* o, const wdr_synthetic* syn, const char* rng_in,
                           int8_t* sampled_out, char** rng_out, wdr_segment_list** out) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    std::vector<wdr_speech_segment> v(segs, segs + n_segs);
    std::string lang;
    bool has_lang = false;
    const double t = now_s();
    c->st->times = StageTimes{};
    c->cs = wdr_context::ChainStats{};
    RngCarry carry;
    const std::string in = rng_in ? std::string(rng_in) : std::string();
    if (rng_in) carry.rng_in = &in;
    std::vector<Seg> res = run_pipeline(c, v, o, nullptr, syn_of(syn), nullptr, &lang, &has_lang, true, &carry);
    c->st->times.glue = now_s() - t;
    for (size_t i = 0; i < n_segs; ++i) sampled_out[i] = carry.sampled[i];
    *rng_out = strdup(carry.rng_out.c_str());
    *out = to_list(res, has_lang ? &lang : nullptr);
    return 0;
  })
}

void wdr_segment_list_free(wdr_segment_list* l) {
  if (!l) return;
  for (size_t i = 0; i < l->n_segments; ++i) {
    wdr_segment& s = l->segments[i];
    free((void*)s.text);
    for (size_t k = 0; k < s.n_words; ++k) free((void*)s.words[k].text);
    free((void*)s.words);
    free((void*)s.speaker_id);
  }
  free(l->segments);
  free((void*)l->detected_lang);
  free((void*)l->speech_index);
  free(l);
}

int wdr_dbg_set_early_fixup(wdr_context* c, int32_t mode) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    if (mode < -1 || mode > 3) return fail("early fix-up mode: -1 (env default), 0, 1, 2 or 3");
    c->early_fixup = mode;
    return 0;
  })
}

int wdr_dbg_set_gemm32(int32_t mfma) {
  WDR_GUARD({
    set_gemm32_mfma(mfma != 0);
    return 0;
  })
}

int wdr_context_set_encoder_fp8(wdr_context* c, int8_t on) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    c->ctx->fp8_encoder = on != 0;
    for (auto& p : c->peers) p->fp8_encoder = on != 0;
    return 0;
  })
}

int wdr_context_devices(const wdr_context* c, int32_t* n, int32_t* device_ids, int32_t cap) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    *n = (int32_t)c->devices.size();
    for (int32_t i = 0; device_ids && i < cap && i < *n; ++i) device_ids[i] = c->devices[i];
    return 0;
  })
}

int wdr_context_set_chains(wdr_context* c, int32_t n) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    if (n < 1) return fail("decode chains: need >= 1");
    c->chains = std::min<int>(n, c->ctx->max_chains);
    return 0;
  })
}

int wdr_context_stage_times(wdr_context* c, wdr_stage_times* o) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    const StageTimes& t = c->st->times;
    *o = wdr_stage_times{t.mel,          t.encode,   t.decode,  t.dtw,        0.0,  t.glue, t.windows,
                         t.decode_steps, t.prefills, t.lang,    t.prompt_gpu, c->embed_s};
    o->chains = c->cs.chains;
    o->batch_launches = c->cs.launches;
    o->batch_rows = c->cs.rows;
    o->fixup_segments = c->cs.fixups;
    o->replay_segments = c->cs.replays;
    o->spec_s = c->cs.spec_s;
    o->fixup_s = c->cs.fixup_s;
    o->batch_step_s = c->cs.step_s;
    o->early_fixup_segments = c->cs.early;
    o->batch_prefill_rows = c->cs.prefill_rows;
    o->batch_dtw_rows = c->cs.dtw_rows;
    o->batch_prefills = c->cs.prefills;
    o->batch_dtws = c->cs.dtws;
    o->batch_mixed = c->cs.mixed;
    o->batch_xattn_groups = c->cs.vgroups;
    o->batch_xattn_tiles = c->cs.tiles;
    o->dtwq_passes = c->cs.dq_passes;
    o->dtwq_rows = c->cs.dq_rows;
    o->dtwq_jobs = c->cs.dq_jobs;
    o->lang_passes = t.lang_passes;
    o->lang_rows = t.lang_rows;
    return 0;
  })
}

int wdr_context_hparams(wdr_context* c, int32_t* o) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    const HParams& h = c->ctx->model.hp;
    const int32_t v[10] = {h.n_vocab, h.n_audio_ctx, h.n_audio_state, h.n_audio_head, h.n_audio_layer,
                           h.n_text_ctx, h.n_text_state, h.n_text_head, h.n_text_layer, h.n_mels};
    memcpy(o, v, sizeof v);
    return 0;
  })
}

int wdr_state_full(wdr_context* c, const float* samples, size_t n, const wdr_transcribe_options* o,
                   const wdr_synthetic* syn, const char* initial_prompt, wdr_result_seg** segs, size_t* n_segs,
                   int32_t* lang_id) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    FullParams p = setup_params(o, syn_of(syn));
    if (initial_prompt) {
      p.initial_prompt = initial_prompt;
      p.has_initial_prompt = true;
    }
    const int rc = c->st->full(p, samples, (int)n);
    if (rc != 0) return fail("failed to transcribe");
    const auto& r = c->st->result_all;
    *n_segs = r.size();
    *segs = (wdr_result_seg*)calloc(std::max<size_t>(1, r.size()), sizeof(wdr_result_seg));
    for (size_t i = 0; i < r.size(); ++i) {
      (*segs)[i].t0 = r[i].t0;
      (*segs)[i].t1 = r[i].t1;
      (*segs)[i].text = strdup(r[i].text.c_str());
      auto* t = (wdr_token*)calloc(std::max<size_t>(1, r[i].tokens.size()), sizeof(wdr_token));
      for (size_t k = 0; k < r[i].tokens.size(); ++k) {
        const TokenData& d = r[i].tokens[k];
        t[k] = {d.id, d.tid, d.p, d.plog, d.pt, d.ptsum, d.t0, d.t1, d.t_dtw};
      }
      (*segs)[i].tokens = t;
      (*segs)[i].n_tokens = r[i].tokens.size();
    }
    *lang_id = c->st->lang_id;
    return 0;
  })
}

void wdr_result_free(wdr_result_seg* segs, size_t n) {
  if (!segs) return;
  for (size_t i = 0; i < n; ++i) {
    free((void*)segs[i].text);
    free((void*)segs[i].tokens);
  }
  free(segs);
}

int wdr_dbg_log_mel(wdr_context* c, const float* x, size_t n, int32_t seek, float* out) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    c->st->compute_mel(x, (int)n);
    c->st->read_mel_window(seek, out);
    return 0;
  })
}

int wdr_dbg_mfma_scale(const uint8_t* a, const uint8_t* b, const int32_t* sa, const int32_t* sb, float* out) {
  WDR_GUARD({
    DevMem d(64 * 32 * 2 + 64 * 4 * 2 + 64 * 16);
    char* p = (char*)d.p;
    WDR_HIP(hipMemcpy(p, a, 2048, hipMemcpyHostToDevice));
    WDR_HIP(hipMemcpy(p + 2048, b, 2048, hipMemcpyHostToDevice));
    WDR_HIP(hipMemcpy(p + 4096, sa, 256, hipMemcpyHostToDevice));
    WDR_HIP(hipMemcpy(p + 4352, sb, 256, hipMemcpyHostToDevice));
    launch_probe_mfma_scale(p, p + 2048, (const int*)(p + 4096), (const int*)(p + 4352), (float*)(p + 4608), nullptr);
    WDR_HIP(hipMemcpy(out, p + 4608, 1024, hipMemcpyDeviceToHost));
    return 0;
  })
}

int wdr_dbg_energy(const float* x, size_t n, float* out) {
  WDR_GUARD({
    DevMem dx(std::max<size_t>(1, n) * 4), de(std::max<size_t>(1, n) * 4);
    WDR_HIP(hipMemcpy(dx.p, x, n * 4, hipMemcpyHostToDevice));
    launch_energy(dx.as<float>(), (int)n, de.as<float>(), nullptr);
    WDR_HIP(hipMemcpy(out, de.p, n * 4, hipMemcpyDeviceToHost));
    return 0;
  })
}

int wdr_dbg_encode(wdr_context* c, const float* mel_window, float* enc_out) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    c->st->encode_from_mel_window(mel_window);
    c->st->read_encoder_out(enc_out);
    return 0;
  })
}

int wdr_dbg_cross_kv(wdr_context* c, float* out) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    c->st->read_cross_kv(out);
    return 0;
  })
}

int wdr_dbg_decode(wdr_context* c, const int32_t* tokens, size_t n, float* logits_out) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    c->st->decode_logits(tokens, (int)n, logits_out);
    return 0;
  })
}

int wdr_dbg_step(wdr_context* c, const int32_t* tokens, size_t n, float* logits_out) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    c->st->dbg_step(tokens, (int)n, logits_out);
    return 0;
  })
}

int wdr_dbg_logits(wdr_context* c, const float* logits, int32_t R, const int32_t* ctl, const float* temperature,
                   float max_initial_ts, int32_t suppress_blank, int32_t* ids_out, float* f_out) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    WDR_CHECK(R >= 1 && R <= 8, "dbg_logits: 1..8 rows");
    std::vector<LogitsCtl> lc(R);
    for (int r = 0; r < R; ++r) {
      const int32_t* q = ctl + 7 * r;
      lc[r] = LogitsCtl{q[0], q[1], q[2], q[3], q[4], q[5], q[6], temperature[r]};
    }
    std::vector<TokenData> out(R);
    std::vector<float> nosp(R);
    c->st->dbg_logits(logits, R, lc.data(), max_initial_ts, suppress_blank != 0, out.data(), nosp.data());
    for (int r = 0; r < R; ++r) {
      ids_out[2 * r] = out[r].id;
      ids_out[2 * r + 1] = out[r].tid;
      float* f = f_out + 5 * r;
      f[0] = out[r].p;
      f[1] = out[r].plog;
      f[2] = out[r].pt;
      f[3] = out[r].ptsum;
      f[4] = nosp[r];
    }
    return 0;
  })
}

int wdr_dbg_batch_step(wdr_context* c, const int32_t* tokens, size_t n, int32_t rows, int32_t iters,
                       double* ms_per_step) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    *ms_per_step = c->st->dbg_batch_step(tokens, (int)n, rows, iters);
    return 0;
  })
}

int wdr_dbg_capture(wdr_context* c, const int32_t* tokens, size_t n, float* cap_out) {
  WDR_GUARD({
    WDR_USE(ctx, c);
    if (c->ctx->aheads.empty()) return fail("context created without DTW");
    c->st->dtw_capture(tokens, (int)n, cap_out);
    return 0;
  })
}

int wdr_dbg_dtw(const float* cap, int32_t A, int32_t N, int32_t M, int32_t sot_len, int32_t seek, float* x_out,
                int32_t* times_out, int32_t* n_times) {
  WDR_GUARD({
    DevMem dcap((size_t)A * N * 1500 * 4), dn((size_t)A * N * M * 4), dx((size_t)N * M * 4), dt((N + 8) * 4);
    WDR_HIP(hipMemcpy(dcap.p, cap, dcap.bytes, hipMemcpyHostToDevice));
    launch_dtw(dcap.as<float>(), A, N, 1500, M, sot_len, seek, dn.as<float>(), dx.as<float>(), dt.as<int>(),
               dt.as<int>() + N + 4, nullptr);
    WDR_HIP(hipDeviceSynchronize());
    const int rows = N - sot_len - 1;
    WDR_HIP(hipMemcpy(x_out, dx.p, (size_t)rows * M * 4, hipMemcpyDeviceToHost));
    std::vector<int> t(N + 8);
    WDR_HIP(hipMemcpy(t.data(), dt.p, t.size() * 4, hipMemcpyDeviceToHost));
    *n_times = t[N + 4];
    for (int i = 0; i < *n_times; ++i) times_out[i] = t[i];
    return 0;
  })
}

int wdr_dbg_dtw_dp(const float* x, int32_t rows, int32_t cols, int32_t seek, int32_t* times_out, int32_t* n_times) {
  WDR_GUARD({
    DevMem dx((size_t)rows * cols * 4), dt((rows + 8) * 4);
    WDR_HIP(hipMemcpy(dx.p, x, dx.bytes, hipMemcpyHostToDevice));
    launch_dtw_dp_only(dx.as<float>(), rows, cols, seek, dt.as<int>(), dt.as<int>() + rows + 4, nullptr);
    std::vector<int> t(rows + 8);
    WDR_HIP(hipMemcpy(t.data(), dt.p, t.size() * 4, hipMemcpyDeviceToHost));
    *n_times = t[rows + 4];
    for (int i = 0; i < *n_times; ++i) times_out[i] = t[i];
    return 0;
  })
}

// fp8 encoder projection (MX): a, w quantised on the GPU (launch_quant_f8: e4m3 + one E8M0 scale
// per 32 k), the fp8 GEMM k_gemm8 with the epilogue `epi` (out f32 in / out, as wdr_dbg_proj;
// EPI_F8_GELU: out = the dequantised e4m3 GELU output); the quantised bytes and the scale bytes
// ([rows][K/32]) come back for the reference product
int wdr_dbg_proj_fp8(const uint16_t* a16, const uint16_t* w16, const float* bias, int32_t M, int32_t N, int32_t K,
                     int32_t epi, float* out, uint8_t* a8_out, uint8_t* a_sc_out, uint8_t* w8_out, uint8_t* w_sc_out) {
  WDR_GUARD({
    WDR_CHECK(M > 64 && N % 256 == 0 && K % 128 == 0, "dbg fp8 projection: M > 64, N % 256, K % 128");
    const int mp = (M + 255) / 256 * 256;
    DevMem da((size_t)M * K * 2), dw((size_t)N * K * 2), db(bias ? (size_t)N * 4 : 0), dout((size_t)M * N * 4);
    DevMem a8((size_t)M * K), w8((size_t)N * K), as((size_t)K / 128 * mp * 4), ws((size_t)K / 128 * N * 4);
    DevMem osc((size_t)N / 128 * mp * 4);
    WDR_HIP(hipMemcpy(da.p, a16, da.bytes, hipMemcpyHostToDevice));
    WDR_HIP(hipMemcpy(dw.p, w16, dw.bytes, hipMemcpyHostToDevice));
    if (bias) WDR_HIP(hipMemcpy(db.p, bias, db.bytes, hipMemcpyHostToDevice));
    launch_quant_f8(da.as<f16>(), K, M, K, a8.as<uint8_t>(), K, as.as<uint32_t>(), mp, nullptr);
    launch_quant_f8(dw.as<f16>(), K, N, K, w8.as<uint8_t>(), K, ws.as<uint32_t>(), N, nullptr);
    const bool f16out = epi == EPI_F16 || epi == EPI_F16_GELU;
    if (!f16out && epi != EPI_F8_GELU) WDR_HIP(hipMemcpy(dout.p, out, dout.bytes, hipMemcpyHostToDevice));
    ProjArgs p{nullptr, K, nullptr, K, bias ? db.as<float>() : nullptr, dout.p, N, nullptr, 0, M, N, K, epi};
    p.A8 = a8.as<uint8_t>();
    p.a_sc = as.as<uint32_t>();
    p.ld_asc = mp;
    p.B8 = w8.as<uint8_t>();
    p.b_sc = ws.as<uint32_t>();
    p.ld_bsc = N;
    p.o_sc = osc.as<uint32_t>();
    p.ld_osc = mp;
    launch_proj_fp8(p, nullptr);
    WDR_HIP(hipDeviceSynchronize());
    // a scale image [K/128][ld] of u32 -> bytes [rows][K/32]
    auto unscale = [](const DevMem& d, int rows, int ld, int K, uint8_t* dst) {
      std::vector<uint32_t> h(d.bytes / 4);
      WDR_HIP(hipMemcpy(h.data(), d.p, d.bytes, hipMemcpyDeviceToHost));
      for (int r = 0; r < rows; ++r)
        for (int b = 0; b < K / 32; ++b) dst[(size_t)r * (K / 32) + b] = (uint8_t)(h[(size_t)(b / 4) * ld + r] >> (8 * (b % 4)));
    };
    if (epi == EPI_F8_GELU) {
      std::vector<uint8_t> q((size_t)M * N), sc((size_t)M * (N / 32));
      WDR_HIP(hipMemcpy(q.data(), dout.p, q.size(), hipMemcpyDeviceToHost));
      unscale(osc, M, mp, N, sc.data());
      for (int r = 0; r < M; ++r)
        for (int c = 0; c < N; ++c) {
          const uint8_t v = q[(size_t)r * N + c];
          // OCP e4m3fn: s eeee mmm, bias 7, no infinities, 0x7f / 0xff NaN
          const int e = (v >> 3) & 15, mt = v & 7;
          float x = e ? std::ldexp(1.0f + mt / 8.0f, e - 7) : std::ldexp(mt / 8.0f, -6);
          if ((v & 0x7f) == 0x7f) x = NAN;
          x = (v & 0x80) ? -x : x;
          out[(size_t)r * N + c] = std::ldexp(x, (int)sc[(size_t)r * (N / 32) + c / 32] - 127);
        }
    } else if (f16out) {
      std::vector<f16> h((size_t)M * N);
      WDR_HIP(hipMemcpy(h.data(), dout.p, h.size() * 2, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < h.size(); ++i) out[i] = (float)h[i];
    } else {
      WDR_HIP(hipMemcpy(out, dout.p, dout.bytes, hipMemcpyDeviceToHost));
    }
    if (a8_out) WDR_HIP(hipMemcpy(a8_out, a8.p, a8.bytes, hipMemcpyDeviceToHost));
    if (a_sc_out) unscale(as, M, mp, K, a_sc_out);
    if (w8_out) WDR_HIP(hipMemcpy(w8_out, w8.p, w8.bytes, hipMemcpyDeviceToHost));
    if (w_sc_out) unscale(ws, N, N, K, w_sc_out);
    return 0;
  })
}

int wdr_dbg_proj(const uint16_t* a16, const uint16_t* w16, const float* bias, int32_t M, int32_t N, int32_t K,
                 int32_t epi, float* out) {
  WDR_GUARD({
    DevMem da((size_t)M * K * 2), dw((size_t)N * K * 2), db(bias ? (size_t)N * 4 : 0), dout((size_t)M * N * 4);
    WDR_HIP(hipMemcpy(da.p, a16, da.bytes, hipMemcpyHostToDevice));
    WDR_HIP(hipMemcpy(dw.p, w16, dw.bytes, hipMemcpyHostToDevice));
    if (bias) WDR_HIP(hipMemcpy(db.p, bias, db.bytes, hipMemcpyHostToDevice));
    // epi | WDR_DBG_PROJ_ROWS: the decoder-rows kernel (ProjArgs::rows_mma, any M); <= 64 rows
    // run on it anyway
    if (epi & 0x100) return fail("WDR_DBG_PROJ_STEP: the decode-step GEMV schedule was removed (the row kernel serves every row count)");
    const bool rows = (epi & 0x200) != 0;
    if (epi & 0x400) return fail("WDR_DBG_PROJ_SPLIT: the split-K residual projections were removed (k_skinny runs them whole)");
    const bool gemm_ref = (epi & 0x800) != 0;
    epi &= 0xff;
    const bool f16out = epi == EPI_F16 || epi == EPI_F16_GELU;
    std::vector<f16> h16;
    if (!f16out) WDR_HIP(hipMemcpy(dout.p, out, dout.bytes, hipMemcpyHostToDevice));
    ProjArgs a{da.as<f16>(), K, dw.as<f16>(), K, bias ? db.as<float>() : nullptr, dout.p, N, nullptr, 0, M, N, K, epi};
    a.rows_mma = rows ? 1 : 0;
    a.gemm_ref = gemm_ref ? 1 : 0;
    launch_proj(a, nullptr);
    WDR_HIP(hipDeviceSynchronize());
    if (f16out) {
      h16.resize((size_t)M * N);
      WDR_HIP(hipMemcpy(h16.data(), dout.p, h16.size() * 2, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < h16.size(); ++i) out[i] = (float)h16[i];
    } else {
      WDR_HIP(hipMemcpy(out, dout.p, dout.bytes, hipMemcpyDeviceToHost));
    }
    return 0;
  })
}

int wdr_dbg_proj_ln(const float* x, const float* gamma, const float* beta, const uint16_t* w16, const float* bias,
                    int32_t M, int32_t N, int32_t K, int32_t epi, int32_t fused, float* out) {
  WDR_GUARD({
    // K % 128: the fused prologue's 16-chunk row swizzle (csrc/rows.cpp launch_rows)
    if (M < 1 || N < 1 || K < 128 || K > 1280 || K % 128) return fail("dbg_proj_ln: M >= 1, K % 128 == 0, K <= 1280");
    if (epi != EPI_F16 && epi != EPI_F16_GELU && epi != EPI_F32) return fail("dbg_proj_ln: epi 0, 1 or 3");
    DevMem dx((size_t)M * K * 4), dg((size_t)K * 4), dbt((size_t)K * 4), dw((size_t)N * K * 2),
        db(bias ? (size_t)N * 4 : 0), dh((size_t)M * K * 2), dout((size_t)M * N * 4);
    WDR_HIP(hipMemcpy(dx.p, x, dx.bytes, hipMemcpyHostToDevice));
    WDR_HIP(hipMemcpy(dg.p, gamma, dg.bytes, hipMemcpyHostToDevice));
    WDR_HIP(hipMemcpy(dbt.p, beta, dbt.bytes, hipMemcpyHostToDevice));
    WDR_HIP(hipMemcpy(dw.p, w16, dw.bytes, hipMemcpyHostToDevice));
    if (bias) WDR_HIP(hipMemcpy(db.p, bias, db.bytes, hipMemcpyHostToDevice));
    ProjArgs a{nullptr, K, dw.as<f16>(), K, bias ? db.as<float>() : nullptr, dout.p, N, nullptr, 0, M, N, K, epi};
    a.rows_mma = 1;
    if (fused) {   // rows_forward's fused form (csrc/rows.cpp)
      a.ln_x = dx.as<float>();
      a.ldln = K;
      a.ln_g = dg.as<float>();
      a.ln_b = dbt.as<float>();
    } else {
      launch_layernorm(dx.as<float>(), K, dg.as<float>(), dbt.as<float>(), dh.as<f16>(), K, M, K, nullptr);
      a.A = dh.as<f16>();
    }
    launch_proj(a, nullptr);
    WDR_HIP(hipDeviceSynchronize());
    if (epi == EPI_F32) {
      WDR_HIP(hipMemcpy(out, dout.p, dout.bytes, hipMemcpyDeviceToHost));
    } else {
      std::vector<f16> h((size_t)M * N);
      WDR_HIP(hipMemcpy(h.data(), dout.p, h.size() * 2, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < h.size(); ++i) out[i] = (float)h[i];
    }
    return 0;
  })
}

int wdr_dbg_attn(const uint16_t* q, const uint16_t* k, const uint16_t* v, int32_t Tq, int32_t Tk, int32_t H,
                 int32_t causal, float* out) {
  WDR_GUARD({
    const int d = H * 64;
    DevMem dq((size_t)Tq * d * 2), dk((size_t)Tk * d * 2), dv((size_t)Tk * d * 2), dout((size_t)Tq * d * 2);
    WDR_HIP(hipMemcpy(dq.p, q, dq.bytes, hipMemcpyHostToDevice));
    WDR_HIP(hipMemcpy(dk.p, k, dk.bytes, hipMemcpyHostToDevice));
    WDR_HIP(hipMemcpy(dv.p, v, dv.bytes, hipMemcpyHostToDevice));
    FlashArgs fa{dq.as<f16>(), d, 0, dk.as<f16>(), d, 0, dv.as<f16>(), d, 0, dout.as<f16>(), d, 0, nullptr, Tq, Tk, H,
                 causal, 0.125f};
    DevMem po, pml;
    if (!causal && Tq <= 256 && Tk >= 512) {   // exercise the split-K path the decoder prefill uses
      fa.nsplit = 12;
      po = DevMem((size_t)12 * Tq * H * 64 * 4);
      pml = DevMem((size_t)12 * H * Tq * 8);
      fa.part_o = po.as<float>();
      fa.part_ml = pml.as<float2>();
    }
    launch_flash_attn(fa, 1, nullptr);
    std::vector<f16> h((size_t)Tq * d);
    WDR_HIP(hipMemcpy(h.data(), dout.p, h.size() * 2, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < h.size(); ++i) out[i] = (float)h[i];
    return 0;
  })
}

// decode-step cross-attention (kernels/attn.hip k_xattn_dec) over 1500 keys: q [R][H*64],
// kv [S][1500][2 * H * 64] (K then V per key), row_slot [R] (null: every row on slot 0 through
// the shared-K/V form, R <= 8), grp [R] group sizes (XAttnArgs::grp, or null); run `iters`
// times on the same arrival counters; out [R][H * 64]
int wdr_dbg_xattn(const uint16_t* q, const uint16_t* kv, const int32_t* row_slot, const int32_t* grp, int32_t R,
                  int32_t S, int32_t H, int32_t iters, float* out) {
  WDR_GUARD({
    WDR_CHECK(R >= 1 && R <= 1024 && S >= 1 && H >= 1 && H <= 32 && iters >= 1, "dbg xattn: bad shape");
    const int d = H * 64, T = 1500;
    DevMem dq((size_t)R * d * 2), dkv((size_t)S * T * 2 * d * 2), dout((size_t)R * d * 2);
    DevMem po((size_t)24 * R * H * 64 * 4), pml((size_t)24 * R * H * 8);
    DevMem drk(R * sizeof(void*)), dg(R * 4), dl(R * 4);
    WDR_HIP(hipMemcpy(dq.p, q, dq.bytes, hipMemcpyHostToDevice));
    WDR_HIP(hipMemcpy(dkv.p, kv, dkv.bytes, hipMemcpyHostToDevice));
    XAttnArgs xa{dq.as<f16>(), d, dkv.as<f16>(), dkv.as<f16>() + d, 2 * d, T, R, H, 0.125f, po.as<float>(),
                 pml.as<float2>(), dout.as<f16>(), d};
    if (row_slot) {
      std::vector<const f16*> rk(R);
      for (int r = 0; r < R; ++r) {
        WDR_CHECK(row_slot[r] >= 0 && row_slot[r] < S, "dbg xattn: slot out of range");
        rk[r] = dkv.as<f16>() + (size_t)row_slot[r] * T * 2 * d;
      }
      WDR_HIP(hipMemcpy(drk.p, rk.data(), R * sizeof(void*), hipMemcpyHostToDevice));
      xa.row_k = drk.as<const f16*>();
      xa.v_off = d;   // this probe's K/V: [S][1500][2d], K then V per key
      bool big = false;
      for (int r = 0; grp && r < R; ++r) big = big || grp[r] > XATTN_GRP_MAX;
      if (grp && big) {
        // the decoder-rows form (rows_forward): groups of <= XATTN_GRP_MAX rows on the VALU kernel,
        // larger ones as MFMA row tiles of <= 128 rows, one combine for every row
        std::vector<int> g(R, 0), lead;
        std::vector<int4> tiles;
        for (int r = 0; r < R; ++r) {
          if (grp[r] == 0) continue;
          WDR_CHECK(r + grp[r] <= R, "dbg xattn: bad group");
          if (grp[r] <= XATTN_GRP_MAX) {
            g[r] = grp[r];
            lead.push_back(r);
          } else {
            for (int t = 0; t < grp[r]; t += 128) tiles.push_back(make_int4(r + t, std::min(128, grp[r] - t), 1 << 30, 0));
          }
        }
        WDR_HIP(hipMemcpy(dg.p, g.data(), R * 4, hipMemcpyHostToDevice));
        if (!lead.empty()) WDR_HIP(hipMemcpy(dl.p, lead.data(), lead.size() * 4, hipMemcpyHostToDevice));
        DevMem dt(std::max<size_t>(16, tiles.size() * 16));
        if (!tiles.empty()) WDR_HIP(hipMemcpy(dt.p, tiles.data(), tiles.size() * 16, hipMemcpyHostToDevice));
        xa.grp = dg.as<int>();
        xa.lead = dl.as<int>();
        xa.n_vgrp = (int)lead.size();
        xa.vgrp_max = 1;
        for (int r : lead) xa.vgrp_max = std::max(xa.vgrp_max, g[r]);
        xa.tiles = dt.as<int4>();
        xa.n_tiles = (int)tiles.size();
        for (int i = 0; i < iters; ++i) launch_xattn_rows(xa, nullptr);
        WDR_HIP(hipDeviceSynchronize());
        std::vector<f16> h((size_t)R * d);
        WDR_HIP(hipMemcpy(h.data(), dout.p, h.size() * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < h.size(); ++i) out[i] = (float)h[i];
        return 0;
      }
      if (grp) {
        int ng = 0;
        for (int r = 0; r < R; ++r) {
          WDR_CHECK(grp[r] >= 0 && grp[r] <= XATTN_GRP_MAX && r + grp[r] <= R, "dbg xattn: bad group");
          ng += grp[r] > 0;
        }
        WDR_HIP(hipMemcpy(dg.p, grp, R * 4, hipMemcpyHostToDevice));
        xa.grp = dg.as<int>();
        xa.n_grp = ng;
        // one workgroup row per group, as the step batcher launches it
        std::vector<int> lead;
        for (int r = 0; r < R; ++r)
          if (grp[r] > 0) lead.push_back(r);
        WDR_HIP(hipMemcpy(dl.p, lead.data(), lead.size() * 4, hipMemcpyHostToDevice));
        xa.lead = dl.as<int>();
      }
    }
    for (int i = 0; i < iters; ++i) launch_xattn(xa, nullptr);
    WDR_HIP(hipDeviceSynchronize());
    std::vector<f16> h((size_t)R * d);
    WDR_HIP(hipMemcpy(h.data(), dout.p, h.size() * 2, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < h.size(); ++i) out[i] = (float)h[i];
    return 0;
  })
}

}  // extern "C"
