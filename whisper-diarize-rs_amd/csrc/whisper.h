// Whisper model, context and state on one MI355X (csrc side of SURVEY.md §8(a) a2-a13).
//
// Context  ~ whisper.cpp whisper_context  (created by transcribe::create_context,
//            src/transcribe.rs:89-166): hparams, vocab, weights resident in HBM,
//            DTW preset (alignment heads).
// State    ~ whisper.cpp whisper_state (ctx.create_state(), src/transcribe.rs:335):
//            device work buffers, KV caches, streams, and the host-side decode loop
//            `full()` = whisper_full_with_state as the reference drives it.
#pragma once

#include <exception>
#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "common.h"
#include "kernels/kernels.h"
#include "vocab.h"

namespace wdr {

uint64_t fnv1a64(const std::string& s);   // synthetic-weight seed of a tensor name

struct HParams {
  int n_vocab = 51864, n_audio_ctx = 1500, n_audio_state = 512, n_audio_head = 8, n_audio_layer = 6;
  int n_text_ctx = 448, n_text_state = 512, n_text_head = 8, n_text_layer = 6, n_mels = 80;
};
bool hparams_for(const std::string& name, HParams* hp);

std::vector<std::pair<int, int>> alignment_heads_for(const std::string& model_name);

// serialises device / pinned allocation and free with hipGraph captures (whisper_ctx.cpp)
std::recursive_mutex& hip_alloc_mutex();
// a stream on a dedicated hardware queue (env knob `knob`, default `def`; else priority `prio`)
hipStream_t dedicated_stream(const char* knob, bool def, int prio);
// destroys the process-wide pools of CU-masked streams (wdr_shutdown; no context may be alive)
void destroy_stream_pools();

struct DevMem {
  void* p = nullptr;
  size_t bytes = 0;
  DevMem() = default;
  explicit DevMem(size_t n);
  ~DevMem();
  DevMem(const DevMem&) = delete;
  DevMem& operator=(const DevMem&) = delete;
  DevMem(DevMem&& o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
  DevMem& operator=(DevMem&& o) noexcept;
  template <typename T> T* as() const { return (T*)p; }
};

struct EncLayer {
  f16 *w_qkv, *w_o, *w_fc1, *w_fc2;
  float *b_qkv, *b_o, *b_fc1, *b_fc2, *ln1_g, *ln1_b, *ln2_g, *ln2_b;
};
struct DecLayer {
  f16 *w_qkv, *w_o, *w_xq, *w_xo, *w_fc1, *w_fc2;
  float *b_qkv, *b_o, *b_xq, *b_xo, *b_fc1, *b_fc2;
  float *ln1_g, *ln1_b, *ln2_g, *ln2_b, *ln3_g, *ln3_b;
};

struct Model {
  HParams hp;
  int kp1 = 0;   // conv1 im2col K padded to a multiple of 32
  f16 *conv1_w = nullptr, *conv2_w = nullptr;
  float *conv1_b = nullptr, *conv2_b = nullptr, *enc_pos = nullptr, *ln_post_g = nullptr, *ln_post_b = nullptr;
  std::vector<EncLayer> enc;
  std::vector<DecLayer> dec;
  f16* w_xkv = nullptr;    // [L*2d][d]: per decoder layer cross K rows then cross V rows
  float* b_xkv = nullptr;  // [L*2d]
  f16* tok_emb = nullptr;
  float *dec_pos = nullptr, *ln_g = nullptr, *ln_b = nullptr;
  float *mel_filters = nullptr, *hann = nullptr, *cos_tab = nullptr, *sin_tab = nullptr;
  DevMem storage;
  size_t weight_bytes = 0;
};

// the encoder's fp8 plan from the environment (whisper_ctx.cpp): one nibble per layer
std::vector<uint8_t> fp8_plan_for(int n_layer);

struct ContextParams {
  bool use_gpu = true;
  int gpu_device = 0;
  bool dtw = true;
  bool flash_attn = false;
  double weight_std = 0.02;   // synthetic weights (oracle/weights.py uses the same doubles)
  double emb_std = 0.02;
};

class Context {
 public:
  // gf: weights, mel filters and vocabulary from a whisper.cpp ggml file; null: synthetic
  Context(const std::string& model_name, const HParams& hp, const ContextParams& cp,
          const class GgmlFile* gf = nullptr);
  ~Context();
  std::string name;
  ContextParams cp;
  Model model;
  Vocab vocab;
  std::vector<std::pair<int, int>> aheads;        // (layer, head) DTW preset
  std::vector<std::vector<int>> aheads_per_layer;
  DevMem aheads_dev;                              // per-layer head lists (device)
  std::vector<int> aheads_dev_off;
  hipStream_t stream = nullptr;
  hipStream_t low_prime = nullptr;   // WDR_PRIME_LOWQ (whisper_ctx.cpp)
  std::vector<hipStream_t> prime_streams;   // WDR_PRIME_POOLS (whisper_ctx.cpp)
  // self-attention KV caches of every decode chain (State), one pool so that the step
  // batcher can address rows of several chains: [L][max_chains * NSLOT][n_text_ctx][d] f16
  int max_chains = 1;
  DevMem kv_k, kv_v;
  long long kv_seq_stride = 0, kv_layer_stride = 0;   // elements per (layer, sequence) / per layer
  // multi-chain batched steps (created on demand): WDR_BATCHERS groups of chains, each its own
  // batcher and stream, so the latency-bound step chains of two groups overlap on the GPU;
  // `chain` is the State's chain index on this context
  std::vector<std::unique_ptr<class StepBatcher>> batchers;
  int n_batchers = 1;
  StepBatcher& step_batcher(int chain = 0);
  // WDR_PREFILL_SPLIT=1 (A/B): the chains' prompt prefills on a batcher (and stream) of their own
  // beside the other chains' decode steps instead of riding in them -- measured slower (711-715
  // vs 729-733 xRT: a 47-row prefill pass beside the decode steps took 13.6 ms, the chain waiting
  // for it; profiles/r04/ab_psplit.txt), so off by default (created on demand)
  std::unique_ptr<class StepBatcher> prefill_b;
  bool prefill_split = false;
  StepBatcher& prefill_batcher();
  // multi-chain runs: the windows' DTW re-forwards of every chain, batched off the decode
  // chain's critical path (DtwQueue, created on demand; WDR_DTW_QUEUE=0: they ride in the step
  // batcher's requests instead)
  std::unique_ptr<class DtwQueue> dtwq;
  class DtwQueue& dtw_queue();
  struct BatchStats {
    long long launches = 0, rows = 0, prefill_rows = 0, dtw_rows = 0, prefills = 0, dtws = 0, mixed = 0;
    long long vgroups = 0, tiles = 0;   // cross-attention groups (VALU) / row tiles (MFMA) launched
    double step_s = 0;                  // the slowest batcher's launch wall
    long long dq_passes = 0, dq_rows = 0, dq_jobs = 0;   // the DTW queue's
  };
  BatchStats batcher_stats();
  // fp8 (MX e4m3) encoder GEMMs (BASELINE configs[4]; wdr_context_set_encoder_fp8,
  // WDR_FP8_ENCODER): the encoder layers' projection weights as e4m3 with one E8M0 scale per 32 k,
  // made once on first use; the activations are quantised by their producers in the encoder
  std::atomic<bool> fp8_encoder{false};
  // which projections of which encoder layers run fp8 when fp8_encoder is on: one nibble per
  // layer, bit 0 qkv, 1 o, 2 fc1, 3 fc2 (fp8_plan_for; WDR_FP8_PLAN / WDR_FP8_PROJ /
  // WDR_FP8_F16_HEAD / WDR_FP8_F16_TAIL select other plans for the parity ablation)
  std::vector<uint8_t> fp8_plan;
  enum { F8_QKV = 1, F8_O = 2, F8_FC1 = 4, F8_FC2 = 8 };
  struct Fp8W {
    DevMem w, s;   // [N][K] e4m3, scale words [K/128][N] (byte b of word (t, n): k 128t + 32b ..)
  };
  struct Fp8Layer {
    Fp8W qkv, o, fc1, fc2;
  };
  const std::vector<Fp8Layer>& fp8_layers();   // thread-safe lazy quantisation

 private:
  std::mutex fp8_mu_;
  std::vector<Fp8Layer> fp8_layers_;
  void fp8_build();
};

struct FullParams {
  bool greedy = false;      // strategy: greedy vs beam search (src/transcribe.rs:25-33)
  int best_of = 5, beam_size = 5;
  std::string language = "auto";
  bool translate = false;
  int n_max_text_ctx = 16384;
  std::string initial_prompt;
  bool has_initial_prompt = false;
  float temperature = 0.f, temperature_inc = 0.2f;
  float entropy_thold = 2.4f, logprob_thold = -1.f, no_speech_thold = 0.6f;
  float thold_pt = 0.01f, thold_ptsum = 0.01f, max_initial_ts = 1.f, length_penalty = -1.f;
  bool suppress_blank = true, single_segment = true, token_timestamps = true;
  int max_tokens = 0;
  float force_len_rate = 0.f;   // synthetic workload pin (0 = off)
};

struct TokenData {
  int id = 0, tid = 0;
  float p = 0, plog = 0, pt = 0, ptsum = 0;
  long long t0 = -1, t1 = -1, t_dtw = -1;
  float vlen = 0;
};

struct ResultSeg {
  long long t0, t1;
  std::string text;
  std::vector<TokenData> tokens;
};

struct StageTimes {   // host wall-clock per phase (seconds), accumulated
  double mel = 0, encode = 0, decode = 0, dtw = 0, glue = 0;
  long long windows = 0, decode_steps = 0, prefills = 0;
  double lang = 0, prompt_gpu = 0;   // language-detect wall time; GPU time of the prompt prefills
  long long lang_passes = 0, lang_rows = 0;   // language-detection decoder passes and their rows
};

// Multi-chain decoding: several States ("chains", each decoding its own contiguous block of
// speech segments on its own host thread) hand their decoder work -- a decode step (one row,
// or the live beams of a segment with top-K candidates per row), a segment's prompt prefill,
// a window's DTW re-forward -- to this batcher, which runs everything submitted as ONE rows
// forward (rows.h: the weights streamed once for all rows, each row with its own KV-pool
// sequence, the rows of a request sharing their segment's cross-K/V slot) on its own stream.
// Lockstep: a batch launches once every chain inside the batcher has submitted its request.
class StepBatcher {
 public:
  explicit StepBatcher(Context& ctx);
  ~StepBatcher();
  static constexpr int kRows = 8;   // rows of one request (the beams / decoders of a segment)
  struct Req {
    int n = 1;                 // decode rows (0: none)
    int tok[kRows], seq[kRows], pos[kRows];   // seq: absolute KV-pool sequence
    LogitsCtl ctl[kRows];
    const f16* xkv = nullptr;  // the segment's cross-K/V slot (all its rows)
    VocabIds vids{};
    int K = 0;                 // beam candidates per row (0: the greedy pick only)
    TokenData out[kRows];
    BeamCand cand[kRows * BEAM_KMAX];   // [row][K]
    // prompt prefill (pn > 0): tokens ptok at positions 0.. of sequence pseq (absolute) on slot
    // pxkv; its last row's logits go through the rules with pctl -> pout, pnosp
    int pn = 0;
    const int* ptok = nullptr;
    int pseq = 0;
    const f16* pxkv = nullptr;
    LogitsCtl pctl{};
    TokenData pout;
    float pnosp = 0.f;
    BeamCand pcand[BEAM_KMAX];   // with K > 0: the top-K candidates of the prefill's logit row
    // DTW re-forward (dn > 0): tokens dtok at positions 0.. of sequence dseq on slot dxkv, the
    // alignment heads' probabilities captured into dcap ([n_aheads][dn][1500], device); the
    // cross-attention stops at layer dl_end
    int dn = 0;
    const int* dtok = nullptr;
    int dseq = 0;
    const f16* dxkv = nullptr;
    float* dcap = nullptr;
    int dl_end = 1 << 30;
    // language detection of a later segment (ln = 1): SOT at position 0 of sequence lseq on slot
    // lxkv, one row whose language logits (the n_lang tokens after SOT) come back in lout --
    // whisper.cpp's detection pass riding in a batched step instead of a pass of its own
    int ln = 0;
    int lseq = 0;
    const f16* lxkv = nullptr;
    float lout[100];
    // set by the launch that carried this request (under the batcher's lock)
    bool done = false;
    std::exception_ptr err;
  };
  void enter();
  void leave();
  void step(Req& r);           // blocks until the batch holding r has run
  void run(std::vector<Req*>& batch) { launch(batch); }   // one batch, caller's thread (test seam)
  long long launches = 0, rows = 0, prefill_rows = 0, dtw_rows = 0, prefills = 0, dtws = 0, mixed = 0;
  long long vgroups = 0, tiles = 0;
  double step_s = 0;           // wall of the launches (submit -> results on the host)
  struct Impl;

 private:
  Context& ctx_;
  std::unique_ptr<Impl> m_;
  void launch(std::vector<Req*>& batch);
};

struct Seq;           // one decoder's sequence (whisper_ctx.cpp)

// a window's DTW job in flight on the DTW stream (State::dtw_timestamps)
// one window's DTW re-forward queued to the context's DtwQueue (multi-chain runs)
struct DtwQJob {
  std::vector<int> toks;
  int seq = 0;                 // absolute KV-pool sequence (the chain's DTW sequence)
  const f16* xkv = nullptr;    // the window's cross-K/V slot
  int sot_len = 0, seek = 0, n_audio = 0;
  int* blk = nullptr;          // pinned: the times land at blk + 3 * RMAX (State::resolve_dtw)
  hipEvent_t done = nullptr;   // recorded after the times copy (the state's event)
  hipEvent_t fwd = nullptr;    // recorded after the pass: the slot's cross-K/V has been read
  bool issued = false;         // the queue has enqueued the pass and both events
  double t_submit = 0;
  size_t cap_off = 0;          // the queue's capture buffer offset (floats)
  std::exception_ptr err;      // failure of the pass that carried this job (rethrown to its waiters)
  DtwQJob();
  ~DtwQJob();
};

struct DtwTicket {
  int i0 = 0, n = 0;          // result range of the full() call that enqueued it
  int* blk = nullptr;         // pinned tokens + times
  void* event = nullptr;      // hipEvent_t
  std::shared_ptr<DtwQJob> q; // queued re-forward (null: stream-ordered on the state)
};

// The DTW re-forwards of all chains of a context as few wide passes on a stream of their own
// (dtw_rows_forward: projections on the tiled GEMM family, the pass stopping after the last
// alignment-head layer), then each window's DTW kernels.  Submitting never blocks the chain; a
// chain waits only where it needs a result: before a slot the pass reads is overwritten
// (State::top_up / on-demand encodes) and when it resolves the times at the end of its block.
// A pass starts when WDR_DTW_MIN_ROWS rows are queued (256), when the oldest job is
// WDR_DTW_AGE_MS old (50) or when a chain waits; one job per chain per pass (each chain has one
// DTW KV sequence).
class DtwQueue {
 public:
  explicit DtwQueue(Context& ctx);
  ~DtwQueue();
  DtwQueue(const DtwQueue&) = delete;
  DtwQueue& operator=(const DtwQueue&) = delete;
  void submit(const std::shared_ptr<DtwQJob>& j);
  void wait_issued(const std::shared_ptr<DtwQJob>& j);   // starts its pass at once if still queued
  bool is_issued(const std::shared_ptr<DtwQJob>& j);
  long long passes = 0, rows = 0, jobs = 0;

 private:
  struct Impl;
  std::unique_ptr<Impl> m_;
  Context& ctx_;
  void run();
  void issue(std::vector<std::shared_ptr<DtwQJob>>& batch);
};

class State {
 public:
  explicit State(Context& ctx, int chain = 0);
  ~State();
  // whisper_full_with_state on host f32 samples. Returns 0 on success.
  // job >= 0: segment `job` of the current plan (samples / n come from the plan).
  // async_dtw: leave the windows' DTW jobs in flight (take_dtw_jobs / resolve_dtw); otherwise
  // full() resolves them into result_all before returning.
  int full(const FullParams& p, const float* samples, int n, int job = -1, bool async_dtw = false);
  std::vector<DtwTicket> take_dtw_jobs();
  void alt_dtw_fence();                           // queued DTW pass reading the spare cross-K/V -> host waits
  void slot_dtw_fence(int slot, hipStream_t s);   // queued DTW pass reading the slot -> s waits
  void dtw_queue_fence(hipStream_t s);            // queued passes writing the DTW sequence -> s waits
  void resolve_dtw(DtwTicket& t, std::vector<ResultSeg>& segs);
  // encode-ahead: the pipeline's whole segment list (int16 PCM), see whisper_ctx.cpp
  void plan(const int16_t* const* pcm, const int* n, int count, bool detect_lang = false);
  void unplan();
  std::vector<ResultSeg> result_all;
  int lang_id = 0;
  StageTimes times;
  long long t_beg = 0, t_last = 0, tid_last = 0;
  std::vector<float> energy;
  int chain = 0;                // decode chain (KV pool sequences chain*NSLOT ..)
  bool batched = false;         // greedy steps go through ctx.step_batcher() (multi-chain run)
  // lang "auto": the language window 0 of this segment already detected (the engine's fix-up
  // re-decodes; -1: detect)
  int lang_hint = -1;
  bool sampled = false;         // the last full() drew random numbers (t > 0 decoders)
  void reset_rng();             // decoder 0's std::mt19937 back to its per-state seed
  std::string rng_state() const;
  void set_rng_state(const std::string& s);

  // test seams
  void compute_mel(const float* x_host, int n);
  // R-row batched step (StepBatcher) on this state's window, `iters` times: host ms per step
  double dbg_batch_step(const int* toks, int n, int R, int iters);
  void read_mel_window(int seek, float* out);              // [n_mels][3000] normalised
  hipStream_t encode_window(int seek);   // the stream it ran on (the caller synchronises)
  void encode_from_mel_window(const float* mel_window);    // [n_mels][3000] normalised, host
  void read_encoder_out(float* out);                       // [1500][d] (ln_post output, f16 -> f32)
  void read_cross_kv(float* out);                          // [1500][L][2][d] of the last encoded window
  void decode_logits(const int* toks, int n, float* logits_out);   // prefill from an empty cache
  void dbg_step(const int* toks, int n, float* logits_out);
  void dtw_capture(const int* toks, int n, float* cap_out);        // [n_aheads][n][1500]
  // the logit rules + greedy pick (k_logits_process) on host-given logits [R][n_vocab], with
  // full()'s rule constants for (max_initial_ts, suppress_blank)
  void dbg_logits(const float* logits, int R, const LogitsCtl* ctl, float max_initial_ts, bool suppress_blank,
                  TokenData* out, float* nosp);

  struct Impl;

 private:
  Context& ctx_;
  hipStream_t s_;
  std::unique_ptr<Impl> m_;
  // pieces of full()
  void top_up(int job);              // encodes through segment job + lookahead issued (waits)
  bool top_up_batch(int job);        // issue the next encode-ahead batch if allowed; false: none
  void enc_loop();                   // the encode-ahead host thread (WDR_ENC_THREAD)
  void enc_quiesce();                // no batch in flight on the encode-ahead thread
  Seq decode_sample(const std::vector<int>& prompt, const FullParams& params, float t_cur, int seek, int seek_end,
                    int Lf, int window, float* nosp);
  // pre_batched: the prompt is not prefilled yet -- its prefill rides in the first batched step
  Seq decode_beam(const std::vector<int>& prompt, const FullParams& params, float t_cur, int seek, int seek_end, int Lf,
                  int window, float* nosp, bool pre_batched = false);
  void decoder_prefill(const int* toks, int n, int seq, bool want_logits, bool capture);
  void prefill_on(const int* toks, int n, int seq, bool want_logits, bool capture, bool dtw_set, hipStream_t st,
                  const f16* xkv_base);
  void decoder_step(const int* toks, const int* seqs, const int* pos, int R);
  void step_and_sample(const int* toks, const int* seqs, const int* pos, const LogitsCtl* ctl, int R, TokenData* out,
                       int K = 0, BeamCand* cands = nullptr);
  void logits_topk(int R, int K, BeamCand* out);
  void kv_reorder(const std::vector<std::pair<int, int>>& moves, int n_rows);
  void run_logits(int R, const LogitsCtl* ctl, TokenData* out, float* nosp);
  void heuristic_timestamps(int i_segment, const FullParams& p);
  void dtw_attach(StepBatcher::Req& q);
  void dtw_after_step();
  void flush_dtw();
  void dtw_timestamps(int i_segment, int n_segments, int seek, int n_frames, const std::string& language);
};

}  // namespace wdr
