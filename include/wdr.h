/*
 * wdr.h — C ABI of libwdr, the MI355X-native drop-in for the hot path of
 * tmoroney/whisper-diarize-rs (Engine::transcribe_audio and the five seam calls it
 * makes).
 *
 * Everything is extern "C", plain pointers and sizes; no C++ exceptions cross it.
 * Status convention: int return 0 = ok, < 0 = error; the message is kept per thread
 * and returned by wdr_last_error() (the Rust shim maps it to eyre::Report).
 *
 * Option<T> encoding: Option<bool> -> int8_t (-1 None, 0 false, 1 true);
 * Option<i32/usize/f32/f64> -> value + int8_t has_ flag; Option<String> -> nullable
 * NUL-terminated UTF-8.
 *
 * Reference interface each entry point replaces (file:line in the reference crate):
 *   wdr_engine_new / wdr_engine_free     Engine::new                      src/engine.rs:58-63
 *   wdr_transcribe_audio                 Engine::transcribe_audio         src/engine.rs:65-200
 *   wdr_read_wav                         audio::read_wav                  src/audio.rs:4-24
 *   wdr_vad_get_segments                 vad::get_segments                src/vad.rs:6-85
 *   wdr_vad_merge                        (the crate's own merge, src/vad.rs:33-84)
 *   wdr_context_create / _free           transcribe::create_context       src/transcribe.rs:89-166
 *   wdr_run_pipeline                     transcribe::run_transcription_pipeline src/transcribe.rs:323-535
 *   wdr_segment_list_free                (drop of Vec<Segment>)
 * The wdr_dbg_* functions are kernel-level test seams (parity tests call them).
 */
#ifndef WDR_H
#define WDR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WDR_ABI_VERSION 6

typedef struct wdr_engine wdr_engine;
typedef struct wdr_context wdr_context;   /* ~ whisper_rs::WhisperContext (+ its state) */

/* EngineConfig, src/engine.rs:9-18 */
typedef struct {
  const char* cache_dir;                  /* PathBuf; default "./cache" */
  int8_t enable_dtw;                      /* Option<bool>, default Some(true) */
  int8_t enable_flash_attn;               /* Option<bool>, default Some(false) */
  int8_t use_gpu;                         /* Option<bool>, default Some(true) */
  int8_t has_gpu_device;
  int32_t gpu_device;                     /* Option<i32> */
  const char* vad_model_path;             /* Option<String> */
  const char* diarize_segment_model_path; /* Option<String> */
  const char* diarize_embedding_model_path; /* Option<String> */
} wdr_engine_config;

/* AdvancedTranscribe, src/types.rs:16-24 */
typedef struct {
  const char* sampling_strategy;          /* "beam_search" | "greedy" | NULL */
  int8_t has_best_of_or_beam_size; int32_t best_of_or_beam_size;
  int8_t has_n_threads; int32_t n_threads;
  int8_t has_temperature; float temperature;
  int8_t has_max_text_ctx; int32_t max_text_ctx;
  const char* init_prompt;
  int8_t has_diarize_threshold; float diarize_threshold;
} wdr_advanced;

/* TranscribeOptions, src/types.rs:28-45 */
typedef struct {
  int8_t has_offset; double offset;       /* default Some(0.0) */
  const char* model;                      /* default "base" */
  const char* lang;                       /* default Some("auto") */
  int8_t whisper_to_english;              /* default Some(false) */
  const char* translate_target;           /* network translation: out of scope (error if set) */
  int8_t enable_vad;                      /* default Some(true) */
  int8_t enable_diarize;                  /* default None */
  int8_t has_max_speakers; uint64_t max_speakers;
  const wdr_advanced* advanced;           /* nullable */
} wdr_transcribe_options;

/* DiarizeOptions, src/types.rs:93-98: built by Engine::transcribe_audio (src/engine.rs:101-111) and
 * passed to run_transcription_pipeline, whose speaker embeddings + assignment it switches on
 * (src/transcribe.rs:339-345).  A NULL model path selects synthetic seeded weights (no model
 * files exist offline); a non-NULL path is loaded or the call fails. */
typedef struct {
  const char* segment_model_path;         /* String (segmentation-3.0.onnx) */
  const char* embedding_model_path;       /* String (wespeaker_en_voxceleb_CAM++.onnx) */
  float threshold;                        /* f32, the Engine's default 0.5 */
  uint64_t max_speakers;                  /* usize, the Engine maps None / Some(0) to usize::MAX */
} wdr_diarize_options;

/* Synthetic-weights / workload knobs (no checkpoints on this machine).
 * Not part of the reference API; NULL everywhere means defaults. */
typedef struct {
  double weight_std;                      /* default 0.02 */
  double emb_std;                         /* default 0.02 */
  float force_len_rate;                   /* >0: pin decode length (tokens per audio second) */
  int8_t disable_fallback;                /* 1: logprob/entropy fallback thresholds off */
} wdr_synthetic;

/* FormattingOverrides, src/formatting.rs:37-51 (every field optional; Option<bool> as -1/0/1) */
typedef struct {
  int8_t has_max_chars_per_line; uint64_t max_chars_per_line;
  int8_t has_max_lines; uint64_t max_lines;
  int8_t has_cps_cap; double cps_cap;
  int8_t has_split_gap_sec; double split_gap_sec;
  int8_t has_comma_min_chars_before_allow; uint64_t comma_min_chars_before_allow;
  int8_t has_min_word_dur; double min_word_dur;
  int8_t has_min_sub_dur; double min_sub_dur;
  int8_t has_max_sub_dur; double max_sub_dur;
  int8_t has_soft_max_words_per_line; uint64_t soft_max_words_per_line;
  int8_t insert_interword_space;
  int8_t use_grapheme_len;
  int8_t enforce_kinsoku;
  int8_t allow_comma_split;
} wdr_formatting_overrides;

/* WordTimestamp, src/types.rs:64-70 */
typedef struct {
  const char* text;
  double start, end;
  int8_t has_probability; float probability;
} wdr_word;

/* Segment, src/types.rs:74-82 */
typedef struct {
  double start, end;
  const char* text;
  const wdr_word* words; size_t n_words;  /* words == NULL <-> None */
  const char* speaker_id;                 /* NULL <-> None */
} wdr_segment;

typedef struct {
  wdr_segment* segments; size_t n_segments;
  const char* detected_lang;              /* Option<String> (run_transcription_pipeline's second result) */
  const int64_t* speech_index;            /* wdr_run_pipeline only: index of the input SpeechSegment each
                                             segment came from (NULL elsewhere); not in the Rust API */
} wdr_segment_list;

/* SpeechSegment, src/types.rs:86-90 (samples borrowed) */
typedef struct {
  double start, end;
  const int16_t* samples; size_t n_samples;
} wdr_speech_segment;

/* Callbacks, src/engine.rs:35-40 + src/types.rs:12-13; all fire on the calling thread */
typedef struct {
  void* user;
  void (*progress)(void* user, int32_t pct, int32_t type /*0 Download,1 Transcribe,2 Translate*/, const char* label);
  void (*new_segment)(void* user, const wdr_segment* seg);   /* borrowed for the callback only */
  int (*is_cancelled)(void* user);
} wdr_callbacks;

/* per-stage wall-clock accounting of the last run (seconds) */
typedef struct {
  double mel, encode, decode, dtw, vad, total;
  int64_t windows, decode_steps, prefills;
  double lang, prompt_gpu, embed;   /* language detect wall, prompt-prefill GPU time, speaker embeddings */
  /* multi-chain decoding (wdr_context_set_chains): chains used, batched steps launched and
   * the rows they carried, segments re-decoded by the prompt fix-up / the sampled-tail
   * replay, wall time of the speculative and the fix-up phases */
  int64_t chains, batch_launches, batch_rows, fixup_segments, replay_segments;
  double spec_s, fixup_s;
  double batch_step_s;   /* wall of the batched steps (submit -> tokens on the host), summed */
  int64_t early_fixup_segments;   /* of fixup_segments: re-decoded by the early fix-up */
  /* ABI 3: what the batched launches carried besides decode rows -- prompt-prefill rows and DTW
   * re-forward rows (and how many of each), launches holding any (eager), and the cross-K/V
   * reads: one-row / beam groups (VALU kernel) and MFMA row tiles, each one slot per layer */
  int64_t batch_prefill_rows, batch_dtw_rows, batch_prefills, batch_dtws, batch_mixed;
  int64_t batch_xattn_groups, batch_xattn_tiles;
  /* ABI 4: the DTW queue (multi-chain runs: every chain's DTW re-forwards batched off the decode
   * chain) -- passes launched, the rows they carried, windows queued */
  int64_t dtwq_passes, dtwq_rows, dtwq_jobs;
  /* ABI 5: language-detection decoder passes (lang "auto": one per encode-ahead batch, its
   * windows as one-row groups; or one SOT prefill per on-demand segment) and their rows.  A
   * multi-chain run keeps the encode-ahead pass for a plan's first batch only (WDR_LANG_PIGGYBACK,
   * default 1): later segments' detection rows ride in the batched steps and are counted there */
  int64_t lang_passes, lang_rows;
} wdr_stage_times;

const char* wdr_last_error(void);
int wdr_abi_version(void);
int wdr_device_count(void);
/* ABI 5: releases every handle the caller has not freed (engines, contexts with their worker
 * threads, VADs, diarizers, speaker managers) and the process-wide stream pools / profiler
 * buffers, while the HIP runtime is still up.  Registered with atexit() when the first handle is
 * created; a host may call it earlier.  Freeing a handle it released is a no-op.  A handle that
 * an entry point is still using on another thread (a call in flight) is not released; every entry
 * point rejects a released handle with an error, and a released handle's address is never
 * reused by a later one. */
void wdr_shutdown(void);

/* ---- Engine (whole-call drop-in) ---- */
int wdr_engine_new(const wdr_engine_config* cfg, wdr_engine** out);
void wdr_engine_free(wdr_engine* e);
/* Synthetic mode (an explicit opt-in): models the Engine cannot find on disk (ggml-<model>.bin in
 * the cache, the VAD / diarization model files) run on synthetic seeded weights.  Without it a
 * missing whisper model fails with "whisper file doesn't exist" as the reference does
 * (src/transcribe.rs:99-101), and a missing VAD / diarization model fails likewise. */
int wdr_engine_set_synthetic(wdr_engine* e, const wdr_synthetic* syn);
int wdr_transcribe_audio(wdr_engine* e, const char* audio_path, const wdr_transcribe_options* opts,
                         const wdr_formatting_overrides* fmt, const wdr_callbacks* cb, wdr_segment_list** out);

/* ---- seams ---- */
int wdr_read_wav(const char* path, int16_t** samples, size_t* n);
/* test seam (host only, no GPU): parse a VAD / diarization model file the way the models load
 * it -- kind 0 whisper.cpp Silero ggml, 1 segmentation-3.0 ONNX, 2 CAM++ ONNX -- and return its
 * tensors under the oracle's names: names_out "name:count\n" per tensor (sorted), data_out the
 * values concatenated in that order.  Free both with wdr_free. */
int wdr_dbg_model_file(int32_t kind, const char* path, char** names_out, float** data_out, size_t* n_values);
/* formatting::process_segments (src/formatting.rs:240-313) with PostProcessConfig::for_language(lang)
 * + overrides (nullable), and a VadMaskOracle over vad_mask (2 doubles per interval) when
 * has_mask (src/engine.rs:192-199).  Free the result with wdr_segment_list_free. */
int wdr_process_segments(const wdr_segment* segs, size_t n_segs, const char* lang, const wdr_formatting_overrides* ov,
                         int8_t has_mask, const double* vad_mask, size_t n_mask, wdr_segment_list** out);
void wdr_free(void* p);
int wdr_vad_merge(const double* starts_cs, const double* ends_cs, size_t n_segs, const int16_t* samples,
                  size_t n_samples, double* mask_out /* [2*n_segs] */, size_t* n_mask,
                  double* merged_out /* [2*n_segs] start,end seconds */, int64_t* merged_idx /* [2*n_segs] */,
                  size_t* n_merged);
/* Silero VAD (src/vad.rs:6-85; whisper.cpp WhisperVadContext + segments_from_samples).
 * model_path: whisper.cpp's ggml-silero-v5.1.2.bin (loaded, or the call fails); NULL selects
 * synthetic seeded weights. */
typedef struct wdr_vad wdr_vad;
int wdr_vad_create(const char* model_path, int8_t has_gpu_device, int32_t gpu_device, wdr_vad** out);
void wdr_vad_free(wdr_vad* v);
/* one probability per 512-sample chunk: probs_out[ceil(n/512)]; us_per_step (nullable) = GPU
 * time of the forward per chunk (the LSTM scan dominates) */
int wdr_vad_probs(wdr_vad* v, const int16_t* samples, size_t n, float* probs_out, double* us_per_step);
/* GPU time of the last forward per 512-sample chunk (microseconds) */
int wdr_vad_stats(wdr_vad* v, double* us_per_chunk);
/* whisper.cpp whisper_vad_segments_from_probs with the reference's params (min silence 100 ms):
 * cs_out[2*k] = start_cs, [2*k+1] = end_cs; capacity 2*n_probs */
int wdr_vad_segments_from_probs(const float* probs, size_t n_probs, float* cs_out, size_t* n_out);
/* vad::get_segments: raw mask (seconds, 2 per entry) + merged speech segments whose samples
 * point into `samples` (borrowed).  Free both arrays with wdr_free. */
int wdr_vad_get_segments(wdr_vad* v, const int16_t* samples, size_t n, double** mask_out, size_t* n_mask,
                         wdr_speech_segment** segs_out, size_t* n_segs);

/* pyannote diarization (src/engine.rs:89-122, src/transcribe.rs:339-345, 461-497):
 * segmentation-3.0 + get_segments stitching, Kaldi fbank + CMN, CAM++ embedding.
 * Paths: the ONNX files (segmentation-3.0.onnx, wespeaker_en_voxceleb_CAM++.onnx), whose
 * initializers are read by libwdr's own protobuf reader (loaded, or the call fails); NULL selects
 * synthetic seeded weights for that model. */
typedef struct wdr_diarizer wdr_diarizer;
int wdr_diarizer_create(const char* segment_model_path, const char* embedding_model_path, int8_t has_gpu_device,
                        int32_t gpu_device, wdr_diarizer** out);
void wdr_diarizer_free(wdr_diarizer* d);
/* per-frame argmax class of every 10-s window of the zero-padded input (pyannote-rs
 * find_max_index: last max): cls_out[n_windows * 589], n_windows = n / 160000 + 1;
 * logprobs_out (nullable) [n_windows][589][7] */
int wdr_diarize_frame_classes(wdr_diarizer* d, const int16_t* samples, size_t n, int32_t* cls_out, float* logprobs_out);
/* pyannote_rs::get_segments: one allocation holding the segments and copies of their samples
 * (slices of the zero-padded buffer); free with wdr_free(*segs_out) */
int wdr_diarize_get_segments(wdr_diarizer* d, const int16_t* samples, size_t n, wdr_speech_segment** segs_out,
                             size_t* n_segs);
/* the same stitching from frame classes computed elsewhere (e.g. window shards on several GPUs):
 * cls [n / 160000 + 1][589] of the n-sample file; free with wdr_free(*segs_out) */
int wdr_diarize_segments_from_classes(const int32_t* cls, size_t n_windows, const int16_t* samples, size_t n,
                                      wdr_speech_segment** segs_out, size_t* n_segs);
/* EmbeddingExtractor::compute pieces: features after CMN [T][80] (capacity n/160 + 1 rows), and
 * the 512-d embedding; ok = 0 where the reference's ONNX call fails (fewer than 400 samples) */
int wdr_diarize_fbank(wdr_diarizer* d, const int16_t* samples, size_t n, float* feats_out, size_t* n_frames);
int wdr_diarize_embedding(wdr_diarizer* d, const int16_t* samples, size_t n, float* emb_out, int8_t* ok);
/* B utterances in one batched CAM++ forward (what the pipeline's embedding worker runs):
 * emb_out [B][512], ok[b] as wdr_diarize_embedding's; bit-identical per utterance to it */
int wdr_diarize_embedding_batch(wdr_diarizer* d, const int16_t* const* samples, const size_t* n, int32_t B,
                                float* emb_out, int8_t* ok);
/* GPU time of the last segmentation / embedding call (ms) */
int wdr_diarize_stats(wdr_diarizer* d, double* seg_ms, double* emb_ms);
/* EmbeddingManager + the reference's choice of get_best_speaker_match / search_speaker
 * (src/transcribe.rs:478-497); emb NULL -> "?" (embedding error) */
typedef struct wdr_speakers wdr_speakers;
int wdr_speakers_new(int8_t has_max_speakers, uint64_t max_speakers, wdr_speakers** out);
void wdr_speakers_free(wdr_speakers* m);
int wdr_speakers_assign(wdr_speakers* m, const float* emb, int32_t dim, float threshold, char* id_out, size_t cap);

/* model_path: a whisper.cpp ggml file (missing -> "whisper file doesn't exist").  NULL model_path
 * with a non-NULL syn selects synthetic seeded weights of the named configuration; NULL with
 * NULL syn fails like a missing file. */
int wdr_context_create(const char* model_path, const char* model_name, int8_t has_gpu_device, int32_t gpu_device,
                       int8_t use_gpu, int8_t enable_dtw, int8_t enable_flash_attn, int8_t has_num_samples,
                       uint64_t num_samples, const wdr_synthetic* syn, wdr_context** out);
void wdr_context_free(wdr_context* c);
/* parse a whisper.cpp ggml model file without loading it (no GPU): hparams[11] = n_vocab,
 * n_audio_ctx, n_audio_state, n_audio_head, n_audio_layer, n_text_ctx, n_text_state, n_text_head,
 * n_text_layer, n_mels, ftype; wdr_context_create loads such a file when model_path is given */
int wdr_ggml_info(const char* path, int32_t* hparams, int64_t* n_tensors, int64_t* n_vocab_tokens);
/* diarize: NULL = no speakers (the reference's `None`); else speaker embeddings of every speech
 * segment + EmbeddingManager assignment per whisper segment */
int wdr_run_pipeline(wdr_context* c, const wdr_speech_segment* segs, size_t n_segs, const wdr_transcribe_options* opts,
                     const wdr_diarize_options* diarize, const wdr_synthetic* syn, const wdr_callbacks* cb,
                     wdr_segment_list** out);
/* run_pipeline without the cross-segment overlap clip and without speaker assignment, with
 * speech_index set: building block of the multi-GPU one-file path (wdr/distributed.py), which
 * applies both over the merged, ordered blocks of every GPU */
int wdr_run_pipeline_raw(wdr_context* c, const wdr_speech_segment* segs, size_t n_segs,
                         const wdr_transcribe_options* opts, const wdr_synthetic* syn, wdr_segment_list** out);
/* run_pipeline_raw continuing decoder 0's random-number stream (the multi-GPU one-file path,
 * wdr/distributed.py: a GPU's block of the file starts from the RNG state the blocks before it
 * left, as the reference's one state would, src/transcribe.rs:335): rng_in (NULL = the fresh
 * state's) and rng_out (malloc'd; free with wdr_free) are decoder 0's std::mt19937 state as
 * text; sampled_out[n_segs] = 1 where a segment drew random numbers (t > 0 decoders) */
int wdr_run_pipeline_block(wdr_context* c, const wdr_speech_segment* segs, size_t n_segs,
                           const wdr_transcribe_options* opts, const wdr_synthetic* syn, const char* rng_in,
                           int8_t* sampled_out, char** rng_out, wdr_segment_list** out);
void wdr_segment_list_free(wdr_segment_list* l);
/* decode chains of run_pipeline (greedy decoding): n States decode n contiguous blocks of the
 * speech segments concurrently, their greedy steps batched into one n-row step, with an exact
 * prompt-chain fix-up (results identical to one chain).  Default WDR_DECODE_CHAINS or 40,
 * capped by the context's KV pool (max chains fixed at creation).  Not in the Rust API. */
int wdr_context_set_chains(wdr_context* c, int32_t n);
/* GPUs the context runs on: gpu_device Some(d) -> 1 (device d); None -> every visible GPU (up to
 * 8; WDR_DEVICES="a,b,.." lists them), each holding the model, the decode chains spread over
 * them (chain k on GPU k % n) with the same exact prompt fix-up; device_ids (nullable) receives
 * the ordinals, at most `cap` */
int wdr_context_devices(const wdr_context* c, int32_t* n, int32_t* device_ids, int32_t cap);
/* fp8 encoder GEMMs (BASELINE configs[4]): the encoder's qkv / o / fc1 / fc2 projections on the
 * block-scaled fp8 MFMA with MX operands -- OCP e4m3 values, one E8M0 scale per 32 k (weights
 * quantised on first use, activations by the LayerNorm / GELU kernels that produce them);
 * attention, residuals, the cross-K/V projection and the decoder stay f16/f32.  Default off
 * (WDR_FP8_ENCODER=1 turns it on at creation).  Not in the Rust API. */
int wdr_context_set_encoder_fp8(wdr_context* c, int8_t on);
/* test seam: early prompt fix-up 0 off, 1 when the predecessor chain already finished, 2 always
 * (chain k waits for chain k-1 to finish, then redoes its first segments from the known prompt),
 * 3 (default) chain k waits only for chain k-1's speculative pass and redoes from the prompt it
 * left; -1 restores the WDR_EARLY_FIXUP environment default.  The fix-up rounds keep every mode
 * exact. */
int wdr_dbg_set_early_fixup(wdr_context* c, int32_t mode);
/* test seam: the diarization contractions on the f32 MFMA kernel (1, default) or the VALU f32
 * kernel (0) for every later launch in the process */
int wdr_dbg_set_gemm32(int32_t mfma);
int wdr_context_stage_times(wdr_context* c, wdr_stage_times* out);
int wdr_context_hparams(wdr_context* c, int32_t* out /* [10] */);

/* ---- live kernel timing (HIP events on the launching stream) for bench.py's roofline:
 * class 1 = MFMA GEMM (encoder / prefill / DTW projections), 2 = decoder GEMV, 3 = flash attention,
 * 4 = decoder cross-attention.  Setting a class resets the counters. */
int wdr_prof_set(int32_t cls);
/* several classes at once: bit (1 << cls) per class; read each with wdr_prof_read_class */
int wdr_prof_set_mask(int32_t mask);
int wdr_prof_read_class(int32_t cls, double* total_ms, int64_t* launches, double* algo_bytes, double* algo_flops);
/* the same sampled launches timed by the kernels' own clock (first wave start -> last wave end,
 * wall_clock64; the span rocprofv3's dispatch timestamps measure) instead of HIP events, which
 * under multi-stream concurrency also absorb the launch's wait for the GPU */
int wdr_prof_read_clock(int32_t cls, double* total_ms, int64_t* launches, double* algo_bytes, double* algo_flops);
int wdr_prof_read(double* total_ms, int64_t* launches, double* algo_bytes, double* algo_flops);

/* ---- whisper_full-level test seam: one state.full() call, raw token data ---- */
typedef struct {
  int32_t id, tid;
  float p, plog, pt, ptsum;
  int64_t t0, t1, t_dtw;
} wdr_token;
typedef struct {
  int64_t t0, t1;
  const char* text;
  const wdr_token* tokens; size_t n_tokens;
} wdr_result_seg;
int wdr_state_full(wdr_context* c, const float* samples, size_t n, const wdr_transcribe_options* opts,
                   const wdr_synthetic* syn, const char* initial_prompt, wdr_result_seg** segs, size_t* n_segs,
                   int32_t* lang_id);
void wdr_result_free(wdr_result_seg* segs, size_t n);

/* ---- kernel-level test seams (host buffers in / out) ---- */
int wdr_dbg_log_mel(wdr_context* c, const float* x, size_t n, int32_t seek, float* window_out /* [n_mels][3000] */);
int wdr_dbg_energy(const float* x, size_t n, float* out);
/* one v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3) on raw per-lane operands: a / b [64 lanes][32 B],
 * scale registers sa / sb [64] (op_sel 0), out [64 lanes][4] accumulators */
int wdr_dbg_mfma_scale(const uint8_t* a, const uint8_t* b, const int32_t* sa, const int32_t* sb, float* out);
int wdr_dbg_encode(wdr_context* c, const float* mel_window /* [n_mels][3000] */, float* enc_out /* [1500][d] */);
/* cross K/V of the last wdr_dbg_encode window: [1500][n_text_layer][2 (K, V)][d] (f16 -> f32) */
int wdr_dbg_cross_kv(wdr_context* c, float* out);
int wdr_dbg_decode(wdr_context* c, const int32_t* tokens, size_t n, float* logits_out /* [n_vocab] */);
/* prefill tokens[0..n-2], then one decode step of tokens[n-1] (its logits); the decoder-rows
 * contract makes them bit-identical to the n-token prefill's for n <= 8 (larger prefills run
 * their cross-attention on the MFMA tile kernel) */
int wdr_dbg_step(wdr_context* c, const int32_t* tokens, size_t n, float* logits_out /* [n_vocab] */);
/* whisper.cpp's logit rules + greedy pick (k_logits_process) on given logits
 * [R][n_vocab] (R <= 8); per row ctl[7] = {n_tokens, last_ts, pen_ts, has_ts, seek_delta, force_kind
 * (0 none, 1 only force_tok, 2 text only), force_tok} and a temperature; max_initial_ts /
 * suppress_blank as whisper_full_params.  Out: ids [R][2] = {id, tid}, f [R][5] = {p, log p, pt,
 * ptsum, no-speech probability} */
int wdr_dbg_logits(wdr_context* c, const float* logits, int32_t R, const int32_t* ctl, const float* temperature,
                   float max_initial_ts, int32_t suppress_blank, int32_t* ids_out, float* f_out);
/* multi-chain batched step (StepBatcher) with `rows` rows on the last encoded window, `iters`
 * times after prefilling tokens[0..n-2]: host milliseconds per step (probe seam) */
int wdr_dbg_batch_step(wdr_context* c, const int32_t* tokens, size_t n, int32_t rows, int32_t iters,
                       double* ms_per_step);
int wdr_dbg_capture(wdr_context* c, const int32_t* tokens, size_t n, float* cap_out /* [n_aheads][n][1500] */);
int wdr_dbg_dtw(const float* cap, int32_t n_heads, int32_t n_tok, int32_t n_audio, int32_t sot_len, int32_t seek,
                float* x_out /* [n_tok-sot_len-1][n_audio] */, int32_t* times_out, int32_t* n_times);
int wdr_dbg_discrete(const float* w, size_t n, uint32_t seed, int32_t n_draws, int32_t* out);
int wdr_dbg_dtw_dp(const float* x, int32_t rows, int32_t cols, int32_t seek, int32_t* times_out, int32_t* n_times);
/* fp8 (MX e4m3) encoder projection (BASELINE configs[4]): a [M][K] and w [N][K] quantised on the
 * GPU to e4m3 with one E8M0 scale per 32 k, the block-scaled fp8 MFMA GEMM, epilogue as
 * wdr_dbg_proj (7 = GELU written back as e4m3 + scales, returned dequantised); M > 64, N % 256,
 * K % 128.  The quantised bytes and the scale bytes ([rows][K/32], E8M0) are returned (nullable) */
int wdr_dbg_proj_fp8(const uint16_t* a_f16, const uint16_t* w_f16, const float* bias, int32_t M, int32_t N, int32_t K,
                     int32_t epi, float* out, uint8_t* a8_out, uint8_t* a_scale_out, uint8_t* w8_out,
                     uint8_t* w_scale_out);
int wdr_dbg_proj(const uint16_t* a_f16, const uint16_t* w_f16, const float* bias, int32_t M, int32_t N, int32_t K,
                 int32_t epi, float* out /* [M][N] f32 (f16 epilogues are widened) */);
/* epi | WDR_DBG_PROJ_ROWS: the decoder-rows kernel (any M, per-row arithmetic independent of M);
 * projections of <= 64 rows run on it anyway (0x100, the removed decode-step GEMV schedule of
 * ABI <= 4, and 0x400, a split-K residual form tried in round 4, are rejected) */
#define WDR_DBG_PROJ_ROWS 0x200
/* epi | WDR_DBG_PROJ_GEMM1: M > 64 on the register-staged reference tile (k_gemm) whatever the
 * dispatch rule picks -- the tiled GEMM family is bit-identical to it */
#define WDR_DBG_PROJ_GEMM1 0x800
/* A decoder-rows projection of LayerNorm(x) (x [M][K] f32, gamma / beta [K], K % 128 == 0, K <= 1280): fused = 1
 * normalises inside the row kernel's prologue (every workgroup its own row tiles), 0 = a separate
 * LayerNorm launch into f16 rows first; the two must agree bit for bit at every M (rows_forward
 * fuses up to 64 rows).  epi as wdr_dbg_proj (0 / 1 / 3; out [M][N] f32) */
int wdr_dbg_proj_ln(const float* x, const float* gamma, const float* beta, const uint16_t* w_f16, const float* bias,
                    int32_t M, int32_t N, int32_t K, int32_t epi, int32_t fused, float* out);
int wdr_dbg_attn(const uint16_t* q, const uint16_t* k, const uint16_t* v, int32_t Tq, int32_t Tk, int32_t n_head,
                 int32_t causal, float* out /* [Tq][n_head*64] */);
// decode-step cross-attention over 1500 keys (beam groups / per-row slots; see engine.cpp)
/* decode cross-attention probe: R rows (<= 1024) over S slots [S][1500][2 * 64 H] (K then V per key);
 * grp[r] = size of the group row r leads (0 for followers): groups above 8 rows run the decoder-
 * rows MFMA tile kernel (every row as rows_forward computes it), else the VALU split kernel */
int wdr_dbg_xattn(const uint16_t* q, const uint16_t* kv, const int32_t* row_slot, const int32_t* grp, int32_t R,
                  int32_t S, int32_t H, int32_t iters, float* out);

#ifdef __cplusplus
}
#endif
#endif /* WDR_H */
