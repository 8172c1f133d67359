// Kernel argument structs and launchers shared by the runtime (csrc/*.cpp) and kernels.
#pragma once
#include "../common.h"

namespace wdr {

struct MelArgs {
  const float* x; int n;           // segment samples (f32), unpadded
  int n_frames;                    // frames computed through the FFT: min(n_eff/160 + 1, n_len)
  int n_mels;
  const float* hann;               // [400]
  const float* cos_tab; const float* sin_tab;   // [400]: cos(2 pi k / 400), -sin(2 pi k / 400)
  const float* filters;            // [n_mels][201]
  float* mel;                      // [n_frames][n_mels] raw log10
  int* gmax;                       // ordered-int running max of the raw log-mel
};
void launch_mel(const MelArgs& a, hipStream_t s);
void launch_gmax_init(int* gmax, hipStream_t s);

struct Im2colMelArgs {
  const float* mel; int n_mels, n_fft_frames;
  const int* gmax;
  int seek;
  int kp;                          // padded K (multiple of 32)
  f16* out;                        // [3000][kp]
};
void launch_im2col_mel(const Im2colMelArgs& a, hipStream_t s);
void launch_busy(int blocks, int iters, float* sink, hipStream_t s);   // queue priming (Context)
void launch_im2col_conv2(const f16* x, int d, int nb, f16* out, hipStream_t s);   // nb windows
void launch_mel_window(const float* mel, int n_mels, int n_fft_frames, const int* gmax, int seek, float* out,
                       hipStream_t s);
void launch_energy(const float* x, int n, float* e, hipStream_t s);
void launch_i16_to_f32(const int16_t* in, int n, float* out, hipStream_t s);
void launch_synth_fill(void* dst, long long rows, int src_cols, int dst_cols, uint64_t seed, float scale, bool f16out,
                       int mode, float cval, hipStream_t s);
void launch_layernorm(const float* x, int ldx, const float* g, const float* b, f16* y, int ldy, int rows, int d,
                      hipStream_t s);
void launch_embed(const f16* E, const float* P, const int* tok, const int* pos, int R, int d, float* x, hipStream_t s);
void launch_kv_scatter(const f16* qkv, int ldqkv, int d, const int* row_seq, const int* row_pos, int R, f16* kc, f16* vc,
                       long long seq_stride, hipStream_t s);

struct LogitsCtl {
  int n_tokens;        // tokens already sampled in this sequence (0 -> initial step)
  int last_ts, pen_ts; // last / penultimate token is a timestamp (pen_ts also when < 2 tokens)
  int has_ts, seek_delta;
  int force_kind;      // 0 none, 1 only force_tok, 2 text only (synthetic workload pin)
  int force_tok;
  float temperature;
};
struct VocabIds {
  int n_vocab, eot, sot, translate, transcribe, solm, prev, nosp, not_, beg, space;
  int lang0, n_lang;
  int max_initial_tid;  // round(max_initial_ts / precision); -1 disables
  int suppress_blank;
};
constexpr int BEAM_KMAX = 8;
struct BeamCand {   // one beam-search candidate of a row: token, p, log p (id -1: none)
  int id;
  float p, plog;
};
struct TokOut {
  int id, tid;
  float p, plog, pt, ptsum;
  float nosp_prob;
  int pad;
};
void launch_logits_topk(const float* logits, int ld, const LogitsCtl* ctls, const VocabIds& v, int R, int K,
                        float* work, BeamCand* out, hipStream_t s);
void launch_logits_probs(const float* logits, int ld, const LogitsCtl* ctls, const VocabIds& v, int R, float* work,
                         float* probs, float* logprobs, hipStream_t s);
void launch_kv_copy(f16* kc, f16* vc, long long seq_stride, int nslot, int L, const int* pairs_dev, int n_pairs,
                    int n_rows, int d, hipStream_t s);
void launch_logits_process(const float* logits, int ld, const LogitsCtl* ctls, const VocabIds& v, int R, float* work,
                           TokOut* out, hipStream_t s);

void launch_dtw(const float* cap, int A, int N_tok, int Tk, int n_audio, int sot_len, int seek, float* nrm, float* x,
                int* times, int* n_times, hipStream_t s);
void launch_dtw_dp_only(const float* x, int rows, int M, int seek, int* times, int* n_times, hipStream_t s);

// attention (kernels/attn.hip)
struct FlashArgs {
  const f16* q; int ldq; long long q_bs;
  const f16* k; int ldk; long long k_bs;
  const f16* v; int ldv; long long v_bs;
  f16* o; int ldo; long long o_bs;
  float2* ml;
  int Tq, Tk, n_head;
  int causal;
  float scale;
  long long k_hs = 64, v_hs = 64;   // head stride of K / V (elements): 64 interleaved, XKV_HS cross K/V
  // split-K over keys (few query rows against 1500 cross keys): partial O (unnormalised, f32)
  // and (max, sum) per split, merged by a combine kernel.  nsplit <= 64, n_batch must be 1.
  int nsplit = 1;
  float* part_o = nullptr;     // [nsplit][Tq][n_head][64]
  float2* part_ml = nullptr;   // [nsplit][n_head][Tq]
  unsigned long long* ts = nullptr;   // live kernel clock (common.h ProfClock)
};
inline unsigned long long* prof_attach(FlashArgs& a) { return a.ts = prof_slot(); }
void launch_flash_attn(const FlashArgs& a, int n_batch, hipStream_t s);
struct DecSelfArgs {
  const f16* q; int ldq;
  const f16* kc; const f16* vc;
  long long seq_stride; int d;
  const int* row_seq; const int* row_pos;
  f16* o; int ldo;
  float scale;
};
void launch_dec_self_attn(const DecSelfArgs& a, int R, int n_head, hipStream_t s);
struct XAttnArgs {
  const f16* q; int ldq;
  const f16* k; const f16* v; int ldkv;
  int Tk, R, n_head;
  float scale;
  float* part_o;
  float2* part_ml;
  f16* o; int ldo;
  // per-row cross K/V (rows from different speech segments): row r's K at row_k[r] + layer_off
  // (device array of slot bases), its V v_off elements further; k / v unused then
  const f16* const* row_k = nullptr;
  long long layer_off = 0;
  long long v_off = 0;
  long long hs = 64;                  // head stride of K / V (elements; XKV_HS for the slots)
  unsigned long long* ts = nullptr;   // live kernel clock (common.h ProfClock)
  // row groups sharing one cross K/V (the beams of one segment in a batched step), row_k mode:
  // grp[r] = the size of the group row r leads (rows r .. r + grp[r] - 1, <= XATTN_GRP_MAX, K/V
  // at row_k[r]), 0 for the other rows of a group (device array [R]); n_grp = groups (for the
  // byte count).  Null: every row its own group; without row_k one group of all R rows (k / v)
  const int* grp = nullptr;
  int n_grp = 0;
  // with grp: the n_grp leading rows (device array), so the launch has one workgroup per group
  // and chunk instead of one per row (the other rows' workgroups would only exit)
  const int* lead = nullptr;
  // decoder rows (rows_forward): the groups of a DTW re-forward stop after its last alignment-head
  // layer -- lend[leader row] (VALU groups) / tiles[].z (MFMA tiles) is the first layer skipped
  int layer = 0;
  const int* lend = nullptr;
  // MFMA row tiles (prompt prefills / DTW re-forwards of more than XATTN_GRP_MAX rows): tile t
  // = rows tiles[t].x .. + tiles[t].y - 1 (<= 128) of one group, cross K/V at row_k[tiles[t].x]
  const int4* tiles = nullptr;
  int n_tiles = 0;
  int n_vgrp = 0;                     // VALU groups (lead list length); 0 with tiles: none
  int vgrp_max = 1;                   // largest VALU group (1: the 47-VGPR one-row kernel)
  float2* ml_out = nullptr;           // combine: (max, sum) per (row, head) for the DTW capture
};
constexpr int XATTN_GRP_MAX = 8;   // rows sharing one K/V without row_k
inline unsigned long long* prof_attach(XAttnArgs& a) { return a.ts = prof_slot(); }
void launch_xattn(const XAttnArgs& a, hipStream_t s);
struct CaptureArgs {
  const f16* q; int ldq;
  const f16* k; int ldk;
  const float2* ml;
  const int* heads;
  float* out;
  int slot0, R, Tk;
  float scale;
  long long hs = 64;                  // head stride of K (elements)
};
void launch_aheads_capture(const CaptureArgs& a, int n_sel, hipStream_t s);
// decoder rows (rows_forward): the cross-attention partials of the VALU groups and the MFMA
// tiles of one layer, then the combine of every row
void launch_xattn_rows(const XAttnArgs& a, hipStream_t s);
// alignment-head capture of rows of several DTW re-forwards (rows_forward): capture row j is
// batch row crow[j]; head-slot i of the layer lands at cdst[j] + (slot0 + i) * cstride[j]
struct CaptureRowsArgs {
  const f16* q; int ldq;
  const f16* const* row_k; long long layer_off, hs;
  const float2* ml;                   // [R][n_head] from the combine
  const int* heads;                   // this layer's alignment heads
  const int* crow; float* const* cdst; const int* cstride;
  int n_cap, slot0, Tk, n_head;
  float scale;
};
void launch_aheads_capture_rows(const CaptureRowsArgs& a, int n_sel, hipStream_t s);
void launch_layernorm_rows(const float* x, int ldx, const float* g, const float* b, f16* y, int ldy, int rows, int d,
                           const int* row_map, hipStream_t s);

// Silero VAD (kernels/vad.hip); layouts [out][in*k] f16, biases f32
struct VadWeights {
  const f16* stft;                  // [258][256]
  const f16* c0w; const float* c0b; // [128][129*3]
  const f16* c1w; const float* c1b; // [64][128*3]
  const f16* c2w; const float* c2b; // [64][64*3]
  const f16* c3w; const float* c3b; // [128][64*3]
  const f16* wih; const float* bih; // [512][128]
  const f16* whh; const float* bhh; // [512][128]
  const f16* wo;  const float* bo;  // [128], [1]
};
void launch_vad(const float* x, long long n, const VadWeights& w, float* xg, float* hout, float* probs,
                hipStream_t s);

// Diarization (kernels/diar.hip), all f32
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_LRELU = 2, ACT_SIGMOID = 3, ACT_ABS = 4 };
struct Gemm32Args {
  const float* A; int lda;           // [M][K]
  const float* B; int ldb;           // [N][K] (torch [out][in...] layout)
  float* C; int ldc;                 // [M][N]
  int M, N, K;
  const float* bias = nullptr;       // [N]
  const float* scale = nullptr;      // [N] affine after bias (inference BatchNorm)
  const float* shift = nullptr;
  const float* pro_scale = nullptr;  // [K] prologue: A' = relu(A * s + b) (BN-ReLU before a linear)
  const float* pro_shift = nullptr;
  int act = ACT_NONE;
  int accum = 0;                     // C = act(v + C_old)
};
void launch_gemm32(const Gemm32Args& a, hipStream_t s);
void set_gemm32_mfma(bool on);   // the f32 MFMA kernel (default) or the VALU one
void launch_im2col_1d(const float* X, int ldx, int T, int C, int k, int stride, int dil, int pad, int To, float* col,
                      hipStream_t s);
void launch_im2col_2d(const float* X, int T, int F, int C, int kf, int kt, int sf, int Fo, float* col, hipStream_t s);
void launch_maxpool3(const float* x, long long bs, int T, int C, int B, float* y, long long ybs, hipStream_t s);
void launch_inorm(float* y, long long bs, int T, int C, int B, const float* g, const float* beta, int act,
                  hipStream_t s);
void launch_lstm_scan(const float* xg, long long xbs, int ldxg, int T, int B, const float* whh, const float* bhh,
                      float* out, long long obs, int ldo, hipStream_t s);
void launch_logsoftmax7(float* z, int rows, int* cls, hipStream_t s);
void launch_fbank(const float* x, int T, const float* povey, const float* cos_t, const float* sin_t, const float* banks,
                  float* out, hipStream_t s);
void launch_colstats(float* x, int ld, int T, int C, int mode, float* out, hipStream_t s);
void launch_cam_context(const float* h, int ldh, int T, int C, float* out, hipStream_t s);
void launch_i16_scale(const int16_t* in, long long n, float scale, float* out, hipStream_t s);
void launch_cam_gate(const float* y, int ldy, const float* m, int T, int G, float* out, int ldo, hipStream_t s);
// batched CAM++: utterance b owns rows [off[b], off[b] + len[b]) (device arrays, off[B] = total)
struct SegRows {
  const int* off;
  const int* len;
  int B;
};
void launch_im2col_2d_b(const float* X, const SegRows& sr, int Ttot, int F, int C, int kf, int kt, int sf, int Fo,
                        float* col, hipStream_t s);
void launch_im2col_1d_b(const float* X, int ldx, const SegRows& in, const SegRows& out, int Ttot_out, int C, int k,
                        int stride, int dil, int pad, float* col, hipStream_t s);
void launch_colstats_b(float* x, int ld, const SegRows& sr, int C, int mode, float* out, hipStream_t s);
void launch_cam_context_b(const float* h, int ldh, const SegRows& sr, const int* ctx_off, int C, float* out,
                          hipStream_t s);
void launch_cam_gate_b(const float* y, int ldy, const float* m, const SegRows& sr, const int* ctx_off, int Ttot, int G,
                       float* out, int ldo, hipStream_t s);

}  // namespace wdr
