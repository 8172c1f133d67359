// Diarization host side: synthetic weights, the segmentation / embedding forwards as kernel
// sequences, pyannote-rs stitching and the speaker manager.  Mirrors oracle/diarize.py
// (test-only restatement); reference call sites src/engine.rs:117-122 and
// src/transcribe.rs:339-345, 461-497.
#include "diarize.h"

#include <cmath>
#include <array>
#include <cstring>

#include "model_files.h"
#include "prof.h"

namespace wdr {

static uint64_t splitmix64_host(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

std::vector<float> synth_f32_host(const std::string& name, size_t n, double std) {
  const uint64_t seed = fnv1a64(name);
  const float scale = (float)(std * std::sqrt(3.0));
  std::vector<float> v(n);
  for (size_t i = 0; i < n; ++i) {
    const uint64_t h = splitmix64_host(seed + (uint64_t)i);
    const float u = (float)(uint32_t)(h >> 40) * 1.1920928955078125e-07f - 1.0f;
    v[i] = u * scale;
  }
  return v;
}

namespace {
// one device arena filled from host vectors
struct Arena {
  std::vector<float> host;
  size_t add(const std::vector<float>& v) {
    const size_t off = host.size();
    host.insert(host.end(), v.begin(), v.end());
    host.resize((host.size() + 63) / 64 * 64, 0.f);
    return off;
  }
};
std::vector<float> plus_one(std::vector<float> v) {
  for (auto& x : v) x = x + 1.0f;
  return v;
}
}  // namespace

// ================================================================== segmentation-3.0
static constexpr int kWin = 160000, kFrames = 589, kFrameStart = 721, kFrameSize = 270;
static constexpr int kSegBatch = 128;  // windows per forward: the BiLSTM scans run one workgroup per (window, direction), so 128 windows fill the GPU (16 left 224 of 256 CUs idle for the whole scan)
static constexpr float kClass0Offset = 0.86f;   // oracle/diarize.py SEG_CLASS0_OFFSET

struct SegModel::W {
  DevMem arena;
  const float *wn_g, *wn_b, *sinc, *ng[3], *nb[3], *c1w, *c1b, *c2w, *c2b, *wih[4], *bih[4], *whh[4], *bhh[4];
  const float *l0w, *l0b, *l1w, *l1b, *cw, *cb;
  DevMem pcm, x, col, s1, p1, s2, p2, s3, p3, xg, h0, h1, la, lb, z, cls;
};

SegModel::SegModel(int dev, const std::string& path) : device(dev) {
  // segmentation-3.0.onnx (model_files.cpp), or the seeded synthetic weights of oracle/diarize.py
  const TensorMap file = path.empty() ? TensorMap() : load_segmentation_onnx(path);
  auto get = [&](const std::string& n, size_t cnt, double sd, bool plus1) {
    if (file.empty()) return plus1 ? plus_one(synth_f32_host("seg." + n, cnt, sd)) : synth_f32_host("seg." + n, cnt, sd);
    const std::vector<float>& v = file.at(n);
    WDR_CHECK(v.size() == cnt, "segmentation model: tensor " + n + " size mismatch");
    return v;
  };
  WDR_HIP(hipSetDevice(dev));
  WDR_HIP(hipStreamCreateWithFlags(&s_, hipStreamNonBlocking));
  stream_note("seg", s_);
  WDR_HIP(hipEventCreate(&e0_));
  WDR_HIP(hipEventCreate(&e1_));
  w_ = new W;
  Arena A;
  auto f = [&](const std::string& n, size_t cnt, double sd) { return A.add(get(n, cnt, sd, false)); };
  auto one = [&](const std::string& n, size_t cnt) { return A.add(get(n, cnt, 0.1, true)); };
  size_t o_wng = one("wav_norm.weight", 1), o_wnb = f("wav_norm.bias", 1, 0.1);
  size_t o_sinc = f("sinc.weight", 80 * 251, 1.0 / std::sqrt(251.0));
  size_t o_ng[3], o_nb[3];
  const int nc[3] = {80, 60, 60};
  for (int i = 0; i < 3; ++i) {
    o_ng[i] = one("norm" + std::to_string(i) + ".weight", nc[i]);
    o_nb[i] = f("norm" + std::to_string(i) + ".bias", nc[i], 0.1);
  }
  size_t o_c1w = f("conv1.weight", 60 * 80 * 5, 1.0 / std::sqrt(400.0)), o_c1b = f("conv1.bias", 60, 0.05);
  size_t o_c2w = f("conv2.weight", 60 * 60 * 5, 1.0 / std::sqrt(300.0)), o_c2b = f("conv2.bias", 60, 0.05);
  size_t o_wih[4], o_bih[4], o_whh[4], o_bhh[4];
  for (int l = 0; l < 4; ++l) {
    const int I = l == 0 ? 60 : 256;
    const std::string L = std::to_string(l);
    // both directions stacked: rows [0,512) forward, [512,1024) reverse
    std::vector<float> wih = get("lstm.weight_ih_l" + L, 512 * I, 1.0 / std::sqrt(128.0), false);
    std::vector<float> wr = get("lstm.weight_ih_l" + L + "_reverse", 512 * I, 1.0 / std::sqrt(128.0), false);
    wih.insert(wih.end(), wr.begin(), wr.end());
    o_wih[l] = A.add(wih);
    std::vector<float> bih = get("lstm.bias_ih_l" + L, 512, 0.05, false);
    std::vector<float> br = get("lstm.bias_ih_l" + L + "_reverse", 512, 0.05, false);
    bih.insert(bih.end(), br.begin(), br.end());
    o_bih[l] = A.add(bih);
    std::vector<float> whh = get("lstm.weight_hh_l" + L, 512 * 128, 1.0 / std::sqrt(128.0), false);
    std::vector<float> whr = get("lstm.weight_hh_l" + L + "_reverse", 512 * 128, 1.0 / std::sqrt(128.0), false);
    whh.insert(whh.end(), whr.begin(), whr.end());
    o_whh[l] = A.add(whh);
    std::vector<float> bhh = get("lstm.bias_hh_l" + L, 512, 0.05, false);
    std::vector<float> bhr = get("lstm.bias_hh_l" + L + "_reverse", 512, 0.05, false);
    bhh.insert(bhh.end(), bhr.begin(), bhr.end());
    o_bhh[l] = A.add(bhh);
  }
  size_t o_l0w = f("linear0.weight", 128 * 256, 1.0 / std::sqrt(256.0)), o_l0b = f("linear0.bias", 128, 0.05);
  size_t o_l1w = f("linear1.weight", 128 * 128, 1.0 / std::sqrt(128.0)), o_l1b = f("linear1.bias", 128, 0.05);
  size_t o_cw = f("classifier.weight", 7 * 128, 8.0 / std::sqrt(128.0));
  std::vector<float> cb = get("classifier.bias", 7, 0.05, false);
  if (file.empty()) cb[0] = cb[0] + kClass0Offset;   // synthetic calibration only (oracle/diarize.py)
  size_t o_cb = A.add(cb);
  W& w = *w_;
  w.arena = DevMem(A.host.size() * 4);
  WDR_HIP(hipMemcpy(w.arena.p, A.host.data(), A.host.size() * 4, hipMemcpyHostToDevice));
  const float* b = w.arena.as<float>();
  w.wn_g = b + o_wng; w.wn_b = b + o_wnb; w.sinc = b + o_sinc;
  for (int i = 0; i < 3; ++i) { w.ng[i] = b + o_ng[i]; w.nb[i] = b + o_nb[i]; }
  w.c1w = b + o_c1w; w.c1b = b + o_c1b; w.c2w = b + o_c2w; w.c2b = b + o_c2b;
  for (int l = 0; l < 4; ++l) { w.wih[l] = b + o_wih[l]; w.bih[l] = b + o_bih[l]; w.whh[l] = b + o_whh[l]; w.bhh[l] = b + o_bhh[l]; }
  w.l0w = b + o_l0w; w.l0b = b + o_l0b; w.l1w = b + o_l1w; w.l1b = b + o_l1b; w.cw = b + o_cw; w.cb = b + o_cb;
  const size_t B = kSegBatch;
  w.pcm = DevMem(B * kWin * 2);
  w.x = DevMem(B * kWin * 4);
  w.col = DevMem(B * 15975 * 251 * 4);
  w.s1 = DevMem(B * 15975 * 80 * 4);
  w.p1 = DevMem(B * 5325 * 80 * 4);
  w.s2 = DevMem(B * 5321 * 60 * 4);
  w.p2 = DevMem(B * 1773 * 60 * 4);
  w.s3 = DevMem(B * 1769 * 60 * 4);
  w.p3 = DevMem(B * kFrames * 60 * 4);
  w.xg = DevMem(B * kFrames * 1024 * 4);
  w.h0 = DevMem(B * kFrames * 256 * 4);
  w.h1 = DevMem(B * kFrames * 256 * 4);
  w.la = DevMem(B * kFrames * 128 * 4);
  w.lb = DevMem(B * kFrames * 128 * 4);
  w.z = DevMem(B * kFrames * 7 * 4);
  w.cls = DevMem(B * kFrames * 4);
}

SegModel::~SegModel() {
  delete w_;
  if (e0_) (void)hipEventDestroy(e0_);
  if (e1_) (void)hipEventDestroy(e1_);
  if (s_) (void)hipStreamDestroy(s_);
}

static void gemm(hipStream_t s, const float* A, int lda, const float* B, int ldb, float* C, int ldc, int M, int N, int K,
                 const float* bias, int act, const float* scale = nullptr, const float* shift = nullptr,
                 const float* pro_s = nullptr, const float* pro_b = nullptr, int accum = 0) {
  Gemm32Args a{A, lda, B, ldb, C, ldc, M, N, K};
  a.bias = bias;
  a.scale = scale;
  a.shift = shift;
  a.pro_scale = pro_s;
  a.pro_shift = pro_b;
  a.act = act;
  a.accum = accum;
  launch_gemm32(a, s);
}

std::vector<int> SegModel::frame_classes(const int16_t* pcm, size_t n, std::vector<float>* logprobs) {
  WDR_HIP(hipSetDevice(device));
  W& w = *w_;
  const size_t padded = n + (kWin - n % kWin);
  const int nw = (int)(padded / kWin);
  std::vector<int> cls((size_t)nw * kFrames);
  if (logprobs) logprobs->assign((size_t)nw * kFrames * 7, 0.f);
  WDR_HIP(hipEventRecord(e0_, s_));
  for (int w0 = 0; w0 < nw; w0 += kSegBatch) {
    const int B = std::min(kSegBatch, nw - w0);
    // windows of the zero-padded buffer: raw int16 values as f32 (no 1/32768)
    WDR_HIP(wdr_memset_async(w.pcm.p, 0, (size_t)B * kWin * 2, s_));
    const size_t s0 = (size_t)w0 * kWin;
    const size_t avail = s0 < n ? std::min(n - s0, (size_t)B * kWin) : 0;
    if (avail) WDR_HIP(wdr_memcpy_async(w.pcm.p, pcm + s0, avail * 2, hipMemcpyHostToDevice, s_));
    launch_i16_scale(w.pcm.as<int16_t>(), (long long)B * kWin, 1.0f, w.x.as<float>(), s_);
    launch_inorm(w.x.as<float>(), kWin, kWin, 1, B, w.wn_g, w.wn_b, ACT_NONE, s_);
    // SincNet
    for (int b = 0; b < B; ++b)
      launch_im2col_1d(w.x.as<float>() + (size_t)b * kWin, 1, kWin, 1, 251, 10, 1, 0, 15975,
                       w.col.as<float>() + (size_t)b * 15975 * 251, s_);
    gemm(s_, w.col.as<float>(), 251, w.sinc, 251, w.s1.as<float>(), 80, B * 15975, 80, 251, nullptr, ACT_ABS);
    launch_maxpool3(w.s1.as<float>(), 15975ll * 80, 15975, 80, B, w.p1.as<float>(), 5325ll * 80, s_);
    launch_inorm(w.p1.as<float>(), 5325ll * 80, 5325, 80, B, w.ng[0], w.nb[0], ACT_LRELU, s_);
    for (int b = 0; b < B; ++b)
      launch_im2col_1d(w.p1.as<float>() + (size_t)b * 5325 * 80, 80, 5325, 80, 5, 1, 1, 0, 5321,
                       w.col.as<float>() + (size_t)b * 5321 * 400, s_);
    gemm(s_, w.col.as<float>(), 400, w.c1w, 400, w.s2.as<float>(), 60, B * 5321, 60, 400, w.c1b, ACT_NONE);
    launch_maxpool3(w.s2.as<float>(), 5321ll * 60, 5321, 60, B, w.p2.as<float>(), 1773ll * 60, s_);
    launch_inorm(w.p2.as<float>(), 1773ll * 60, 1773, 60, B, w.ng[1], w.nb[1], ACT_LRELU, s_);
    for (int b = 0; b < B; ++b)
      launch_im2col_1d(w.p2.as<float>() + (size_t)b * 1773 * 60, 60, 1773, 60, 5, 1, 1, 0, 1769,
                       w.col.as<float>() + (size_t)b * 1769 * 300, s_);
    gemm(s_, w.col.as<float>(), 300, w.c2w, 300, w.s3.as<float>(), 60, B * 1769, 60, 300, w.c2b, ACT_NONE);
    launch_maxpool3(w.s3.as<float>(), 1769ll * 60, 1769, 60, B, w.p3.as<float>(), (long long)kFrames * 60, s_);
    launch_inorm(w.p3.as<float>(), (long long)kFrames * 60, kFrames, 60, B, w.ng[2], w.nb[2], ACT_LRELU, s_);
    // 4 x BiLSTM: input projections of both directions in one GEMM, then the scans
    const float* in = w.p3.as<float>();
    int in_dim = 60;
    float* hb[2] = {w.h0.as<float>(), w.h1.as<float>()};
    for (int l = 0; l < 4; ++l) {
      gemm(s_, in, in_dim, w.wih[l], in_dim, w.xg.as<float>(), 1024, B * kFrames, 1024, in_dim, w.bih[l], ACT_NONE);
      launch_lstm_scan(w.xg.as<float>(), (long long)kFrames * 1024, 1024, kFrames, B, w.whh[l], w.bhh[l], hb[l & 1],
                       (long long)kFrames * 256, 256, s_);
      in = hb[l & 1];
      in_dim = 256;
    }
    gemm(s_, in, 256, w.l0w, 256, w.la.as<float>(), 128, B * kFrames, 128, 256, w.l0b, ACT_LRELU);
    gemm(s_, w.la.as<float>(), 128, w.l1w, 128, w.lb.as<float>(), 128, B * kFrames, 128, 128, w.l1b, ACT_LRELU);
    gemm(s_, w.lb.as<float>(), 128, w.cw, 128, w.z.as<float>(), 7, B * kFrames, 7, 128, w.cb, ACT_NONE);
    launch_logsoftmax7(w.z.as<float>(), B * kFrames, w.cls.as<int>(), s_);
    WDR_HIP(wdr_memcpy_async(cls.data() + (size_t)w0 * kFrames, w.cls.p, (size_t)B * kFrames * 4, hipMemcpyDeviceToHost,
                           s_));
    if (logprobs)
      WDR_HIP(wdr_memcpy_async(logprobs->data() + (size_t)w0 * kFrames * 7, w.z.p, (size_t)B * kFrames * 7 * 4,
                             hipMemcpyDeviceToHost, s_));
    WDR_HIP(hipStreamSynchronize(s_));   // host staging of the next batch reuses the buffers
  }
  WDR_HIP(hipEventRecord(e1_, s_));
  WDR_HIP(hipStreamSynchronize(s_));
  float ms = 0.f;
  WDR_HIP(hipEventElapsedTime(&ms, e0_, e1_));
  last_ms = ms;
  return cls;
}

// pyannote_rs::get_segments: frame k of the file sits at sample 721 + 270 k (continuing across
// windows); a run of argmax != 0 frames becomes a segment when a class-0 frame follows.  The
// lazy iterator yields one queued segment per window and stops at the first window whose
// queue is empty (restated as published).
std::vector<DiarSegment> SegModel::get_segments(const int16_t* pcm, size_t n) {
  return diar_stitch(frame_classes(pcm, n), n);
}

std::vector<DiarSegment> diar_stitch(const std::vector<int>& cls, size_t n) {
  const size_t padded = n + (kWin - n % kWin);
  const size_t nw = padded / kWin;
  size_t offset = kFrameStart;
  bool speaking = false;
  double start_offset = 0.0;
  std::vector<DiarSegment> queue, out;
  size_t qh = 0;
  for (size_t w = 0; w < nw; ++w) {
    for (int k = 0; k < kFrames; ++k) {
      if (cls[w * kFrames + k] != 0) {
        if (!speaking) {
          start_offset = (double)offset;
          speaking = true;
        }
      } else if (speaking) {
        const double start = start_offset / 16000.0, end = (double)offset / 16000.0;
        const size_t si = (size_t)std::min(start * 16000.0, (double)(padded - 1));
        const size_t ei = (size_t)std::min(end * 16000.0, (double)padded);
        speaking = false;
        queue.push_back({start, end, si, ei});
      }
      offset += kFrameSize;
    }
    if (qh < queue.size()) {
      out.push_back(queue[qh++]);
    } else {
      return out;
    }
  }
  for (; qh < queue.size(); ++qh) out.push_back(queue[qh]);
  return out;
}

// ================================================================== fbank + CAM++
static constexpr int kCamBlocks[3][3] = {{12, 3, 1}, {24, 3, 2}, {16, 3, 2}};

struct CamModel::W {
  DevMem arena;
  // fbank tables
  const float *povey, *cos_t, *sin_t, *banks;
  // FCM
  const float *c1, *bn1s, *bn1b;
  struct Res {
    const float *w1, *s1, *b1, *w2, *s2, *b2, *sc, *scs, *scb;
  } res[4];
  const float *c2, *bn2s, *bn2b;
  const float *tdnn, *tds, *tdb;
  struct Layer {
    const float *s1, *b1, *lin1, *s2, *b2, *local, *cam1w, *cam1b, *cam2w, *cam2b;
  };
  std::vector<Layer> layers[3];
  const float *trs[3], *trb[3], *trw[3];
  const float *outs, *outb, *dense, *dens, *denb;
  // activations
  DevMem pcm, x, fb, a, b, r, col, XA, XB, h, y, ctx, c1buf, m, st, emb;
  DevMem tab;                 // batched runs: utterance row tables (SegRows) + context offsets
  int* h_tab = nullptr;       // pinned staging of tab
  int tab_cap = 0;            // utterances
  int B_cap = 0;              // st / emb rows
  size_t pcm_cap = 0;         // samples
};

static double mel_k(double f) { return 1127.0 * std::log(1.0 + f / 700.0); }

CamModel::CamModel(int dev, const std::string& path) : device(dev) {
  // wespeaker_en_voxceleb_CAM++.onnx (model_files.cpp), or the seeded synthetic weights
  const TensorMap file = path.empty() ? TensorMap() : load_campplus_onnx(path);
  auto get = [&](const std::string& n, size_t cnt, double sd, bool plus1) {
    if (file.empty()) return plus1 ? plus_one(synth_f32_host("cam." + n, cnt, sd)) : synth_f32_host("cam." + n, cnt, sd);
    const std::vector<float>& v = file.at(n);
    WDR_CHECK(v.size() == cnt, "embedding model: tensor " + n + " size mismatch");
    return v;
  };
  WDR_HIP(hipSetDevice(dev));
  // lowest priority: embeddings run beside the latency-bound decode chain (EmbedAhead)
  int lo = 0, hi = 0;
  WDR_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
  WDR_HIP(hipStreamCreateWithPriority(&s_, hipStreamNonBlocking, lo));
  stream_note("cam", s_);
  WDR_HIP(hipEventCreate(&e0_));
  WDR_HIP(hipEventCreate(&e1_));
  w_ = new W;
  Arena A;
  // Kaldi tables (double math, stored f32)
  std::vector<float> pov(400), ct(512), st(512), banks(80 * 256, 0.f);
  const double pi = 3.14159265358979323846;
  for (int i = 0; i < 400; ++i) pov[i] = (float)std::pow(0.5 - 0.5 * std::cos(2.0 * pi * i / 399.0), 0.85);
  for (int i = 0; i < 512; ++i) {
    ct[i] = (float)std::cos(2.0 * pi * i / 512.0);
    st[i] = (float)std::sin(2.0 * pi * i / 512.0);
  }
  {
    const double ml = mel_k(20.0), mh = mel_k(8000.0), delta = (mh - ml) / 81.0;
    for (int bnk = 0; bnk < 80; ++bnk) {
      const double left = ml + bnk * delta, center = ml + (bnk + 1) * delta, right = ml + (bnk + 2) * delta;
      for (int i = 0; i < 256; ++i) {
        const double m = mel_k(31.25 * i);
        if (m > left && m < right)
          banks[bnk * 256 + i] = (float)(m <= center ? (m - left) / (center - left) : (right - m) / (right - center));
      }
    }
  }
  size_t o_pov = A.add(pov), o_ct = A.add(ct), o_st = A.add(st), o_banks = A.add(banks);
  auto f = [&](const std::string& n, size_t cnt, double sd) { return A.add(get(n, cnt, sd, false)); };
  auto bn = [&](const std::string& n, size_t c, size_t* s, size_t* b) {
    *s = A.add(get(n + ".scale", c, 0.1, true));
    *b = A.add(get(n + ".shift", c, 0.1, false));
  };
  const int m = 32;
  size_t o_c1 = f("head.conv1", m * 9, 1.0 / 3.0), o_bn1s, o_bn1b;
  bn("head.bn1", m, &o_bn1s, &o_bn1b);
  size_t o_res[4][9];
  for (int L = 1; L <= 2; ++L)
    for (int bb = 0; bb < 2; ++bb) {
      const std::string p = "head.layer" + std::to_string(L) + "." + std::to_string(bb);
      size_t* o = o_res[(L - 1) * 2 + bb];
      o[0] = f(p + ".conv1", m * m * 9, 1.0 / std::sqrt(9.0 * m));
      bn(p + ".bn1", m, &o[1], &o[2]);
      o[3] = f(p + ".conv2", m * m * 9, 1.0 / std::sqrt(9.0 * m));
      bn(p + ".bn2", m, &o[4], &o[5]);
      if (bb == 0) {
        o[6] = f(p + ".shortcut", m * m, 1.0 / std::sqrt((double)m));
        bn(p + ".shortcut_bn", m, &o[7], &o[8]);
      } else {
        o[6] = o[7] = o[8] = 0;
      }
    }
  size_t o_c2 = f("head.conv2", m * m * 9, 1.0 / std::sqrt(9.0 * m)), o_bn2s, o_bn2b;
  bn("head.bn2", m, &o_bn2s, &o_bn2b);
  // TDNN weight: torch input channel c*10 + f, ours (FCM output [T][F][C]) f*32 + c
  size_t o_tdnn;
  {
    std::vector<float> wt = get("tdnn.linear", 128 * 320 * 5, 1.0 / std::sqrt(320.0 * 5), false);
    std::vector<float> wp(wt.size());
    for (int o = 0; o < 128; ++o)
      for (int c = 0; c < 32; ++c)
        for (int fq = 0; fq < 10; ++fq)
          for (int j = 0; j < 5; ++j)
            wp[((size_t)o * 320 + fq * 32 + c) * 5 + j] = wt[((size_t)o * 320 + c * 10 + fq) * 5 + j];
    o_tdnn = A.add(wp);
  }
  size_t o_tds, o_tdb;
  bn("tdnn.bn", 128, &o_tds, &o_tdb);
  std::vector<std::vector<std::array<size_t, 10>>> o_layers(3);
  size_t o_tr[3][3];
  int ch = 128;
  for (int bi = 0; bi < 3; ++bi) {
    const int nl = kCamBlocks[bi][0], k = kCamBlocks[bi][1];
    for (int li = 0; li < nl; ++li) {
      const std::string p = "block" + std::to_string(bi + 1) + "." + std::to_string(li);
      const int cin = ch + li * 32;
      std::array<size_t, 10> o;
      bn(p + ".bn1", cin, &o[0], &o[1]);
      o[2] = f(p + ".linear1", 128 * (size_t)cin, 1.0 / std::sqrt((double)cin));
      bn(p + ".bn2", 128, &o[3], &o[4]);
      o[5] = f(p + ".local", 32 * 128 * (size_t)k, 1.0 / std::sqrt(128.0 * k));
      o[6] = f(p + ".cam1.weight", 64 * 128, 1.0 / std::sqrt(128.0));
      o[7] = f(p + ".cam1.bias", 64, 0.05);
      o[8] = f(p + ".cam2.weight", 32 * 64, 1.0 / std::sqrt(64.0));
      o[9] = f(p + ".cam2.bias", 32, 0.05);
      o_layers[bi].push_back(o);
    }
    ch += nl * 32;
    bn("transit" + std::to_string(bi + 1) + ".bn", ch, &o_tr[bi][0], &o_tr[bi][1]);
    o_tr[bi][2] = f("transit" + std::to_string(bi + 1) + ".linear", (size_t)(ch / 2) * ch, 1.0 / std::sqrt((double)ch));
    ch /= 2;
  }
  size_t o_outs, o_outb, o_dens, o_denb;
  bn("out.bn", ch, &o_outs, &o_outb);
  size_t o_dense = f("dense.linear", 512 * 2 * (size_t)ch, 1.0 / std::sqrt(2.0 * ch));
  bn("dense.bn", 512, &o_dens, &o_denb);
  W& w = *w_;
  w.arena = DevMem(A.host.size() * 4);
  WDR_HIP(hipMemcpy(w.arena.p, A.host.data(), A.host.size() * 4, hipMemcpyHostToDevice));
  const float* b = w.arena.as<float>();
  w.povey = b + o_pov; w.cos_t = b + o_ct; w.sin_t = b + o_st; w.banks = b + o_banks;
  w.c1 = b + o_c1; w.bn1s = b + o_bn1s; w.bn1b = b + o_bn1b;
  for (int i = 0; i < 4; ++i) {
    const size_t* o = o_res[i];
    w.res[i] = {b + o[0], b + o[1], b + o[2], b + o[3], b + o[4], b + o[5], o[6] ? b + o[6] : nullptr,
                o[7] ? b + o[7] : nullptr, o[8] ? b + o[8] : nullptr};
  }
  w.c2 = b + o_c2; w.bn2s = b + o_bn2s; w.bn2b = b + o_bn2b;
  w.tdnn = b + o_tdnn; w.tds = b + o_tds; w.tdb = b + o_tdb;
  for (int bi = 0; bi < 3; ++bi) {
    for (auto& o : o_layers[bi])
      w.layers[bi].push_back({b + o[0], b + o[1], b + o[2], b + o[3], b + o[4], b + o[5], b + o[6], b + o[7], b + o[8],
                              b + o[9]});
    w.trs[bi] = b + o_tr[bi][0]; w.trb[bi] = b + o_tr[bi][1]; w.trw[bi] = b + o_tr[bi][2];
  }
  w.outs = b + o_outs; w.outb = b + o_outb; w.dense = b + o_dense; w.dens = b + o_dens; w.denb = b + o_denb;
  w.st = DevMem(1024 * 4);
  w.emb = DevMem(512 * 4);
}

CamModel::~CamModel() {
  if (s_) (void)hipStreamSynchronize(s_);
  if (w_ && w_->h_tab) (void)hipHostFree(w_->h_tab);
  delete w_;
  if (e0_) (void)hipEventDestroy(e0_);
  if (e1_) (void)hipEventDestroy(e1_);
  if (s_) (void)hipStreamDestroy(s_);
}

void CamModel::ensure(int T, int T2tot, int nsegtot) {
  if (T <= T_cap_ && T2tot <= T2_cap_ && nsegtot <= nseg_cap_) return;
  T = std::max(T, T_cap_);
  T2tot = std::max(T2tot, T2_cap_);
  nsegtot = std::max(nsegtot, nseg_cap_);
  W& w = *w_;
  const size_t t = (size_t)T;
  const size_t t2 = (size_t)T2tot + 2;
  w.fb = DevMem(t * 80 * 4);
  w.a = DevMem(t * 80 * 32 * 4);
  w.b = DevMem(t * 80 * 32 * 4);
  w.r = DevMem(t * 80 * 32 * 4);
  w.col = DevMem(std::max(t * 40 * 288, t2 * 1600) * 4);
  w.XA = DevMem(t2 * 1024 * 4);
  w.XB = DevMem(t2 * 1024 * 4);
  w.h = DevMem(t2 * 128 * 4);
  w.y = DevMem(t2 * 32 * 4);
  const size_t nseg = (size_t)nsegtot + 1;
  w.ctx = DevMem(nseg * 128 * 4);
  w.c1buf = DevMem(nseg * 64 * 4);
  w.m = DevMem(nseg * 32 * 4);
  T_cap_ = T;
  T2_cap_ = T2tot;
  nseg_cap_ = nsegtot;
}

int CamModel::run_fbank(const int16_t* pcm, size_t n) {
  W& w = *w_;
  const int T = n < 400 ? 0 : (int)(1 + (n - 400) / 160);
  if (T == 0) return 0;
  ensure(T, (T - 1) / 2 + 1, ((T - 1) / 2 + 1 + 99) / 100);
  if (w.pcm.bytes < n * 2) {
    w.pcm = DevMem(n * 2);
    w.x = DevMem(n * 4);
  }
  WDR_HIP(wdr_memcpy_async(w.pcm.p, pcm, n * 2, hipMemcpyHostToDevice, s_));
  launch_i16_scale(w.pcm.as<int16_t>(), (long long)n, 1.0f / 32768.0f, w.x.as<float>(), s_);
  launch_fbank(w.x.as<float>(), T, w.povey, w.cos_t, w.sin_t, w.banks, w.fb.as<float>(), s_);
  launch_colstats(w.fb.as<float>(), 80, T, 80, 0, nullptr, s_);   // CMN
  return T;
}

std::vector<float> CamModel::feats(const int16_t* pcm, size_t n) {
  WDR_HIP(hipSetDevice(device));
  const int T = run_fbank(pcm, n);
  std::vector<float> out((size_t)T * 80);
  if (T) WDR_HIP(wdr_memcpy_async(out.data(), w_->fb.p, out.size() * 4, hipMemcpyDeviceToHost, s_));
  WDR_HIP(hipStreamSynchronize(s_));
  return out;
}

bool CamModel::embed(const int16_t* pcm, size_t n, float* emb_out) {
  char ok = 0;
  embed_batch(&pcm, &n, 1, emb_out, &ok);
  return ok != 0;
}

// Several utterances in one forward: their fbank rows are concatenated, every GEMM runs over
// all utterances' rows at once (the per-utterance convs, CMN, CAM context and stats pooling use
// the batched kernels' row tables).  Per utterance the arithmetic is exactly the one-utterance
// forward's, so each embedding is bit-identical to embed() of that utterance alone.
void CamModel::embed_batch(const int16_t* const* pcm, const size_t* n, int B, float* emb_out, char* ok) {
  WDR_HIP(hipSetDevice(device));
  W& w = *w_;
  WDR_HIP(hipEventRecord(e0_, s_));
  // utterances with frames (fewer than 400 samples: the reference's ORT call fails -> no embedding)
  std::vector<int> idx, T, T2, ns;
  size_t nsamp = 0;
  for (int i = 0; i < B; ++i) {
    ok[i] = 0;
    const int t = n[i] < 400 ? 0 : (int)(1 + (n[i] - 400) / 160);
    if (t == 0) continue;
    idx.push_back(i);
    T.push_back(t);
    T2.push_back((t + 4 - 5) / 2 + 1);
    ns.push_back((T2.back() + 99) / 100);
    nsamp += n[i];
  }
  const int Bv = (int)idx.size();
  if (Bv == 0) return;
  // row tables: offT[Bv+1] lenT[Bv] offT2[Bv+1] lenT2[Bv] ctxoff[Bv+1]
  const int tab_n = 5 * Bv + 3;
  if (w.tab_cap < Bv) {
    std::lock_guard<std::recursive_mutex> g(hip_alloc_mutex());   // not during another thread's capture
    if (w.h_tab) (void)hipHostFree(w.h_tab);
    WDR_HIP(hipHostMalloc((void**)&w.h_tab, (size_t)tab_n * 4, hipHostMallocDefault));
    w.tab = DevMem((size_t)tab_n * 4);
    w.tab_cap = Bv;
  }
  WDR_HIP(hipStreamSynchronize(s_));   // the pinned table may still feed the previous batch's copy
  int* offT = w.h_tab;
  int* lenT = offT + Bv + 1;
  int* offT2 = lenT + Bv;
  int* lenT2 = offT2 + Bv + 1;
  int* ctxoff = lenT2 + Bv;
  offT[0] = offT2[0] = ctxoff[0] = 0;
  for (int b = 0; b < Bv; ++b) {
    lenT[b] = T[b];
    lenT2[b] = T2[b];
    offT[b + 1] = offT[b] + T[b];
    offT2[b + 1] = offT2[b] + T2[b];
    ctxoff[b + 1] = ctxoff[b] + ns[b];
  }
  const int Tt = offT[Bv], T2t = offT2[Bv], nst = ctxoff[Bv];
  ensure(Tt, T2t, nst);
  if (w.B_cap < Bv) {
    w.st = DevMem((size_t)Bv * 1024 * 4);
    w.emb = DevMem((size_t)Bv * 512 * 4);
    w.B_cap = Bv;
  }
  if (w.pcm_cap < nsamp) {
    w.pcm = DevMem(nsamp * 2);
    w.x = DevMem(nsamp * 4);
    w.pcm_cap = nsamp;
  }
  WDR_HIP(wdr_memcpy_async(w.tab.p, w.h_tab, (size_t)tab_n * 4, hipMemcpyHostToDevice, s_));
  const int* d = w.tab.as<int>();
  const SegRows sT{d, d + Bv + 1, Bv};
  const SegRows sT2{d + 2 * Bv + 1, d + 3 * Bv + 2, Bv};
  const int* dctx = d + 4 * Bv + 2;
  // i16 -> /32768 -> fbank per utterance into its rows, then CMN per utterance
  {
    size_t so = 0;
    for (int b = 0; b < Bv; ++b) {
      const int i = idx[b];
      WDR_HIP(wdr_memcpy_async(w.pcm.as<int16_t>() + so, pcm[i], n[i] * 2, hipMemcpyHostToDevice, s_));
      so += n[i];
    }
    launch_i16_scale(w.pcm.as<int16_t>(), (long long)nsamp, 1.0f / 32768.0f, w.x.as<float>(), s_);
    so = 0;
    for (int b = 0; b < Bv; ++b) {
      launch_fbank(w.x.as<float>() + so, T[b], w.povey, w.cos_t, w.sin_t, w.banks, w.fb.as<float>() + (size_t)offT[b] * 80,
                   s_);
      so += n[idx[b]];
    }
    launch_colstats_b(w.fb.as<float>(), 80, sT, 80, 0, nullptr, s_);
  }
  float* col = w.col.as<float>();
  // ---- FCM over [T][F][C]
  launch_im2col_2d_b(w.fb.as<float>(), sT, Tt, 80, 1, 3, 3, 1, 80, col, s_);
  gemm(s_, col, 9, w.c1, 9, w.a.as<float>(), 32, Tt * 80, 32, 9, nullptr, ACT_RELU, w.bn1s, w.bn1b);
  float* cur = w.a.as<float>();
  float* tmp = w.b.as<float>();
  float* res = w.r.as<float>();
  int F = 80;
  for (int i = 0; i < 4; ++i) {
    const W::Res& R = w.res[i];
    const int sf = (i % 2 == 0) ? 2 : 1;
    const int Fo = sf == 2 ? (F + 2 - 3) / 2 + 1 : F;
    // y = relu(bn1(conv1(x)))
    launch_im2col_2d_b(cur, sT, Tt, F, 32, 3, 3, sf, Fo, col, s_);
    gemm(s_, col, 288, R.w1, 288, tmp, 32, Tt * Fo, 32, 288, nullptr, ACT_RELU, R.s1, R.b1);
    // shortcut into res
    if (R.sc) {
      launch_im2col_2d_b(cur, sT, Tt, F, 32, 1, 1, 2, Fo, col, s_);
      gemm(s_, col, 32, R.sc, 32, res, 32, Tt * Fo, 32, 32, nullptr, ACT_NONE, R.scs, R.scb);
    } else {
      WDR_HIP(wdr_memcpy_async(res, cur, (size_t)Tt * Fo * 32 * 4, hipMemcpyDeviceToDevice, s_));
    }
    // out = relu(bn2(conv2(y)) + shortcut)
    launch_im2col_2d_b(tmp, sT, Tt, Fo, 32, 3, 3, 1, Fo, col, s_);
    gemm(s_, col, 288, R.w2, 288, res, 32, Tt * Fo, 32, 288, nullptr, ACT_RELU, R.s2, R.b2, nullptr, nullptr, 1);
    std::swap(cur, res);
    F = Fo;
  }
  // conv2 (stride 2 in frequency) + bn2 + relu: [T][10][32] == [T][320] (column f*32 + c)
  launch_im2col_2d_b(cur, sT, Tt, F, 32, 3, 3, 2, 10, col, s_);
  gemm(s_, col, 288, w.c2, 288, tmp, 32, Tt * 10, 32, 288, nullptr, ACT_RELU, w.bn2s, w.bn2b);
  // ---- TDNN k5 s2 p2 -> X [T2][1024] (ld 1024)
  launch_im2col_1d_b(tmp, 320, sT, sT2, T2t, 320, 5, 2, 1, 2, col, s_);
  float* X = w.XA.as<float>();
  float* Y = w.XB.as<float>();
  gemm(s_, col, 1600, w.tdnn, 1600, X, 1024, T2t, 128, 1600, nullptr, ACT_RELU, w.tds, w.tdb);
  int ch = 128;
  for (int bi = 0; bi < 3; ++bi) {
    const int nl = kCamBlocks[bi][0], k = kCamBlocks[bi][1], dil = kCamBlocks[bi][2];
    for (int li = 0; li < nl; ++li) {
      const W::Layer& Lr = w.layers[bi][li];
      const int cin = ch + li * 32;
      // h = relu(bn2(linear1(relu(bn1(x)))))
      gemm(s_, X, 1024, Lr.lin1, cin, w.h.as<float>(), 128, T2t, 128, cin, nullptr, ACT_RELU, Lr.s2, Lr.b2, Lr.s1,
           Lr.b1);
      // y = local conv (k3, dilation)
      launch_im2col_1d_b(w.h.as<float>(), 128, sT2, sT2, T2t, 128, k, 1, dil, (k - 1) / 2 * dil, col, s_);
      gemm(s_, col, 128 * k, Lr.local, 128 * k, w.y.as<float>(), 32, T2t, 32, 128 * k, nullptr, ACT_NONE);
      // m = sigmoid(W2 relu(W1 (mean + segment mean) + b1) + b2), one row per 100-frame segment
      launch_cam_context_b(w.h.as<float>(), 128, sT2, dctx, 128, w.ctx.as<float>(), s_);
      gemm(s_, w.ctx.as<float>(), 128, Lr.cam1w, 128, w.c1buf.as<float>(), 64, nst, 64, 128, Lr.cam1b, ACT_RELU);
      gemm(s_, w.c1buf.as<float>(), 64, Lr.cam2w, 64, w.m.as<float>(), 32, nst, 32, 64, Lr.cam2b, ACT_SIGMOID);
      launch_cam_gate_b(w.y.as<float>(), 32, w.m.as<float>(), sT2, dctx, T2t, 32, X + cin, 1024, s_);
    }
    ch += nl * 32;
    // transit: linear(relu(bn(x))) -> ch/2 channels; after the last block, out_nonlinear
    // (BN + ReLU) is fused into the epilogue
    if (bi < 2) {
      gemm(s_, X, 1024, w.trw[bi], ch, Y, 1024, T2t, ch / 2, ch, nullptr, ACT_NONE, nullptr, nullptr, w.trs[bi],
           w.trb[bi]);
    } else {
      gemm(s_, X, 1024, w.trw[bi], ch, Y, 1024, T2t, ch / 2, ch, nullptr, ACT_RELU, w.outs, w.outb, w.trs[bi],
           w.trb[bi]);
    }
    std::swap(X, Y);
    ch /= 2;
  }
  // stats pooling + dense + BN (one row per utterance)
  launch_colstats_b(X, 1024, sT2, ch, 1, w.st.as<float>(), s_);
  gemm(s_, w.st.as<float>(), 2 * ch, w.dense, 2 * ch, w.emb.as<float>(), 512, Bv, 512, 2 * ch, nullptr, ACT_NONE,
       w.dens, w.denb);
  std::vector<float> e((size_t)Bv * 512);
  WDR_HIP(wdr_memcpy_async(e.data(), w.emb.p, e.size() * 4, hipMemcpyDeviceToHost, s_));
  WDR_HIP(hipEventRecord(e1_, s_));
  WDR_HIP(hipStreamSynchronize(s_));
  for (int b = 0; b < Bv; ++b) {
    memcpy(emb_out + (size_t)idx[b] * 512, e.data() + (size_t)b * 512, 512 * 4);
    ok[idx[b]] = 1;
  }
  float ms = 0.f;
  WDR_HIP(hipEventElapsedTime(&ms, e0_, e1_));
  last_ms = ms;
}

// ================================================================== speakers
static float cosine(const float* a, const float* b, int n) {
  float dot = 0.f, na = 0.f, nb = 0.f;
  for (int i = 0; i < n; ++i) {
    dot += a[i] * b[i];
    na += a[i] * a[i];
    nb += b[i] * b[i];
  }
  return dot / (std::sqrt(na) * std::sqrt(nb));
}

std::string SpeakerManager::assign(const float* emb, int dim, float threshold) {
  if (!emb) return "?";
  if ((uint64_t)spk_.size() == max_) {
    // get_best_speaker_match
    if (spk_.empty()) return "?";
    int best = 0;
    float best_sim = -INFINITY;
    for (auto& kv : spk_) {
      const float s = cosine(emb, kv.second.data(), dim);
      if (s > best_sim) {
        best = kv.first;
        best_sim = s;
      }
    }
    return std::to_string(best);
  }
  // search_speaker
  int best = -1;
  float best_sim = threshold;
  for (auto& kv : spk_) {
    const float s = cosine(emb, kv.second.data(), dim);
    if (s > best_sim) {
      best = kv.first;
      best_sim = s;
    }
  }
  if (best < 0 && (uint64_t)spk_.size() < max_) {
    best = next_++;
    spk_[best] = std::vector<float>(emb, emb + dim);
  }
  return best < 0 ? "?" : std::to_string(best);
}

}  // namespace wdr
