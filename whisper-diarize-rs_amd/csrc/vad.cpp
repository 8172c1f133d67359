// Silero VAD host side: synthetic weights in HBM, the three-kernel forward, and the
// probability -> segment state machine.  Mirrors oracle/vad.py (test-only restatement).
#include "vad.h"

#include <climits>
#include <cmath>

#include "model_files.h"
#include "prof.h"

namespace wdr {

namespace {
struct VadLayout {
  size_t stft, c0w, c1w, c2w, c3w, wih, whh, wo;         // f16 element offsets
  size_t c0b, c1b, c2b, c3b, bih, bhh, bo;               // f32 element offsets (after the f16 block)
  size_t n16, n32;
};
VadLayout layout() {
  VadLayout L{};
  size_t o = 0;
  auto h = [&](size_t n) { size_t r = o; o += (n + 7) / 8 * 8; return r; };
  L.stft = h(258 * 256); L.c0w = h(128 * 387); L.c1w = h(64 * 384); L.c2w = h(64 * 192); L.c3w = h(128 * 192);
  L.wih = h(512 * 128); L.whh = h(512 * 128); L.wo = h(128);
  L.n16 = o;
  o = 0;
  auto f = [&](size_t n) { size_t r = o; o += (n + 3) / 4 * 4; return r; };
  L.c0b = f(128); L.c1b = f(64); L.c2b = f(64); L.c3b = f(128); L.bih = f(512); L.bhh = f(512); L.bo = f(4);
  L.n32 = o;
  return L;
}
}  // namespace

VadModel::VadModel(int dev, const std::string& path) : device(dev) {
  const TensorMap file = path.empty() ? TensorMap() : load_silero_ggml(path);   // before any GPU work
  WDR_HIP(hipSetDevice(dev));
  WDR_HIP(hipStreamCreateWithFlags(&s_, hipStreamNonBlocking));
  stream_note("vad", s_);
  WDR_HIP(hipEventCreate(&e0_));
  WDR_HIP(hipEventCreate(&e1_));
  const VadLayout L = layout();
  w_ = DevMem(L.n16 * 2 + L.n32 * 4);
  f16* b16 = w_.as<f16>();
  float* b32 = reinterpret_cast<float*>(b16 + L.n16);
  // STFT basis: Hann-windowed real DFT (silero forward_basis_buffer), computed in double
  std::vector<f16> basis(258 * 256);
  const double pi = 3.14159265358979323846;
  for (int k = 0; k < 129; ++k)
    for (int t = 0; t < 256; ++t) {
      const double hann = 0.5 - 0.5 * std::cos(2.0 * pi * t / 256.0);
      const double ang = 2.0 * pi * k * t / 256.0;
      basis[k * 256 + t] = (f16)(std::cos(ang) * hann);
      basis[(129 + k) * 256 + t] = (f16)(-std::sin(ang) * hann);
    }
  std::vector<std::vector<f16>> staged16;   // file mode: host images kept alive until the sync below
  std::vector<std::vector<float>> staged32;
  if (!file.empty()) {
    const std::vector<float>& b = file.at("stft");
    for (size_t i = 0; i < basis.size(); ++i) basis[i] = (f16)b[i];
  }
  WDR_HIP(wdr_memcpy_async(b16 + L.stft, basis.data(), basis.size() * 2, hipMemcpyHostToDevice, s_));
  const double sq3 = std::sqrt(3.0);
  // synthetic: seeded on the GPU; file: the tensor of that name (f16 matrices, f32 biases)
  auto fill = [&](void* dst, const std::string& nm, int n, bool is16, double sd) {
    if (file.empty()) {
      launch_synth_fill(dst, 1, n, n, fnv1a64(nm), (float)(sd * sq3), is16, 0, 0.f, s_);
      return;
    }
    const std::vector<float>& v = file.at(nm);
    WDR_CHECK((int)v.size() == n, "VAD model: tensor size mismatch");
    if (is16) {
      staged16.emplace_back(v.begin(), v.end());
      WDR_HIP(wdr_memcpy_async(dst, staged16.back().data(), (size_t)n * 2, hipMemcpyHostToDevice, s_));
    } else {
      staged32.push_back(v);
      WDR_HIP(wdr_memcpy_async(dst, staged32.back().data(), (size_t)n * 4, hipMemcpyHostToDevice, s_));
    }
  };
  const char* cn[4] = {"_model.encoder.0.reparam_conv", "_model.encoder.1.reparam_conv",
                       "_model.encoder.2.reparam_conv", "_model.encoder.3.reparam_conv"};
  const int co[4] = {128, 64, 64, 128}, ci[4] = {129, 128, 64, 64};
  const size_t wo[4] = {L.c0w, L.c1w, L.c2w, L.c3w}, bo[4] = {L.c0b, L.c1b, L.c2b, L.c3b};
  for (int i = 0; i < 4; ++i) {
    fill(b16 + wo[i], std::string(cn[i]) + ".weight", co[i] * ci[i] * 3, true, 1.0 / std::sqrt((double)ci[i] * 3));
    fill(b32 + bo[i], std::string(cn[i]) + ".bias", co[i], false, 0.02);
  }
  fill(b16 + L.wih, "_model.decoder.rnn.weight_ih", 512 * 128, true, 1.0 / std::sqrt(128.0));
  fill(b16 + L.whh, "_model.decoder.rnn.weight_hh", 512 * 128, true, 1.0 / std::sqrt(128.0));
  fill(b32 + L.bih, "_model.decoder.rnn.bias_ih", 512, false, 0.05);
  fill(b32 + L.bhh, "_model.decoder.rnn.bias_hh", 512, false, 0.05);
  fill(b16 + L.wo, "_model.decoder.decoder.2.weight", 128, true, 3.0);
  fill(b32 + L.bo, "_model.decoder.decoder.2.bias", 1, false, 0.02);
  WDR_HIP(hipStreamSynchronize(s_));
  vw_ = VadWeights{b16 + L.stft, b16 + L.c0w, b32 + L.c0b, b16 + L.c1w, b32 + L.c1b, b16 + L.c2w, b32 + L.c2b,
                   b16 + L.c3w, b32 + L.c3b, b16 + L.wih, b32 + L.bih, b16 + L.whh, b32 + L.bhh, b16 + L.wo,
                   b32 + L.bo};
}

VadModel::~VadModel() {
  if (e0_) (void)hipEventDestroy(e0_);
  if (e1_) (void)hipEventDestroy(e1_);
  if (s_) (void)hipStreamDestroy(s_);
}

std::vector<float> VadModel::probs(const int16_t* pcm, size_t n) {
  WDR_HIP(hipSetDevice(device));
  const size_t nc = (n + 511) / 512;
  std::vector<float> out(nc);
  if (nc == 0) return out;
  if (n > cap_) {
    pcm_ = DevMem(n * 2);
    x_ = DevMem(n * 4);
    xg_ = DevMem(nc * 512 * 4);
    hout_ = DevMem(nc * 128 * 4);
    probs_ = DevMem(nc * 4);
    cap_ = n;
  }
  WDR_CHECK(n < (size_t)INT_MAX, "VAD: input too long");
  WDR_HIP(wdr_memcpy_async(pcm_.p, pcm, n * 2, hipMemcpyHostToDevice, s_));
  launch_i16_to_f32(pcm_.as<int16_t>(), (int)n, x_.as<float>(), s_);
  WDR_HIP(hipEventRecord(e0_, s_));
  launch_vad(x_.as<float>(), (long long)n, vw_, xg_.as<float>(), hout_.as<float>(), probs_.as<float>(), s_);
  WDR_HIP(hipEventRecord(e1_, s_));
  WDR_HIP(wdr_memcpy_async(out.data(), probs_.p, nc * 4, hipMemcpyDeviceToHost, s_));
  WDR_HIP(hipStreamSynchronize(s_));
  float ms = 0.f;
  WDR_HIP(hipEventElapsedTime(&ms, e0_, e1_));
  last_scan_us_per_step = ms * 1e3 / (double)nc;
  return out;
}

// whisper.cpp whisper_vad_segments_from_probs (port of silero get_speech_timestamps)
std::vector<std::pair<float, float>> vad_segments_from_probs(const std::vector<float>& probs, const VadParams& P) {
  const int SR = 16000, NW = 512;
  const int n = (int)probs.size();
  const int min_sil = SR * P.min_silence_ms / 1000;
  const int audio_len = n * NW;
  const int min_speech = SR * P.min_speech_ms / 1000;
  const int pad = SR * P.speech_pad_ms / 1000;
  int max_speech;
  if (P.max_speech_s > 100000.0f) {
    max_speech = INT_MAX / 2;
  } else {
    const int64_t tmp = (int64_t)SR * (int64_t)P.max_speech_s - NW - 2 * pad;
    max_speech = (tmp > INT_MAX || tmp < 0) ? INT_MAX / 2 : (int)tmp;
  }
  const int min_sil_at_max = SR * 98 / 1000;
  float neg = P.threshold - 0.15f;
  if (neg < 0.01f) neg = 0.01f;
  struct Sp { int s, e; };
  std::vector<Sp> sp;
  bool in_speech = false, has_cur = false;
  int temp_end = 0, prev_end = 0, next_start = 0, cur_start = 0;
  for (int i = 0; i < n; ++i) {
    const float pr = probs[i];
    const int cs = NW * i;
    if (pr >= P.threshold && temp_end) {
      temp_end = 0;
      if (next_start < prev_end) next_start = cs;
    }
    if (pr >= P.threshold && !in_speech) {
      in_speech = true;
      cur_start = cs;
      has_cur = true;
      continue;
    }
    if (in_speech && cs - cur_start > max_speech) {
      if (prev_end) {
        sp.push_back({cur_start, prev_end});
        has_cur = true;
        if (next_start < prev_end) {
          in_speech = false;
          has_cur = false;
        } else {
          cur_start = next_start;
        }
        prev_end = next_start = temp_end = 0;
      } else {
        sp.push_back({cur_start, cs});
        prev_end = next_start = temp_end = 0;
        in_speech = false;
        has_cur = false;
        continue;
      }
    }
    if (pr < neg && in_speech) {
      if (!temp_end) temp_end = cs;
      if (cs - temp_end > min_sil_at_max) prev_end = temp_end;
      if (cs - temp_end < min_sil) continue;
      if (temp_end - cur_start > min_speech) sp.push_back({cur_start, temp_end});
      prev_end = next_start = temp_end = 0;
      in_speech = false;
      has_cur = false;
      continue;
    }
  }
  if (has_cur && audio_len - cur_start > min_speech) sp.push_back({cur_start, audio_len});
  for (int i = 0; i + 1 < (int)sp.size(); ++i) {
    if (sp[i + 1].s - sp[i].e < (int)(SR * 0.2)) {
      sp[i].e = sp[i + 1].e;
      sp.erase(sp.begin() + i + 1);
      --i;
    }
  }
  for (int i = 0; i < (int)sp.size(); ++i)
    if (sp[i].e - sp[i].s < min_speech) {
      sp.erase(sp.begin() + i);
      --i;
    }
  std::vector<std::pair<float, float>> out;
  for (int i = 0; i < (int)sp.size(); ++i) {
    if (i == 0) sp[i].s = sp[i].s > pad ? sp[i].s - pad : 0;
    if (i + 1 < (int)sp.size()) {
      const int sil = sp[i + 1].s - sp[i].e;
      if (sil < 2 * pad) {
        sp[i].e += sil / 2;
        sp[i + 1].s = sp[i + 1].s > sil / 2 ? sp[i + 1].s - sil / 2 : 0;
      } else {
        sp[i].e = sp[i].e + pad < audio_len ? sp[i].e + pad : audio_len;
        sp[i + 1].s = sp[i + 1].s > pad ? sp[i + 1].s - pad : 0;
      }
    } else {
      sp[i].e = sp[i].e + pad < audio_len ? sp[i].e + pad : audio_len;
    }
    out.push_back({(float)sp[i].s / (float)SR * 100.0f, (float)sp[i].e / (float)SR * 100.0f});
  }
  return out;
}

}  // namespace wdr
