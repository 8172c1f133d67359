// Silero VAD model + whisper.cpp speech-segment state machine.
#pragma once
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "whisper.h"

namespace wdr {

struct VadParams {   // whisper.cpp whisper_vad_default_params + src/vad.rs:22 (min silence 100 ms)
  float threshold = 0.5f;
  int min_speech_ms = 250;
  int min_silence_ms = 100;
  float max_speech_s = 3.402823466e38f;
  int speech_pad_ms = 30;
};

class VadModel {
 public:
  // path: whisper.cpp's ggml-silero-v5.1.2.bin (model_files.cpp); "" = synthetic seeded weights
  explicit VadModel(int device, const std::string& path = std::string());
  ~VadModel();
  // speech probability per 512-sample chunk of int16 PCM (x / 32768 as src/vad.rs:11-12)
  std::vector<float> probs(const int16_t* pcm, size_t n);
  double last_scan_us_per_step = 0.0;   // LSTM chain latency of the last call
  int device;

 private:
  hipStream_t s_ = nullptr;
  DevMem w_;
  VadWeights vw_{};
  DevMem pcm_, x_, xg_, hout_, probs_;
  size_t cap_ = 0;
  hipEvent_t e0_ = nullptr, e1_ = nullptr;
};

// whisper.cpp whisper_vad_segments_from_probs: (start_cs, end_cs) pairs
std::vector<std::pair<float, float>> vad_segments_from_probs(const std::vector<float>& probs, const VadParams& p);

}  // namespace wdr
