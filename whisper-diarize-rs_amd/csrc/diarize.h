// Diarization models on the GPU: pyannote segmentation-3.0 +
// get_segments stitching, Kaldi fbank + CMN, CAM++ speaker embedding, EmbeddingManager.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "whisper.h"

namespace wdr {

// host copy of the seeded synthetic generator (oracle/weights.py synth_f32): bit-identical
std::vector<float> synth_f32_host(const std::string& name, size_t n, double std);

struct DiarSegment {   // pyannote_rs::Segment
  double start, end;
  size_t start_idx, end_idx;   // into the zero-padded buffer
};

// pyannote_rs::get_segments' stitching of per-window frame classes [n/160000 + 1][589] of an
// n-sample file (the classes may come from several GPUs' window shards)
std::vector<DiarSegment> diar_stitch(const std::vector<int>& cls, size_t n);

class SegModel {
 public:
  // path: segmentation-3.0.onnx (model_files.cpp); "" = synthetic seeded weights
  explicit SegModel(int device, const std::string& path = std::string());
  ~SegModel();
  // per-window frame classes (argmax, last max on ties) of the zero-padded file:
  // [n_windows][589]; optionally the log-probabilities [n_windows][589][7]
  std::vector<int> frame_classes(const int16_t* pcm, size_t n, std::vector<float>* logprobs = nullptr);
  // pyannote_rs::get_segments (src/engine.rs:117-122)
  std::vector<DiarSegment> get_segments(const int16_t* pcm, size_t n);
  double last_ms = 0.0;
  int device;

 private:
  struct W;
  W* w_ = nullptr;
  hipStream_t s_ = nullptr;
  hipEvent_t e0_ = nullptr, e1_ = nullptr;
};

class CamModel {
 public:
  // path: wespeaker_en_voxceleb_CAM++.onnx (model_files.cpp); "" = synthetic seeded weights
  explicit CamModel(int device, const std::string& path = std::string());
  ~CamModel();
  // EmbeddingExtractor::compute: i16 -> /32768 -> fbank -> CMN -> CAM++ -> [512].
  // Returns false where the reference's ORT call fails (fewer than 400 samples: no frames).
  bool embed(const int16_t* pcm, size_t n, float* emb_out);
  // B utterances in one batched forward: emb_out[b * 512 ..], ok[b] = embed()'s return value
  // (bit-identical per utterance to embed())
  void embed_batch(const int16_t* const* pcm, const size_t* n, int B, float* emb_out, char* ok);
  // fbank after CMN, [T][80] (test seam)
  std::vector<float> feats(const int16_t* pcm, size_t n);
  double last_ms = 0.0;
  int device;

 private:
  struct W;
  W* w_ = nullptr;
  hipStream_t s_ = nullptr;
  hipEvent_t e0_ = nullptr, e1_ = nullptr;
  int T_cap_ = 0, T2_cap_ = 0, nseg_cap_ = 0;
  void ensure(int T, int T2tot, int nsegtot);
  int run_fbank(const int16_t* pcm, size_t n);
};

// pyannote_rs::EmbeddingManager + the reference's choice between get_best_speaker_match and
// search_speaker (src/transcribe.rs:478-497).  Ids are visited in ascending order.
class SpeakerManager {
 public:
  explicit SpeakerManager(uint64_t max_speakers) : max_(max_speakers) {}
  std::string assign(const float* emb, int dim, float threshold);   // "?" when no speaker
  size_t n_speakers() const { return spk_.size(); }

 private:
  uint64_t max_;
  std::map<int, std::vector<float>> spk_;
  int next_ = 1;
};

}  // namespace wdr
