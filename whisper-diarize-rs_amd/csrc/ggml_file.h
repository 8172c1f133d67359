// whisper.cpp ggml model file (the `ggml-<model>.bin` files the reference's model manager
// caches, src/model_manager.rs:148-299, loaded by whisper-rs at src/transcribe.rs:154):
//   magic 0x67676d6c, 11 int32 hparams (n_vocab, n_audio_ctx, n_audio_state, n_audio_head,
//   n_audio_layer, n_text_ctx, n_text_state, n_text_head, n_text_layer, n_mels, ftype),
//   mel filters (int32 n_mel, int32 n_fft, f32[n_mel][n_fft]), vocabulary (int32 n, then n x
//   (int32 len, bytes)), then tensors until EOF: int32 n_dims, int32 name_len, int32 type,
//   int32 ne[n_dims] (ne[0] innermost), name bytes, data (type 0 = f32, 1 = f16).
// Memory-mapped read-only; tensors are converted when they are uploaded (whisper_ctx.cpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace wdr {

struct GgmlTensor {
  int type = 0;                 // 0 f32, 1 f16
  std::vector<int64_t> ne;      // ne[0] innermost
  const char* data = nullptr;   // inside the mapping
  int64_t n_elem() const {
    int64_t n = 1;
    for (int64_t x : ne) n *= x;
    return n;
  }
};

class GgmlFile {
 public:
  explicit GgmlFile(const std::string& path);   // throws std::runtime_error("failed to open model: ...")
  ~GgmlFile();
  GgmlFile(const GgmlFile&) = delete;
  GgmlFile& operator=(const GgmlFile&) = delete;

  int32_t hp[11] = {};                  // n_vocab .. n_mels, ftype
  int n_mel = 0, n_fft = 0;
  std::vector<float> filters;           // [n_mel][n_fft]
  std::vector<std::string> vocab;       // the file's token texts (ids 0..n-1)
  std::map<std::string, GgmlTensor> tensors;

  const GgmlTensor& get(const std::string& name) const;   // throws if absent
  // tensor `name` as f32 / f16 values (row-major, element count checked against n)
  std::vector<float> as_f32(const std::string& name, int64_t n) const;
  std::vector<uint16_t> as_f16(const std::string& name, int64_t n) const;

 private:
  void* map_ = nullptr;
  size_t size_ = 0;
};

}  // namespace wdr
