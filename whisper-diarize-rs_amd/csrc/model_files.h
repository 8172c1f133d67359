// Model files of the VAD and diarization stages, read without any runtime dependency:
//   * whisper.cpp's Silero VAD file (ggml-silero-v5.1.2.bin, ggml-org/whisper-vad,
//     src/model_manager.rs:303-319; loaded by WhisperVadContext::new, src/vad.rs:18);
//   * the two ONNX graphs pyannote-rs runs through ONNX Runtime (segmentation-3.0.onnx,
//     wespeaker_en_voxceleb_CAM++.onnx; src/engine.rs:90-91, 117, src/transcribe.rs:343, 466):
//     a hand-written protobuf-subset reader (ModelProto -> GraphProto -> NodeProto /
//     TensorProto) plus a structural mapping of the graph's parametric nodes, in execution
//     order, onto the oracle's tensor names (oracle/vad.py, oracle/diarize.py).
// Every loader returns f32 values keyed by those names; the models convert them to their
// device layouts (vad.cpp, diarize.cpp).  Errors throw std::runtime_error with the reason.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace wdr {

using TensorMap = std::map<std::string, std::vector<float>>;

// --- ONNX protobuf subset
struct OnnxTensor {
  std::vector<int64_t> dims;
  std::vector<float> data;   // FLOAT / FLOAT16 / DOUBLE / INT32 / INT64 widened to f32
  int64_t numel() const {
    int64_t n = 1;
    for (int64_t d : dims) n *= d;
    return n;
  }
};
struct OnnxNode {
  std::string op, name;
  std::vector<std::string> in, out;
  std::map<std::string, double> f;    // float attributes
  std::map<std::string, int64_t> i;   // int attributes
  std::map<std::string, std::string> s;
};
struct OnnxModel {
  explicit OnnxModel(const std::string& path);
  std::vector<OnnxNode> nodes;               // graph order (topological, as exporters write it)
  std::map<std::string, OnnxTensor> init;    // initializers + Constant node values (+ Identity aliases)
  const OnnxTensor* constant(const std::string& name) const;   // null when not a constant
};

// --- loaders (oracle tensor names; see each function for the mapping)
TensorMap load_silero_ggml(const std::string& path);
TensorMap load_segmentation_onnx(const std::string& path);
TensorMap load_campplus_onnx(const std::string& path);

}  // namespace wdr
