// Subtitle post-processing on the output path of Engine::transcribe_audio
// (src/formatting.rs process_segments, applied by src/engine.rs:192-199).  Host C++.
#pragma once
#include <string>
#include <utility>
#include <vector>

namespace wdr {

struct FmtWord {
  std::string text;
  double start = 0, end = 0;
  bool has_p = false;
  float p = 0.f;
};

struct FmtSeg {
  double start = 0, end = 0;
  std::string text;
  bool has_words = false;
  std::vector<FmtWord> words;
  bool has_speaker = false;
  std::string speaker;
};

struct PostProcessConfig {   // src/formatting.rs:94-112 defaults
  size_t max_chars_per_line = 38;
  size_t max_lines = 1;
  double cps_cap = 17.0;
  double split_gap_sec = 0.5;
  size_t comma_min_chars_before_allow = 55;
  double min_word_dur = 0.10;
  double min_sub_dur = 1.0;
  double max_sub_dur = 6.0;
  size_t soft_max_words_per_line = 0;
  bool insert_interword_space = true;
  bool use_grapheme_len = true;
  bool enforce_kinsoku = false;
  bool allow_comma_split = true;
};

PostProcessConfig config_for_language(const std::string& lang);   // presets, src/formatting.rs:139-197

// mask: VAD speech intervals (seconds) for VadMaskOracle, or nullptr for NoSilence
std::vector<FmtSeg> process_segments(const std::vector<FmtSeg>& segs, const PostProcessConfig& cfg,
                                     const std::vector<std::pair<double, double>>* mask);

}  // namespace wdr
