// Whisper vocabulary: special ids, token text, tokenizer (csrc side).
// Restates whisper.cpp whisper_vocab + tokenize() (initial prompt, src/transcribe.rs:384-386);
// synthetic file vocabulary identical to oracle/vocab.py.
#pragma once
#include <string>
#include <unordered_map>
#include <vector>

namespace wdr {

extern const char* const kLangs[100];

struct Vocab {
  int n_vocab = 0;
  bool multilingual = false;
  int num_languages = 0;
  int eot, sot, translate, transcribe, solm, prev, nosp, not_, beg;
  std::vector<std::string> id_to_token;
  std::unordered_map<std::string, int> token_to_id;

  explicit Vocab(int n_vocab);
  int token_lang(int lang_id) const { return sot + 1 + lang_id; }
  std::vector<int> tokenize(const std::string& text) const;
  static std::vector<std::string> split_words(const std::string& text);
};

int lang_id_from_str(const std::string& s);   // -1 if unknown

}  // namespace wdr
