#include "vocab.h"

#include <cctype>
#include <cstdio>
#include <cstring>

namespace wdr {

const char* const kLangs[100] = {
    "en", "zh", "de", "es", "ru", "ko", "fr", "ja", "pt", "tr", "pl", "ca", "nl", "ar", "sv", "it", "id",
    "hi", "fi", "vi", "he", "uk", "el", "ms", "cs", "ro", "da", "hu", "ta", "no", "th", "ur", "hr", "bg",
    "lt", "la", "mi", "ml", "cy", "sk", "te", "fa", "lv", "bn", "sr", "az", "sl", "kn", "et", "mk", "br",
    "eu", "is", "hy", "ne", "mn", "bs", "kk", "sq", "sw", "gl", "mr", "pa", "si", "km", "sn", "yo", "so",
    "af", "oc", "ka", "be", "tg", "sd", "gu", "am", "yi", "lo", "uz", "fo", "ht", "ps", "tk", "nn", "mt",
    "sa", "lb", "my", "bo", "tl", "mg", "as", "tt", "haw", "ln", "ha", "ba", "jw", "su", "yue"};

int lang_id_from_str(const std::string& s) {
  for (int i = 0; i < 100; ++i)
    if (s == kLangs[i]) return i;
  return -1;
}

static std::string letters(int k, int n) {
  std::string s(n, 'a');
  for (int i = n - 1; i >= 0; --i) {
    s[i] = char('a' + k % 26);
    k /= 26;
  }
  return s;
}

Vocab::Vocab(int nv) : n_vocab(nv) {
  multilingual = nv >= 51865;
  num_languages = nv - 51765 - (multilingual ? 1 : 0);
  eot = 50256;
  sot = 50257;
  translate = 50357;
  transcribe = 50358;
  solm = 50359;
  prev = 50360;
  nosp = 50361;
  not_ = 50362;
  beg = 50363;
  if (multilingual) {
    eot++;
    sot++;
    const int dt = num_languages - 98;
    translate += dt;
    transcribe += dt;
    solm += dt;
    prev += dt;
    nosp += dt;
    not_ += dt;
    beg += dt;
  }
  id_to_token.resize(nv);
  char buf[64];
  for (int i = 0; i < nv; ++i) {
    std::string w;
    if (i < eot) {
      if (i < 26) w = std::string(1, char('a' + i));
      else if (i == 26) w = " ";
      else if (i < 27 + 26 * 26 * 26) w = " " + letters(i - 27, 3);
      else w = letters(i - 27 - 26 * 26 * 26, 4);
    } else if (i > beg) {
      snprintf(buf, sizeof buf, "[_TT_%d]", i - beg);
      w = buf;
    } else if (i == eot) w = "[_EOT_]";
    else if (i == sot) w = "[_SOT_]";
    else if (i == translate) w = "[_TRANSLATE_]";
    else if (i == transcribe) w = "[_TRANSCRIBE_]";
    else if (i == solm) w = "[_SOLM_]";
    else if (i == prev) w = "[_PREV_]";
    else if (i == nosp) w = "[_NOSP_]";
    else if (i == not_) w = "[_NOT_]";
    else if (i == beg) w = "[_BEG_]";
    else if (i > sot && i <= sot + num_languages) w = std::string("[_LANG_") + kLangs[i - sot - 1] + "]";
    else {
      snprintf(buf, sizeof buf, "[_extra_token_%d]", i);
      w = buf;
    }
    id_to_token[i] = w;
    token_to_id[w] = i;
  }
}

// whisper.cpp regex: 's|'t|'re|'ve|'m|'ll|'d| ?[[:alpha:]]+| ?[[:digit:]]+| ?[^\s[:alpha:][:digit:]]+|\s+(?!\S)|\s+
// (byte-level; ASCII classes — the synthetic vocabulary is ASCII)
std::vector<std::string> Vocab::split_words(const std::string& t) {
  std::vector<std::string> out;
  const size_t n = t.size();
  size_t i = 0;
  auto isal = [](unsigned char c) { return std::isalpha(c) != 0; };
  auto isdg = [](unsigned char c) { return std::isdigit(c) != 0; };
  auto issp = [](unsigned char c) { return std::isspace(c) != 0; };
  static const char* sufs[] = {"'s", "'t", "'re", "'ve", "'m", "'ll", "'d"};
  while (i < n) {
    std::string m;
    for (const char* s : sufs) {
      const size_t L = strlen(s);
      if (t.compare(i, L, s) == 0) { m = s; break; }
    }
    if (m.empty()) {
      const size_t j = (t[i] == ' ' && i + 1 < n) ? i + 1 : i;
      for (int cls = 0; cls < 3 && m.empty(); ++cls) {
        auto in = [&](unsigned char c) {
          return cls == 0 ? isal(c) : cls == 1 ? isdg(c) : !(issp(c) || isal(c) || isdg(c));
        };
        if (j < n && in(t[j])) {
          size_t k = j;
          while (k < n && in(t[k])) ++k;
          m = t.substr(i, k - i);
        }
      }
      if (m.empty() && issp(t[i])) {
        size_t k = i;
        while (k < n && issp(t[k])) ++k;
        m = (k < n && k - i > 1) ? t.substr(i, k - 1 - i) : t.substr(i, k - i);
      }
      if (m.empty()) m = t.substr(i, 1);
    }
    out.push_back(m);
    i += m.size();
  }
  return out;
}

std::vector<int> Vocab::tokenize(const std::string& text) const {
  std::vector<int> toks;
  for (const auto& word : split_words(text)) {
    size_t i = 0;
    const size_t n = word.size();
    while (i < n) {
      size_t j = n;
      bool found = false;
      while (j > i) {
        auto it = token_to_id.find(word.substr(i, j - i));
        if (it != token_to_id.end()) {
          toks.push_back(it->second);
          i = j;
          found = true;
          break;
        }
        --j;
      }
      if (!found) ++i;
    }
  }
  return toks;
}

}  // namespace wdr
