// process_segments restated from src/formatting.rs (merge continuations, clamp / merge tiny
// words against neighbours and the VAD mask, group on terminal punctuation and long gaps,
// grow cues under the duration / CPS caps, optional 2-line split scoring).  Mirrors
// oracle/formatting.py.  Character counts use extended grapheme clusters in the reference;
// here code points with combining marks, variation selectors, ZWJ sequences and CRLF folded
// into the previous cluster (exact for ASCII / Latin / CJK).
#include "formatting.h"

#include <algorithm>
#include <cmath>
#include <limits>

namespace wdr {

namespace {

struct Tok {
  std::string word, punc;
  double start, end;
  bool has_p;
  float p;
  bool has_speaker;
  std::string speaker;
  bool leading_space;
};

bool is_punc_byte(unsigned char c) {
  switch (c) {
    case '.': case '!': case '?': case ',': case ';': case ':': case ')': case ']': case '}': case '"':
      return true;
    default:
      return false;
  }
}

bool is_terminal(const std::string& p) {
  return p == "." || p == "!" || p == "?" || p == "\xE2\x80\xA6" || p == "\xE3\x80\x82" || p == "\xEF\xBC\x81" ||
         p == "\xEF\xBC\x9F";
}

bool is_comma_like(const std::string& p) {
  return p == "," || p == "\xEF\xBC\x8C" || p == "\xE3\x80\x81" || p == ";";
}

// decode one UTF-8 code point (invalid bytes count as one point each)
uint32_t next_cp(const std::string& s, size_t& i) {
  const unsigned char c = (unsigned char)s[i];
  int n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 1;
  if (i + n > s.size()) n = 1;
  uint32_t cp = n == 1 ? c : n == 2 ? (c & 0x1F) : n == 3 ? (c & 0x0F) : (c & 0x07);
  for (int k = 1; k < n; ++k) cp = (cp << 6) | ((unsigned char)s[i + k] & 0x3F);
  i += n;
  return cp;
}

bool is_extend(uint32_t cp) {
  return (cp >= 0x0300 && cp <= 0x036F) || (cp >= 0x1AB0 && cp <= 0x1AFF) || (cp >= 0x1DC0 && cp <= 0x1DFF) ||
         (cp >= 0x20D0 && cp <= 0x20FF) || (cp >= 0xFE20 && cp <= 0xFE2F) || (cp >= 0xFE00 && cp <= 0xFE0F) ||
         cp == 0x200D || (cp >= 0x1F3FB && cp <= 0x1F3FF) || (cp >= 0xE0020 && cp <= 0xE007F);
}

size_t graphemes(const std::string& s) {
  size_t n = 0, i = 0;
  bool have_prev = false, after_zwj = false;
  uint32_t prev = 0;
  while (i < s.size()) {
    const uint32_t cp = next_cp(s, i);
    if (have_prev && (is_extend(cp) || after_zwj || (prev == 0x0D && cp == 0x0A))) {
      after_zwj = cp == 0x200D;
      prev = cp;
      continue;
    }
    ++n;
    after_zwj = false;
    prev = cp;
    have_prev = true;
  }
  return n;
}

double rround(double x) { return std::copysign(std::floor(std::fabs(x) + 0.5), x); }
double round3(double x) { return rround(x * 1000.0) / 1000.0; }

void remove_fffd(std::string& s) {
  const std::string r = "\xEF\xBF\xBD";
  size_t p;
  while ((p = s.find(r)) != std::string::npos) s.erase(p, 3);
}

bool is_ascii_word(const std::string& s) {
  if (s.empty()) return false;
  for (unsigned char c : s)
    if (!((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '\'')) return false;
  return true;
}

struct Joined {
  std::string word, punc;
  bool lead;
};

Joined join_tokens(const Tok& a, const Tok& b, bool insert_space) {
  std::string s = a.word + a.punc;
  if (insert_space && b.leading_space && !b.word.empty() && !(s.size() && s.back() == ' ')) s += ' ';
  s += b.word;
  return {s, b.punc, a.leading_space};
}

size_t slice_chars(const std::vector<Tok>& g, size_t i0, size_t i1, const PostProcessConfig& cfg) {
  size_t core = 0, spaces = 0;
  for (size_t i = i0; i < i1; ++i) {
    core += cfg.use_grapheme_len ? graphemes(g[i].word) + graphemes(g[i].punc) : g[i].word.size() + g[i].punc.size();
    if (cfg.insert_interword_space && i > i0 && g[i].leading_space) ++spaces;
  }
  return core + spaces;
}

std::string render_slice(const std::vector<Tok>& g, size_t i0, size_t i1, const PostProcessConfig& cfg) {
  std::string s;
  for (size_t i = i0; i < i1; ++i) {
    if (cfg.insert_interword_space && g[i].leading_space && i > i0) s += ' ';
    s += g[i].word;
    s += g[i].punc;
  }
  return s;
}

double cap_pen(size_t v, size_t cap, double k) {
  if (v <= cap) return 0.0;
  const double d = (double)(v - cap);
  return k * d * d;
}

std::vector<std::string> split_ws(const std::string& s) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f') {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur += c;
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

bool short_funct(std::string w) {
  for (auto& c : w)
    if (c >= 'A' && c <= 'Z') c = (char)(c - 'A' + 'a');
  static const char* F[] = {"i", "to", "a", "the", "and", "or", "of", "in", "on", "for", "with", "at"};
  for (const char* f : F)
    if (w == f) return true;
  return false;
}

double syntax_penalty(const std::string& left, const std::string& right) {
  const auto r = split_ws(right), l = split_ws(left);
  double pen = 0.0;
  if (!r.empty() && short_funct(r.front())) pen += 0.3;
  if (!l.empty() && short_funct(l.back())) pen += 0.25;
  return pen;
}

std::vector<std::string> split_into_lines(const std::vector<Tok>& g, size_t i0, size_t i1,
                                          const PostProcessConfig& cfg) {
  if (i1 <= i0) return {std::string()};
  if (cfg.max_lines <= 1) return {render_slice(g, i0, i1, cfg)};
  const size_t total = slice_chars(g, i0, i1, cfg);
  if (total <= cfg.max_chars_per_line) return {render_slice(g, i0, i1, cfg)};
  const size_t n = i1 - i0;
  std::vector<size_t> cands;
  for (size_t k = 1; k < n; ++k) {
    const std::string& lt = g[i0 + k - 1].punc;
    const double gap = g[i0 + k].start - g[i0 + k - 1].end;
    const bool comma_ok = is_comma_like(lt) && total >= cfg.comma_min_chars_before_allow;
    if (is_terminal(lt) || gap >= cfg.split_gap_sec || comma_ok || k % 2 == 0 || k == n / 2) cands.push_back(k);
  }
  if (cands.empty()) return {render_slice(g, i0, i1, cfg)};
  size_t best_k = cands[0];
  double best = std::numeric_limits<double>::infinity();
  for (size_t k : cands) {
    const size_t lc = slice_chars(g, i0, i0 + k, cfg), rc = slice_chars(g, i0 + k, i1, cfg);
    const std::string lt = render_slice(g, i0, i0 + k, cfg), rt = render_slice(g, i0 + k, i1, cfg);
    double score = cap_pen(lc, cfg.max_chars_per_line, 0.02) + cap_pen(rc, cfg.max_chars_per_line, 0.02);
    if (cfg.soft_max_words_per_line > 0)
      score += cap_pen(k, cfg.soft_max_words_per_line, 0.01) + cap_pen(n - k, cfg.soft_max_words_per_line, 0.01);
    score += syntax_penalty(lt, rt);
    const std::string& p = g[i0 + k - 1].punc;
    const double gap = g[i0 + k].start - g[i0 + k - 1].end;
    const double bonus = (-0.6 * (double)(int)is_terminal(p)) + (-0.3 * (double)(int)(gap >= cfg.split_gap_sec)) +
                         (0.15 * (double)(int)is_comma_like(p));
    score += bonus;
    score += g[i0 + k].leading_space ? 0.0 : 5.0;
    if (score < best) {
      best = score;
      best_k = k;
    }
  }
  return {render_slice(g, i0, i0 + best_k, cfg), render_slice(g, i0 + best_k, i1, cfg)};
}

}  // namespace

PostProcessConfig config_for_language(const std::string& l) {
  PostProcessConfig c;
  auto set = [&](size_t cpl, double cps, bool sp, bool gr, bool ki, bool cm) {
    c.max_chars_per_line = cpl;
    c.cps_cap = cps;
    c.insert_interword_space = sp;
    c.use_grapheme_len = gr;
    c.enforce_kinsoku = ki;
    c.allow_comma_split = cm;
  };
  if (l == "zh" || l == "zh-CN" || l == "zh-TW" || l == "ja" || l == "ko") set(20, 11.5, false, true, true, true);
  else if (l == "th" || l == "lo" || l == "km" || l == "my") set(22, 13.0, true, true, false, false);
  else if (l == "ar" || l == "fa" || l == "ur" || l == "he") set(28, 14.0, true, true, false, true);
  else if (l == "hi" || l == "bn" || l == "ta" || l == "te" || l == "ml" || l == "mr" || l == "gu" || l == "pa" ||
           l == "kn" || l == "or" || l == "si")
    set(30, 15.0, true, true, false, true);
  else set(38, 17.0, true, true, false, true);
  return c;
}

std::vector<FmtSeg> process_segments(const std::vector<FmtSeg>& segs, const PostProcessConfig& cfg,
                                     const std::vector<std::pair<double, double>>* mask_in) {
  // VadMaskOracle (src/formatting.rs:212-237) or NoSilence
  std::vector<std::pair<double, double>> mask;
  if (mask_in) {
    for (auto& m : *mask_in)
      if (m.second > m.first) mask.push_back(m);
    std::stable_sort(mask.begin(), mask.end(), [](auto& a, auto& b) { return a.first < b.first; });
  }
  auto is_silence = [&](double t0, double t1) {
    if (!mask_in) return false;
    if (t1 <= t0) return true;
    for (auto& m : mask) {
      if (m.second <= t0) continue;
      if (m.first >= t1) break;
      if (m.second > t0 && m.first < t1) return false;
    }
    return true;
  };
  // 1) words with their segment's speaker
  std::vector<Tok> toks;
  auto add = [&](const FmtSeg& sg, const std::string& text, double st, double en, bool hp, float p) {
    std::string core = text, punc;
    size_t cut = core.size();
    while (cut > 0 && is_punc_byte((unsigned char)core[cut - 1])) --cut;
    punc = core.substr(cut);
    core = core.substr(0, cut);
    const bool lead = !core.empty() && (core[0] == ' ' || core[0] == '\n');
    size_t b = 0;
    while (b < core.size() && (core[b] == ' ' || core[b] == '\n')) ++b;
    core = core.substr(b);
    remove_fffd(core);
    remove_fffd(punc);
    if (core.empty() && punc.empty()) return;
    toks.push_back({core, punc, st, en, hp, p, sg.has_speaker, sg.speaker, lead});
  };
  for (const FmtSeg& sg : segs) {
    if (sg.has_words) {
      for (const FmtWord& w : sg.words) add(sg, w.text, w.start, w.end, w.has_p, w.p);
    } else {
      bool blank = true;
      for (char c : sg.text)
        if (!(c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f')) blank = false;
      if (!blank) add(sg, sg.text, sg.start, sg.end, false, 0.f);
    }
  }
  if (toks.empty()) return {};
  // 3) merge continuation pieces
  {
    std::vector<Tok> out;
    for (Tok& t : toks) {
      if (!out.empty()) {
        Tok& prev = out.back();
        if (t.word.empty() && !t.punc.empty()) {
          Joined j = join_tokens(prev, t, false);
          prev.word = j.word;
          prev.punc = j.punc;
          prev.end = std::max(prev.end, t.end);
          continue;
        }
        if (!t.leading_space && is_ascii_word(prev.word) && is_ascii_word(t.word) && prev.punc.empty() &&
            (t.start - prev.end) <= 0.03) {
          Joined j = join_tokens(prev, t, false);
          prev.word = j.word;
          prev.punc = j.punc;
          prev.end = std::max(prev.end, t.end);
          continue;
        }
      }
      out.push_back(t);
    }
    toks.swap(out);
  }
  // 4) clamp against neighbours and silence, then merge tiny words
  {
    const size_t n = toks.size();
    for (size_t i = 0; i < n; ++i) {
      const double dur = toks[i].end - toks[i].start;
      if (dur < cfg.min_word_dur) {
        const double grow = (cfg.min_word_dur - dur) / 2.0;
        toks[i].start -= grow;
        toks[i].end += grow;
      }
      if (i > 0) {
        const double mid = 0.5 * (toks[i - 1].end + toks[i].start);
        toks[i - 1].end = std::min(toks[i - 1].end, mid);
        toks[i].start = std::max(toks[i].start, mid);
      }
      if (i + 1 < n) {
        const double mid = 0.5 * (toks[i].end + toks[i + 1].start);
        toks[i].end = std::min(toks[i].end, mid);
        toks[i + 1].start = std::max(toks[i + 1].start, mid);
      }
      const double pad = 0.02;
      if (is_silence(toks[i].start - pad, toks[i].start)) toks[i].start += pad;
      if (is_silence(toks[i].end, toks[i].end + pad)) toks[i].end -= pad;
    }
    std::vector<Tok> out;
    size_t i = 0;
    while (i < n) {
      const double dur = toks[i].end - toks[i].start;
      if (dur < cfg.min_word_dur && i + 1 < n) {
        Tok next = toks[i + 1];
        Joined j = join_tokens(toks[i], next, cfg.insert_interword_space);
        next.word = j.word;
        next.punc = j.punc;
        next.start = std::min(toks[i].start, next.start);
        next.leading_space = j.lead;
        out.push_back(next);
        i += 2;
      } else if (dur < cfg.min_word_dur && i > 0) {
        Tok prev = out.back();
        out.pop_back();
        Joined j = join_tokens(prev, toks[i], cfg.insert_interword_space);
        prev.word = j.word;
        prev.punc = j.punc;
        prev.end = std::max(prev.end, toks[i].end);
        prev.leading_space = j.lead;
        out.push_back(prev);
        i += 1;
      } else {
        out.push_back(toks[i]);
        i += 1;
      }
    }
    toks.swap(out);
  }
  // 5) groups on terminal punctuation / long gaps; 6) cues
  std::vector<std::vector<Tok>> groups;
  {
    std::vector<Tok> cur;
    for (size_t i = 0; i < toks.size(); ++i) {
      cur.push_back(toks[i]);
      const bool long_gap = i + 1 < toks.size() && (toks[i + 1].start - toks[i].end) >= cfg.split_gap_sec;
      if (is_terminal(toks[i].punc) || long_gap) {
        groups.push_back(cur);
        cur.clear();
      }
    }
    if (!cur.empty()) groups.push_back(cur);
  }
  std::vector<FmtSeg> cues;
  for (const auto& g : groups) {
    size_t i = 0;
    while (i < g.size()) {
      size_t j = i + 1;
      while (true) {
        const double t0 = g[i].start, t1 = g[j - 1].end;
        const size_t chars = slice_chars(g, i, j, cfg);
        const double dur = std::max(t1 - t0, 0.001);
        const double cps = (double)chars / dur;
        if (j < g.size() && dur < cfg.max_sub_dur &&
            (cps <= cfg.cps_cap || chars < cfg.max_chars_per_line * cfg.max_lines))
          ++j;
        else
          break;
      }
      const std::vector<std::string> lines = split_into_lines(g, i, j, cfg);
      FmtSeg c;
      c.start = round3(std::max(g[i].start, 0.0));
      c.end = round3(g[j - 1].end);
      for (size_t q = 0; q < lines.size(); ++q) c.text += (q ? "\n" : "") + lines[q];
      c.has_words = true;
      for (size_t q = i; q < j; ++q) c.words.push_back({g[q].word + g[q].punc, round3(g[q].start), round3(g[q].end),
                                                        g[q].has_p, g[q].p});
      c.has_speaker = g[i].has_speaker;
      c.speaker = g[i].speaker;
      cues.push_back(std::move(c));
      i = j;
    }
  }
  return cues;
}

}  // namespace wdr
