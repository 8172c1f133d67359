"""Subtitle post-processing (`process_segments`).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): the Python restatement the C++ version
(csrc/formatting.cpp, on the output path of wdr_transcribe_audio) is checked against.
Reference: src/formatting.rs:240-313 (entry), :139-197 (script presets), :212-237
(VadMaskOracle), :325-643 (merge / clamp / group / cue / line split), applied by
src/engine.rs:192-199 with the detected (else requested) language and the overrides.

Character counts use extended grapheme clusters in the reference (unicode-segmentation);
`graphemes()` below counts code points, folding combining marks, variation selectors,
zero-width joiner sequences and CRLF into the previous cluster -- exact for ASCII and the
common Latin/CJK cases, parity unpinned for complex scripts.
"""
from __future__ import annotations

import dataclasses
import math
from typing import List, Optional, Tuple

PUNC_BYTES = set(b'.!?,;:)]}"')
TERMINAL = {".", "!", "?", "…", "。", "！", "？"}
COMMA_LIKE = {",", "，", "、", ";"}
SHORT_FUNCT = {"i", "to", "a", "the", "and", "or", "of", "in", "on", "for", "with", "at"}


@dataclasses.dataclass
class Config:                      # PostProcessConfig::default (src/formatting.rs:94-112)
    max_chars_per_line: int = 38
    max_lines: int = 1
    cps_cap: float = 17.0
    split_gap_sec: float = 0.5
    comma_min_chars_before_allow: int = 55
    min_word_dur: float = 0.10
    min_sub_dur: float = 1.0
    max_sub_dur: float = 6.0
    soft_max_words_per_line: int = 0
    insert_interword_space: bool = True
    use_grapheme_len: bool = True
    enforce_kinsoku: bool = False
    allow_comma_split: bool = True


PROFILES = {   # (max_chars_per_line, cps_cap, insert_space, grapheme, kinsoku, comma_split)
    "latin": (38, 17.0, True, True, False, True),
    "cjk": (20, 11.5, False, True, True, True),
    "sea": (22, 13.0, True, True, False, False),
    "rtl": (28, 14.0, True, True, False, True),
    "indic": (30, 15.0, True, True, False, True),
}


def profile_for_lang(lang: str) -> str:
    if lang in ("zh", "zh-CN", "zh-TW", "ja", "ko"):
        return "cjk"
    if lang in ("th", "lo", "km", "my"):
        return "sea"
    if lang in ("ar", "fa", "ur", "he"):
        return "rtl"
    if lang in ("hi", "bn", "ta", "te", "ml", "mr", "gu", "pa", "kn", "or", "si"):
        return "indic"
    return "latin"


def config_for_language(lang: str, overrides: Optional[dict] = None) -> Config:
    c = Config()
    p = PROFILES[profile_for_lang(lang)]
    (c.max_chars_per_line, c.cps_cap, c.insert_interword_space, c.use_grapheme_len, c.enforce_kinsoku,
     c.allow_comma_split) = p
    for k, v in (overrides or {}).items():
        if v is not None:
            setattr(c, k, v)
    return c


@dataclasses.dataclass
class Word:
    text: str
    start: float
    end: float
    probability: Optional[float] = None


@dataclasses.dataclass
class Seg:
    start: float
    end: float
    text: str
    words: Optional[List[Word]] = None
    speaker_id: Optional[str] = None


@dataclasses.dataclass
class Tok:
    word: str
    punc: str
    start: float
    end: float
    prob: Optional[float]
    speaker: Optional[str]
    leading_space: bool


def _is_extend(cp: int) -> bool:
    return (0x0300 <= cp <= 0x036F or 0x1AB0 <= cp <= 0x1AFF or 0x1DC0 <= cp <= 0x1DFF or 0x20D0 <= cp <= 0x20FF
            or 0xFE20 <= cp <= 0xFE2F or 0xFE00 <= cp <= 0xFE0F or cp == 0x200D or 0x1F3FB <= cp <= 0x1F3FF
            or 0xE0020 <= cp <= 0xE007F)


def graphemes(s: str) -> int:
    n = 0
    prev = None
    after_zwj = False
    for ch in s:
        cp = ord(ch)
        if prev is not None and (_is_extend(cp) or after_zwj or (prev == 0x0D and cp == 0x0A)):
            after_zwj = cp == 0x200D
            prev = cp
            continue
        n += 1
        after_zwj = False
        prev = cp
    return n


def rround(x: float) -> float:           # Rust f64::round: half away from zero
    return math.copysign(math.floor(abs(x) + 0.5), x)


def round3(x: float) -> float:
    return rround(x * 1000.0) / 1000.0


def split_trailing_punct(s: str) -> Tuple[str, str]:
    """Byte-wise from the end over ASCII punctuation (the reference's u8 -> char test can only
    match ASCII)."""
    b = s.encode("utf-8")
    cut = len(b)
    for i in range(len(b) - 1, -1, -1):
        if b[i] in PUNC_BYTES:
            cut = i
        else:
            break
    return b[:cut].decode("utf-8"), b[cut:].decode("utf-8")


def vad_oracle(mask):
    if mask is None:
        return lambda t0, t1: False
    m = sorted([(s, e) for s, e in mask if e > s], key=lambda t: t[0])

    def is_silence(t0, t1):
        if t1 <= t0:
            return True
        for s0, s1 in m:
            if s1 <= t0:
                continue
            if s0 >= t1:
                break
            if s1 > t0 and s0 < t1:
                return False
        return True
    return is_silence


def join_tokens(a: Tok, b: Tok, insert_space: bool):
    s = a.word + a.punc
    if insert_space and b.leading_space and b.word and not s.endswith(" "):
        s += " "
    s += b.word
    return s, b.punc, a.leading_space


def is_ascii_word(s: str) -> bool:
    return bool(s) and all((c.isascii() and c.isalpha()) or c == "'" for c in s)


def merge_continuations(toks: List[Tok]) -> List[Tok]:
    out: List[Tok] = []
    for t in toks:
        if out:
            prev = out[-1]
            if not t.word and t.punc:
                prev.word, prev.punc, _ = join_tokens(prev, t, False)
                prev.end = max(prev.end, t.end)
                continue
            if (not t.leading_space and is_ascii_word(prev.word) and is_ascii_word(t.word) and not prev.punc
                    and (t.start - prev.end) <= 0.03):
                prev.word, prev.punc, _ = join_tokens(prev, t, False)
                prev.end = max(prev.end, t.end)
                continue
        out.append(t)
    return out


def clamp_and_merge_tiny(toks: List[Tok], cfg: Config, is_silence) -> List[Tok]:
    n = len(toks)
    for i in range(n):
        dur = toks[i].end - toks[i].start
        if dur < cfg.min_word_dur:
            grow = (cfg.min_word_dur - dur) / 2.0
            toks[i].start -= grow
            toks[i].end += grow
        if i > 0:
            mid = 0.5 * (toks[i - 1].end + toks[i].start)
            toks[i - 1].end = min(toks[i - 1].end, mid)
            toks[i].start = max(toks[i].start, mid)
        if i + 1 < n:
            mid = 0.5 * (toks[i].end + toks[i + 1].start)
            toks[i].end = min(toks[i].end, mid)
            toks[i + 1].start = max(toks[i + 1].start, mid)
        pad = 0.02
        if is_silence(toks[i].start - pad, toks[i].start):
            toks[i].start += pad
        if is_silence(toks[i].end, toks[i].end + pad):
            toks[i].end -= pad
    out: List[Tok] = []
    i = 0
    while i < n:
        dur = toks[i].end - toks[i].start
        if dur < cfg.min_word_dur and i + 1 < n:
            nxt = dataclasses.replace(toks[i + 1])
            nxt.word, nxt.punc, nxt.leading_space = join_tokens(toks[i], nxt, cfg.insert_interword_space)
            nxt.start = min(toks[i].start, nxt.start)
            out.append(nxt)
            i += 2
        elif dur < cfg.min_word_dur and i > 0:
            prev = out.pop()
            prev.word, prev.punc, prev.leading_space = join_tokens(prev, toks[i], cfg.insert_interword_space)
            prev.end = max(prev.end, toks[i].end)
            out.append(prev)
            i += 1
        else:
            out.append(dataclasses.replace(toks[i]))
            i += 1
    return out


def split_into_groups(toks: List[Tok], cfg: Config) -> List[List[Tok]]:
    groups, cur = [], []
    for i, t in enumerate(toks):
        cur.append(t)
        long_gap = i + 1 < len(toks) and (toks[i + 1].start - t.end) >= cfg.split_gap_sec
        if t.punc in TERMINAL or long_gap:
            groups.append(cur)
            cur = []
    if cur:
        groups.append(cur)
    return groups


def slice_chars(sl: List[Tok], cfg: Config) -> int:
    if cfg.use_grapheme_len:
        core = sum(graphemes(t.word) + graphemes(t.punc) for t in sl)
    else:
        core = sum(len(t.word.encode()) + len(t.punc.encode()) for t in sl)
    spaces = sum(1 for t in sl[1:] if t.leading_space) if cfg.insert_interword_space else 0
    return core + spaces


def render_slice(sl: List[Tok], cfg: Config) -> str:
    s = ""
    for i, t in enumerate(sl):
        if cfg.insert_interword_space and t.leading_space and i > 0:
            s += " "
        s += t.word + t.punc
    return s


def _pen(v, cap, k):
    return 0.0 if v <= cap else k * float(v - cap) ** 2


def syntax_penalty(left: str, right: str) -> float:
    rw, lw = right.split(), left.split()
    pen = 0.0
    if rw and rw[0].lower() in SHORT_FUNCT:
        pen += 0.3
    if lw and lw[-1].lower() in SHORT_FUNCT:
        pen += 0.25
    return pen


def split_into_lines(sl: List[Tok], cfg: Config) -> List[str]:
    if not sl:
        return [""]
    if cfg.max_lines <= 1:
        return [render_slice(sl, cfg)]
    total = slice_chars(sl, cfg)
    if total <= cfg.max_chars_per_line:
        return [render_slice(sl, cfg)]
    cands = []
    for k in range(1, len(sl)):
        lt = sl[k - 1].punc
        gap = sl[k].start - sl[k - 1].end
        comma_ok = lt in COMMA_LIKE and total >= cfg.comma_min_chars_before_allow
        if lt in TERMINAL or gap >= cfg.split_gap_sec or comma_ok or k % 2 == 0 or k == len(sl) // 2:
            cands.append(k)
    if not cands:
        return [render_slice(sl, cfg)]
    best_k, best = cands[0], math.inf
    for k in cands:
        lc, rc = slice_chars(sl[:k], cfg), slice_chars(sl[k:], cfg)
        lt, rt = render_slice(sl[:k], cfg), render_slice(sl[k:], cfg)
        score = _pen(lc, cfg.max_chars_per_line, 0.02) + _pen(rc, cfg.max_chars_per_line, 0.02)
        if cfg.soft_max_words_per_line > 0:
            score += _pen(k, cfg.soft_max_words_per_line, 0.01) + _pen(len(sl) - k, cfg.soft_max_words_per_line, 0.01)
        score += syntax_penalty(lt, rt)
        p = sl[k - 1].punc
        gap = sl[k].start - sl[k - 1].end
        score += -0.6 * (p in TERMINAL) + -0.3 * (gap >= cfg.split_gap_sec) + 0.15 * (p in COMMA_LIKE)
        score += 5.0 if not sl[k].leading_space else 0.0
        if score < best:
            best, best_k = score, k
    return [render_slice(sl[:best_k], cfg), render_slice(sl[best_k:], cfg)]


def build_cue(g: List[Tok], i: int, cfg: Config):
    j = i + 1
    while True:
        sl = g[i:j]
        t0, t1 = sl[0].start, sl[-1].end
        chars = slice_chars(sl, cfg)
        dur = max(t1 - t0, 0.001)
        cps = chars / dur
        if j < len(g) and dur < cfg.max_sub_dur and (cps <= cfg.cps_cap or chars < cfg.max_chars_per_line * cfg.max_lines):
            j += 1
        else:
            break
    sl = g[i:j]
    t0, t1 = sl[0].start, sl[-1].end
    text = "\n".join(split_into_lines(sl, cfg))
    words = [Word(t.word + t.punc, round3(t.start), round3(t.end), t.prob) for t in sl]
    return j, Seg(round3(max(t0, 0.0)), round3(t1), text, words, sl[0].speaker)


def process_segments(segments: List[Seg], cfg: Config, vad_mask=None) -> List[Seg]:
    is_silence = vad_oracle(vad_mask)
    allw = []
    for seg in segments:
        if seg.words is not None:
            allw += [(seg.speaker_id, w) for w in seg.words]
        elif seg.text.strip():
            allw.append((seg.speaker_id, Word(seg.text, seg.start, seg.end, None)))
    if not allw:
        return []
    toks: List[Tok] = []
    for spk, w in allw:
        core, punc = split_trailing_punct(w.text)
        lead = core.startswith(" ") or core.startswith("\n")
        core = core.lstrip(" \n").replace("�", "")
        punc = punc.replace("�", "")
        if not core and not punc:
            continue
        toks.append(Tok(core, punc, w.start, w.end, w.probability, spk, lead))
    toks = merge_continuations(toks)
    toks = clamp_and_merge_tiny(toks, cfg, is_silence)
    cues = []
    for g in split_into_groups(toks, cfg):
        i = 0
        while i < len(g):
            i, cue = build_cue(g, i, cfg)
            cues.append(cue)
    return cues
