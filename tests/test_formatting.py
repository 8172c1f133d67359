"""process_segments (src/formatting.rs, applied by src/engine.rs:192-199): the C++ version on
the output path of wdr_transcribe_audio against oracle/formatting.py on randomised word lists
(host code through the C ABI, no GPU), plus hand-derived known answers."""
import numpy as np
import pytest

import wdr
from oracle import formatting as F

VOCAB = ["I", "think", "would", "like", "to", "the", "and", "a", "transhuman", "ism", "café", "été",
         "你好", "。", "naïve", "x�", "OK", "it's", "don't", "of"]
PUNCS = ["", "", "", ",", ".", "?", "!", ";", ":", "...", ".\"", ")", "。"]


def _random_segments(rng, n_seg):
    segs, t = [], float(rng.uniform(0, 2))
    for s in range(n_seg):
        words = []
        for _ in range(int(rng.integers(0, 14))):
            w = VOCAB[int(rng.integers(len(VOCAB)))] + PUNCS[int(rng.integers(len(PUNCS)))]
            lead = rng.random() < 0.8
            if rng.random() < 0.07:
                w = PUNCS[int(rng.integers(3, len(PUNCS)))]      # punctuation-only token
            dur = float(rng.choice([0.01, 0.05, 0.12, 0.3, 0.6]))
            gap = float(rng.choice([0.0, 0.01, 0.02, 0.1, 0.7]))
            p = None if rng.random() < 0.3 else float(np.float32(rng.random()))
            words.append(F.Word((" " if lead else "") + w, t + gap, t + gap + dur, p))
            t += gap + dur
        spk = None if rng.random() < 0.5 else str(int(rng.integers(1, 4)))
        text = "".join(w.text for w in words) if words else " hello"
        segs.append(F.Seg(words[0].start if words else t, t, text, words if rng.random() < 0.9 else None, spk))
        t += float(rng.uniform(0, 1))
    return segs


def _to_wdr(segs):
    return [wdr.Segment(s.start, s.end, s.text,
                        None if s.words is None else [wdr.WordTimestamp(w.text, w.start, w.end, w.probability)
                                                      for w in s.words], s.speaker_id) for s in segs]


def _same(got, want):
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert (g.start, g.end, g.text, g.speaker_id) == (w.start, w.end, w.text, w.speaker_id)
        assert len(g.words) == len(w.words)
        for a, b in zip(g.words, w.words):
            assert (a.text, a.start, a.end) == (b.text, b.start, b.end)
            assert (a.probability is None) == (b.probability is None)
            if a.probability is not None:
                assert a.probability == pytest.approx(b.probability, rel=1e-7)


CASES = [("en", None), ("en", dict(max_lines=2, max_chars_per_line=20)), ("ja", None),
         ("th", dict(max_lines=2)), ("en", dict(max_lines=2, soft_max_words_per_line=3, comma_min_chars_before_allow=10)),
         ("ar", dict(min_word_dur=0.2, split_gap_sec=0.3, max_sub_dur=2.0, cps_cap=5.0)),
         ("en", dict(use_grapheme_len=False, insert_interword_space=False, max_lines=2))]


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("lang,ov", CASES)
def test_process_segments_matches_oracle(seed, lang, ov):
    rng = np.random.default_rng(seed * 31 + len(lang))
    segs = _random_segments(rng, int(rng.integers(1, 6)))
    mask = None
    if seed % 2:
        mask = [(float(a), float(a + rng.uniform(0.2, 3))) for a in np.sort(rng.uniform(0, 30, 6))]
    cfg = F.config_for_language(lang, ov)
    want = F.process_segments(segs, cfg, mask)
    got = wdr.process_segments(_to_wdr(segs), lang, wdr.FormattingOverrides(**(ov or {})), mask)
    _same(got, want)


def test_process_segments_known_answers():
    W = F.Word
    segs = [F.Seg(0.0, 2.0, "", [W(" Hello", 0.0, 0.4), W(" world.", 0.4, 0.9), W(" How", 1.5, 1.7),
                                 W(" are", 1.7, 1.9), W(" you?", 1.9, 2.3)], "1")]
    got = wdr.process_segments(_to_wdr(segs), "en")
    assert [s.text for s in got] == ["Hello world.", "How are you?"]
    assert (got[0].start, got[0].end, got[1].start, got[1].end) == (0.0, 0.9, 1.5, 2.3)
    assert all(s.speaker_id == "1" for s in got)
    # continuation pieces merge ("trans" + "human" -> one word); tiny words merge forward
    segs = [F.Seg(0.0, 1.0, "", [W(" trans", 0.0, 0.3), W("human", 0.31, 0.6), W(" a", 0.6, 0.62),
                                 W(" dog.", 0.62, 1.0)])]
    got = wdr.process_segments(_to_wdr(segs), "en")
    assert [w.text for w in got[0].words] == ["transhuman", "a dog."]
    assert got[0].text == "transhuman a dog."
    # empty input
    assert wdr.process_segments([], "en") == []
