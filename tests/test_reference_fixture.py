"""The reference's own output snapshot (`segments.json`, written by examples/test.rs:36-50: the
`small` model, lang auto, VAD on, FormattingOverrides{max_chars_per_line: 20, max_lines: 2}; no
input audio ships with it) kept as a data fixture, tests/golden/reference_segments.json.  It
pins the output format of transcribe_audio (src/formatting.rs via src/engine.rs:192-199):

  * <= max_lines lines per cue, cue.start == words[0].start, cue.end == words[-1].end;
  * times rounded to 3 decimals (src/formatting.rs:33, 499-505);
  * the quirks: "<|endoftext|>" leaks into text (is_whole_control_token strips only "[_..]"
    markers, src/transcribe.rs:206-212) and tiny-word merging can leave start > end
    (src/formatting.rs:418-427).

Host-only (no GPU): libwdr's process_segments through the C ABI."""
import json
import os

import pytest

import wdr

FIX = os.path.join(os.path.dirname(__file__), "golden", "reference_segments.json")
OV = wdr.FormattingOverrides(max_chars_per_line=20, max_lines=2)


@pytest.fixture(scope="module")
def cues():
    return json.load(open(FIX))


def _invariants(segs, max_lines=2):
    for s in segs:
        assert s["text"].count("\n") + 1 <= max_lines, s["text"]
        assert s["start"] == s["words"][0]["start"] and s["end"] == s["words"][-1]["end"]
        for t in [s["start"], s["end"]] + [w[k] for w in s["words"] for k in ("start", "end")]:
            assert round(t, 3) == t


def test_fixture_invariants_and_quirks(cues):
    assert len(cues) == 51
    _invariants(cues)
    leaks = [i for i, c in enumerate(cues) if "<|endoftext|>" in c["text"]]
    assert leaks == [23, 40]
    assert all(cues[i]["start"] > cues[i]["end"] for i in leaks)            # negative durations
    assert max(len(l) for c in cues for l in c["text"].split("\n")) > 20     # CPL is not a hard cap


def _as_input(cues):
    """The fixture's words as raw whisper words (leading space, one whisper segment per cue)."""
    return [wdr.Segment(c["start"], c["end"], c["text"],
                        [wdr.WordTimestamp(" " + w["text"], w["start"], w["end"], w.get("probability"))
                         for w in c["words"]], None) for c in cues]


def test_process_segments_reproduces_the_reference_output(cues):
    """Fed its own output words back (the raw words are not in the snapshot: tokens that merged
    into one word -- "long" + "-term", "hasn" + "'t", "1," + "000" -- come back as one word, so
    the cues holding them are cut differently), libwdr's process_segments reproduces the
    reference's cues text and times exactly for 41 of 51, keeps the invariants everywhere and
    reproduces both quirks (the "<|endoftext|>" text and start > end on the tiny-word merge)."""
    out = [dict(start=s.start, end=s.end, text=s.text,
                words=[dict(text=w.text, start=w.start, end=w.end) for w in s.words])
           for s in wdr.process_segments(_as_input(cues), "en", OV, None)]
    _invariants(out)
    same = sum(1 for o, c in zip(out, cues) if (o["text"], o["start"], o["end"]) == (c["text"], c["start"], c["end"]))
    assert len(out) == len(cues) and same >= 41, same
    leaks = [o for o in out if "<|endoftext|>" in o["text"]]
    assert len(leaks) == 2 and all(o["start"] > o["end"] for o in leaks)


def test_process_segments_reproduces_all_51_cues_from_raw_words(cues):
    """libwdr's process_segments (csrc/formatting.cpp) agrees with the oracle restatement on a
    RECONSTRUCTED input: raw whisper words behind the snapshot rebuilt by
    tests/golden/reconstruct_reference_raw.py (continuation pieces unglued, the hidden BPE splits
    " We" "'re", " has" "n" "'t", "<|endoftext|>" " With" ..., and for five windows raw times found
    by a seeded search until the oracle reproduced the snapshot).  On that input both reproduce
    every one of the 51 cues -- text, cue times, every word's text and times -- exactly.  This is
    oracle-vs-libwdr agreement on one consistent input, not a claim about the reference's real
    raw words (the snapshot does not hold them); the reference-parity evidence is
    test_process_segments_reproduces_the_reference_output (41 of 51 cues from the words the
    cues themselves determine)."""
    raw = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_raw_words.json")))["words"]
    seg = wdr.Segment(0.0, 0.0, "", [wdr.WordTimestamp(t, s, e, None) for t, s, e in raw], None)
    out = wdr.process_segments([seg], "en", OV, None)
    assert len(out) == len(cues) == 51
    for i, (o, c) in enumerate(zip(out, cues)):
        assert (o.text, o.start, o.end) == (c["text"], c["start"], c["end"]), i
        assert [(w.text, w.start, w.end) for w in o.words] == [(w["text"], w["start"], w["end"]) for w in c["words"]], i
