"""Properties the reference's glue guarantees for every segment of a pipeline run, for runs the
oracle cannot follow at their size (tests/test_gpu_configs.py, tests/test_gpu_multidevice.py):

  * one segment list in time order after the overlap clip (src/transcribe.rs:447-459);
  * segment bounds = its first word's start and last word's end (:439-440, the clip moving both);
  * every word inside its speech segment's 30-s window;
  * speaker ids "1".."k" or "?" (src/transcribe.rs:478-497) when diarizing;
  * no control token or embedded marker left in any text (src/transcribe.rs:206-240).
A word may end before it starts (heuristic t0 start, DTW-midpoint end, :291-306; the reference's
own output shows such words): counted, not rejected."""
import re

MARKER = re.compile(r"\[_|<\||\|>|_\]")


def check_pipeline_properties(out, spurts, diarize=True):
    """out: wdr.Segment list of a ground-truth-spurt run (one whisper segment per spurt);
    returns (speaker ids, words, inverted words)."""
    assert len(out) == len(spurts), (len(out), len(spurts))
    speakers = set()
    inverted = words = 0
    for i, s in enumerate(out):
        a, b, _ = spurts[i]
        if i + 1 < len(out):
            assert s.end <= out[i + 1].start + 1e-9, (i, s.end, out[i + 1].start)
            assert s.start <= out[i + 1].start, i
        assert s.text and not MARKER.search(s.text), (i, s.text)
        assert s.words, i
        assert s.start == s.words[0].start and s.end == s.words[-1].end, (i, s.start, s.end)
        for w in s.words:
            assert a - 1e-6 <= w.start <= a + 30.0 + 1e-6 and a - 1e-6 <= w.end <= a + 30.0 + 1e-6, (i, w, a)
            assert w.text and not MARKER.search(w.text), (i, w.text)
            inverted += w.end < w.start
            words += 1
        if diarize:
            assert s.speaker_id is not None
            speakers.add(s.speaker_id)
    if diarize:
        ids = sorted(x for x in speakers if x != "?")
        assert ids and ids == [str(k) for k in range(1, len(ids) + 1)], speakers
    return sorted(speakers), words, inverted
