"""Multi-chain decoding (engine.cpp decode_chains + StepBatcher): C States decode C contiguous
blocks of the speech segments concurrently with their greedy steps batched into one C-row
step, then the exact prompt-chain fix-up.  The result must equal the single-chain pipeline's
EXACTLY (texts, times, words, speakers), including the sampled path (temperature fallback:
decoder 0's RNG state replayed from the first segment that drew)."""
import dataclasses

import numpy as np
import pytest

import wdr
from wdr.synth import synth_speech

pytestmark = pytest.mark.gpu


def _segs(pcm, spurts):
    return [wdr.SpeechSegment(a, b, pcm[int(round(a * 16000)):int(round(b * 16000))]) for a, b, _ in spurts]


def _run(ctx, segs, opts, chains, dopts=None):
    ctx.set_chains(chains)
    out, lang = ctx.run_pipeline(segs, opts, diarize_options=dopts)
    return [dataclasses.asdict(s) for s in out], lang


@pytest.mark.parametrize("name,seconds,fallback,diarize", [
    ("tiny-test", 80.0, False, False),
    ("tiny-test", 80.0, False, True),
    ("tiny-test", 60.0, True, False),
    ("large-v3", 40.0, False, False),
])
def test_chains_equal_single_chain(name, seconds, fallback, diarize):
    syn = wdr.Synthetic(weight_std=0.02, emb_std=0.5, force_len_rate=0.0 if fallback else 3.3,
                        disable_fallback=not fallback)
    ctx = wdr.WhisperContext(name, synthetic=syn)
    pcm, spurts = synth_speech(seconds, seed=11, n_speakers=2)
    segs = _segs(pcm, spurts)
    assert len(segs) >= 6
    opts = wdr.TranscribeOptions(lang="auto", enable_diarize=True if diarize else None,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    dopts = wdr.DiarizeOptions.from_options(opts) if diarize else None
    ref, lang1 = _run(ctx, segs, opts, 1, dopts)
    for chains in (2, 4):
        got, lang = _run(ctx, segs, opts, chains, dopts)
        assert lang == lang1
        assert [s["text"] for s in got] == [s["text"] for s in ref], chains
        assert got == ref, chains
    ctx.close()


@pytest.mark.parametrize("name,seconds", [("tiny-test", 120.0), ("large-v3", 110.0)])
def test_sixteen_chains_equal_single_chain(name, seconds, monkeypatch):
    """16 decode chains: batched steps of 9..16 rows (k_mgemv 16-row shapes, the fc2 step split
    into two 8-row launches) must still give the one-chain result exactly."""
    monkeypatch.setenv("WDR_DECODE_CHAINS", "16")   # KV pool sized for 16 chains at creation
    syn = wdr.Synthetic(weight_std=0.02, emb_std=0.5, force_len_rate=3.3, disable_fallback=True)
    ctx = wdr.WhisperContext(name, synthetic=syn)
    pcm, spurts = synth_speech(seconds, seed=5, n_speakers=2)
    segs = _segs(pcm, spurts)
    assert len(segs) >= 16
    opts = wdr.TranscribeOptions(lang="auto", advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    ref, lang1 = _run(ctx, segs, opts, 1)
    got, lang = _run(ctx, segs, opts, 16)
    assert ctx.stage_times()["chains"] == 16
    assert lang == lang1
    assert got == ref
    ctx.close()


@pytest.mark.parametrize("name,seconds", [("tiny-test", 90.0), ("large-v3", 60.0)])
def test_partial_batches_equal_single_chain(name, seconds, monkeypatch):
    """The step batcher launches once every chain has submitted or WDR_BATCH_WAIT_US after the
    GPU became free: a chain busy on the host joins the next batch.  At 0 us (launch whatever is
    pending the moment the GPU is free: the most fragmented batches) and at -1 (always wait for
    every chain) 8 chains must give the one-chain result exactly -- a row's result does not
    depend on the batch it rides in (csrc/rows.h)."""
    syn = wdr.Synthetic(weight_std=0.02, emb_std=0.5, force_len_rate=3.3, disable_fallback=True)
    pcm, spurts = synth_speech(seconds, seed=17, n_speakers=2)
    segs = _segs(pcm, spurts)
    assert len(segs) >= 8
    opts = wdr.TranscribeOptions(lang="auto", advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    launches = {}
    ref = None
    for wait in ("-1", "0"):
        monkeypatch.setenv("WDR_BATCH_WAIT_US", wait)   # read when the context's batchers are made
        ctx = wdr.WhisperContext(name, synthetic=syn)
        if ref is None:
            ref, lang1 = _run(ctx, segs, opts, 1)
        got, lang = _run(ctx, segs, opts, 8)
        launches[wait] = ctx.stage_times()["batch_launches"]
        ctx.close()
        assert lang == lang1 and got == ref, wait
    assert launches["0"] >= launches["-1"], launches


@pytest.mark.parametrize("fallback", [False, True])
def test_forced_early_fixup_is_exact(fallback):
    """The early prompt fix-up (a chain redoes its first segments from its predecessor's final
    prompt while the others still decode) forced on through the wdr_dbg_set_early_fixup seam:
    it must run (nonzero count) and give the one-chain result, as must the run with it off.
    fallback: whisper.cpp's thresholds active on ~12-s segments (consecutive talk spurts
    merged), whose pinned decode repeats one token past 32 tokens -> entropy < 2.4 -> the
    ladder samples at t = 0.2 .. 1.0; shorter segments pass at t = 0.  Random draws then make
    every later segment depend on the RNG stream, so a redone segment's RNG state and the
    sampled-tail replay (incl. a first sampled segment decoded from a stale RNG) are exercised."""
    syn = wdr.Synthetic(weight_std=0.02, emb_std=0.5, force_len_rate=3.3, disable_fallback=not fallback)
    ctx = wdr.WhisperContext("tiny-test", synthetic=syn)
    pcm, spurts = synth_speech(90.0, seed=13, n_speakers=2)
    segs = _segs(pcm, spurts)
    if fallback:   # merge runs of spurts into ~12-s segments, keep every other one short
        merged, cur = [], []
        for k, sp in enumerate(spurts):
            cur.append(sp)
            if cur[-1][1] - cur[0][0] >= (12.0 if len(merged) % 2 == 0 else 0.0):
                merged.append((cur[0][0], cur[-1][1], None))
                cur = []
        segs = _segs(pcm, merged)
    assert len(segs) >= 6
    opts = wdr.TranscribeOptions(lang="auto", advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    ref, lang1 = _run(ctx, segs, opts, 1)
    ctx.set_early_fixup(2)
    got, lang = _run(ctx, segs, opts, 4)
    st = ctx.stage_times()
    assert st["early_fixup_segments"] > 0, st
    if fallback:
        assert st["replay_segments"] > 0, st
    assert lang == lang1 and got == ref
    ctx.set_early_fixup(3)   # the default: from the predecessor's speculative prompt
    got3, _ = _run(ctx, segs, opts, 4)
    assert ctx.stage_times()["early_fixup_segments"] > 0
    assert got3 == ref
    ctx.set_early_fixup(0)
    got0, _ = _run(ctx, segs, opts, 4)
    assert ctx.stage_times()["early_fixup_segments"] == 0
    assert got0 == ref
    ctx.close()


@pytest.mark.parametrize("name,seconds,chains", [("tiny-test", 80.0, 4), ("large-v3", 60.0, 8)])
def test_beam_chains_equal_single_chain(name, seconds, chains, monkeypatch):
    """The reference's default strategy (beam search, 5 beams: src/transcribe.rs:22-33) with
    decode chains: every chain's live beams join one batched step (rows grouped by segment, the
    segment's cross-K/V read once for its beams, top-5 candidates per row, steps above 16 rows
    as 16-row launches).  The result must equal the one-chain beam search exactly."""
    monkeypatch.setenv("WDR_DECODE_CHAINS", "16")
    syn = wdr.Synthetic(weight_std=0.02, emb_std=0.5, force_len_rate=3.3, disable_fallback=True)
    ctx = wdr.WhisperContext(name, synthetic=syn)
    pcm, spurts = synth_speech(seconds, seed=3, n_speakers=2)
    segs = _segs(pcm, spurts)
    assert len(segs) >= chains
    opts = wdr.TranscribeOptions(lang="auto")   # sampling_strategy unset: beam search, 5 beams
    ref, lang1 = _run(ctx, segs, opts, 1)
    got, lang = _run(ctx, segs, opts, chains)
    st = ctx.stage_times()
    assert st["chains"] == chains
    assert st["batch_rows"] > st["batch_launches"] * 2   # beams batched across chains
    assert lang == lang1
    assert got == ref
    ctx.close()


@pytest.mark.timeout(900)
def test_default_forty_chains_eight_slots_equal_single_chain(monkeypatch):
    """The shipped default: WDR_DECODE_CHAINS = 40, where every State's cross-K/V
    ring drops to 8 slots (whisper_ctx.cpp ring_slots), the default partial-batch wait, lang
    auto (encode-ahead language detection: LANG_SEQ sequences), large-v3 with DTW and speaker
    assignment: 40 chains must give the one-chain result exactly."""
    monkeypatch.setenv("WDR_DECODE_CHAINS", "40")   # the library default; conftest pins 24
    syn = wdr.Synthetic(weight_std=0.05, emb_std=0.5, force_len_rate=3.3, disable_fallback=True)
    ctx = wdr.WhisperContext("large-v3", enable_dtw=True, synthetic=syn)
    pcm, spurts = synth_speech(300.0, seed=23, n_speakers=3)
    segs = _segs(pcm, spurts)
    assert len(segs) > 40
    opts = wdr.TranscribeOptions(lang="auto", enable_diarize=True,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    dopts = wdr.DiarizeOptions.from_options(opts)
    ref, lang1 = _run(ctx, segs, opts, 1, dopts)
    got, lang = _run(ctx, segs, opts, 40, dopts)
    assert ctx.stage_times()["chains"] == 40
    assert lang == lang1
    assert got == ref
    ctx.close()


def test_language_detection_rides_in_batched_steps():
    """Multi-chain runs (WDR_LANG_PIGGYBACK, default): no encode-ahead batch carries a detection
    pass (WDR_LANG_FIRST=0); a plan's segment 0 detects in a one-row batched step, every later
    segment's SOT row rides in one of its chain's batched steps (whisper_ctx.cpp lang_ride) or, when its window was encoded too late, in a batched step
    of its own.  Per-segment languages decide each segment's prompt, so texts equal to the
    one-chain run (a detection pass per encode batch) show the same languages."""
    syn = wdr.Synthetic(weight_std=0.02, emb_std=0.5, force_len_rate=3.3, disable_fallback=True)
    ctx = wdr.WhisperContext("tiny-test", synthetic=syn)
    pcm, spurts = synth_speech(150.0, seed=7, n_speakers=2)
    segs = _segs(pcm, spurts)
    assert len(segs) >= 16
    opts = wdr.TranscribeOptions(lang="auto", advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    ref, lang1 = _run(ctx, segs, opts, 1)
    one = ctx.stage_times()
    got, lang = _run(ctx, segs, opts, 3)
    three = ctx.stage_times()
    assert lang == lang1
    assert got == ref
    assert one["lang_passes"] >= len(segs) // 4
    assert three["chains"] == 3
    # none on the encode stream by default (WDR_LANG_FIRST=0: a plan's segment 0 detects in a
    # one-row batched step); the plans' first batches with WDR_LANG_FIRST=1 (a fix-up round
    # re-plans the segments it redoes)
    assert three["lang_passes"] <= 2 * 3 < one["lang_passes"], (three["lang_passes"], one["lang_passes"])
    ctx.close()
