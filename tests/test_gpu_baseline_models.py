"""Parity at the BASELINE.json model sizes: the HIP path (libwdr through the C ABI) against the
CPU oracle on base.en and large-v3 (synthetic seeded weights, bit-identical on both sides).

Covered here (VERDICT r1 "next round" item 1):
  * one 30-s window: normalised log-mel, encoder output, every decoder layer's cross K/V,
    logits (top-1 and margin), alignment-head capture;
  * a greedy `state.full` with DTW (src/transcribe.rs:389) on a one-window segment;
  * a > 30-s segment: the seek loop over two windows (base.en);
  * configs[0] (C1): base.en, 30-s WAV, enable_vad=false, default options (beam 5, lang auto)
    through wdr_transcribe_audio (src/engine.rs:141-147, 169-199) against the oracle pipeline
    + formatting;
  * the temperature-fallback ladder and the no-speech skip with whisper.cpp's default
    thresholds (entropy 2.4, logprob -1.0, no-speech 0.6) active.

Tolerances (f16 operands, f32 accumulation on both sides, different summation order):
  * log-mel |err| <= 2e-3;
  * encoder output / cross K/V: relative Frobenius error <= 1e-2 (base.en) / 3e-2 (large-v3),
    every row's cosine >= 0.999;
  * logits: |err| <= 3% of the logit spread + 0.03; the top-1 token equal wherever the oracle's
    top-1 / top-2 gap exceeds MARGIN;
  * token ids equal except at a greedy pick whose oracle logprob gap is below MARGIN (an f16
    near-tie: the test stops comparing that segment there and records the flip); heuristic
    t0/t1 within 2 cs; DTW anchors within 2 cs, at most 1 in 20 within 4 cs (near-equal path
    costs of the random-weight alignment matrix, analysed in test_c1_flat_alignment_near_ties);
    C1's words within 20 ms (the north star) on alignment-conditioned weights.
"""
import json
import os

import numpy as np
import pytest

import wdr
from oracle.mel import log_mel, pcm_i16_to_f32
from oracle.model import DecoderState, Whisper
from oracle.vocab import Vocab
from oracle.weights import hparams_for, synth_weights
from oracle.whisper_full import FullParams, WhisperState, aheads_for_model_name
from wdr.synth import synth_speech

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(1200)]

EMB_STD = 0.5
PIN = wdr.Synthetic(weight_std=0.02, emb_std=EMB_STD, force_len_rate=3.3, disable_fallback=True)
MARGIN = {"base.en": 0.05, "large-v3": 0.1}
REL = {"base.en": 1e-2, "large-v3": 3e-2}
REPORT = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "baseline_parity.jsonl")


def _report(**kw):
    """Measured error figures (appended to gpurun_out/ when run on the GPU box)."""
    try:
        os.makedirs(os.path.dirname(REPORT), exist_ok=True)
        with open(REPORT, "a") as f:
            f.write(json.dumps(kw) + "\n")
    except OSError:
        pass
    print(kw)


@pytest.fixture(scope="module", params=["base.en", "large-v3"])
def model(request):
    name = request.param
    hp = hparams_for(name)
    W = synth_weights(hp, std=0.02, emb_std=EMB_STD)
    ctx = wdr.WhisperContext(name, synthetic=PIN)
    m = Whisper(hp, W)
    yield name, ctx, hp, W, m
    ctx.close()


@pytest.fixture(scope="module")
def speech():
    pcm, spurts = synth_speech(75.0, seed=21)
    return pcm, spurts


def _rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _row_cos_min(a, b):
    num = (a * b).sum(-1)
    den = np.linalg.norm(a, axis=-1) * np.linalg.norm(b, axis=-1) + 1e-30
    return float((num / den).min())


def test_window_mel_encoder_cross_kv_logits_capture(model, speech):
    """One 30-s window, stage by stage, each stage fed the ORACLE's input of that stage
    where the seam allows it (mel window -> encoder), else the GPU's own (cross K/V, logits)."""
    name, ctx, hp, W, m = model
    pcm, _ = speech
    x = pcm_i16_to_f32(pcm[:30 * 16000])
    # a4 log-mel
    mel_ref = log_mel(x, hp.n_mels)[:, :3000]
    mel_got = ctx.log_mel_window(x, 0)
    mel_err = float(np.abs(mel_got - mel_ref).max())
    assert mel_err < 2e-3, mel_err
    # a5 + a6: conv front-end + encoder on the same (oracle) mel window
    enc_ref = m.encode(mel_ref)
    enc_got = ctx.encode(mel_ref)
    e_rel, e_cos = _rel(enc_got, enc_ref), _row_cos_min(enc_got, enc_ref)
    # a7: cross K/V of every decoder layer
    cross = m.cross_kv(enc_ref)
    xkv = ctx.cross_kv()
    x_rel = max(max(_rel(xkv[:, l, 0], cross[l][0]), _rel(xkv[:, l, 1], cross[l][1])) for l in range(hp.n_text_layer))
    _report(test="window", model=name, mel_max_abs=mel_err, enc_rel=e_rel, enc_row_cos_min=e_cos, xkv_rel_max=x_rel)
    assert e_rel < REL[name] and e_cos > 0.999, (e_rel, e_cos)
    assert x_rel < REL[name], x_rel
    # a9: logits of a prompt prefill + steps
    v = Vocab(hp.n_vocab)
    rng = np.random.default_rng(5)
    seqs = [[v.sot], [v.sot, v.beg], [v.sot] + list(rng.integers(0, v.eot, 24))]
    if v.multilingual:
        seqs.append([v.sot, v.token_lang(0), v.transcribe, v.beg])
    flips = 0
    for toks in seqs:
        got = ctx.decode(toks)
        ref = DecoderState(m).forward(list(toks), cross)
        err, spread = float(np.abs(got - ref).max()), float(ref.std())
        top2 = np.sort(ref)[-2:]
        _report(test="logits", model=name, n=len(toks), max_abs=err, spread=spread, margin=float(top2[1] - top2[0]))
        assert err < 0.03 * spread + 0.03, (err, spread)
        if int(np.argmax(got)) != int(np.argmax(ref)):
            flips += 1
            assert top2[1] - top2[0] < MARGIN[name], (toks, top2)
    # a12: alignment-head capture over a DTW token sequence
    ah = aheads_for_model_name(name)
    toks = [v.sot] + ([v.token_lang(0)] if v.multilingual else []) + [v.not_] + list(rng.integers(0, v.eot, 16)) + [v.eot]
    cap = ctx.capture(toks, len(ah))
    _, qk = DecoderState(m).forward(toks, cross, want_logits=None, aheads=ah)
    c_err = float(np.abs(cap - qk).max())
    _report(test="capture", model=name, max_abs=c_err, logit_flips=flips)
    assert c_err < 5e-3, c_err
    np.testing.assert_allclose(cap.sum(-1), 1.0, atol=2e-3)


def _compare_results(got, ref, name, where):
    """Token-by-token comparison of state.full results; a mismatch is allowed only at an
    oracle near-tie (greedy logprob gap < MARGIN), after which that segment is not compared.
    Returns the number of tokens compared."""
    assert len(got) >= 1 and len(ref) >= 1
    n_cmp = 0
    for g, r in zip(got, ref):
        ids_g = [t["id"] for t in g["tokens"]]
        ids_r = [t.id for t in r.tokens]
        k = 0
        while k < min(len(ids_g), len(ids_r)) and ids_g[k] == ids_r[k]:
            k += 1
        if k < len(ids_r) or len(ids_g) != len(ids_r):
            m = r.tokens[k].margin if k < len(ids_r) else float("inf")
            _report(test="flip", model=name, where=where, at=k, of=len(ids_r), margin=m)
            assert m < MARGIN[name], ("token mismatch off a near-tie", where, k, ids_g[k:k + 5], ids_r[k:k + 5], m)
            return n_cmp + k
        assert g["text"] == r.text
        assert (g["t0"], g["t1"]) == (r.t0, r.t1)
        d_dtw = [abs(tg["t_dtw"] - tr.t_dtw) for tg, tr in zip(g["tokens"], r.tokens)]
        for tg, tr in zip(g["tokens"], r.tokens):
            assert abs(tg["t0"] - tr.t0) <= 2 and abs(tg["t1"] - tr.t1) <= 2, (where, tg, tr)
            assert abs(tg["p"] - tr.p) < 2e-3, (where, tg, tr)
        # DTW anchors: within one DTW frame (2 cs) except where the random-weight alignment
        # matrix has near-equal path costs -- then within two frames (4 cs); the words built
        # from them (midpoints, src/transcribe.rs:291-306) are held to +-20 ms separately
        _report(test="dtw", where=where, model=name, max_cs=max(d_dtw), over_2cs=sum(d > 2 for d in d_dtw),
                tokens=len(d_dtw))
        assert max(d_dtw) <= 4 and sum(d > 2 for d in d_dtw) <= max(1, len(d_dtw) // 20), (where, d_dtw)
        n_cmp += len(ids_r)
    assert len(got) == len(ref), where
    return n_cmp


def _greedy_params(lang="auto"):
    return FullParams(strategy="greedy", language=lang, force_len_rate=3.3, logprob_thold=-np.inf, entropy_thold=-1.0)


def test_state_full_greedy_dtw_one_window(model, speech):
    """whisper_full on a ~20-s segment (one window): lang auto, greedy, heuristic timestamps
    and DTW, the synthetic decode-length pin."""
    name, ctx, hp, W, m = model
    pcm, spurts = speech
    a = spurts[0][0]
    x = pcm_i16_to_f32(pcm[int(a * 16000):int((a + 20.0) * 16000)])
    opts = wdr.TranscribeOptions(lang="auto", advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    got, lang_id = ctx.state_full(x, opts)
    st = WhisperState(m, Vocab(hp.n_vocab), name)
    st.full(x, _greedy_params())
    if st.lang_margin > MARGIN[name]:
        assert lang_id == st.lang_id
    n = _compare_results(got, st.result_all, name, "one-window")
    _report(test="state_full", model=name, tokens_compared=n, tokens=sum(len(r.tokens) for r in st.result_all))
    assert n >= 3


def test_state_full_beam5_dtw_one_window(model, speech):
    """whisper_full with the reference's DEFAULT strategy -- beam search, 5 beams, patience -1
    (src/transcribe.rs:22-33) -- on the ~20-s segment of the greedy test, lang auto, heuristic
    timestamps and DTW:
    the beams' candidates (top-K per beam, ordered by cumulative log-prob, duplicates dropped,
    KV caches following their parents) and the final ranking, token by token against the
    oracle's WhisperState.decode_beam.  At large-v3 this runs the beam-group cross-attention
    and the rows kernel at the full width."""
    name, ctx, hp, W, m = model
    pcm, spurts = speech
    a = spurts[0][0]
    x = pcm_i16_to_f32(pcm[int(a * 16000):int((a + 20.0) * 16000)])
    opts = wdr.TranscribeOptions(lang="auto")          # advanced None: beam search, 5 beams
    got, lang_id = ctx.state_full(x, opts)
    st = WhisperState(m, Vocab(hp.n_vocab), name)
    st.full(x, FullParams(strategy="beam", beam_size=5, language="auto", force_len_rate=3.3,
                          logprob_thold=-np.inf, entropy_thold=-1.0))
    if st.lang_margin > MARGIN[name]:
        assert lang_id == st.lang_id
    n = _compare_results(got, st.result_all, name, "beam5")
    _report(test="state_full_beam5", model=name, tokens_compared=n, tokens=sum(len(r.tokens) for r in st.result_all))
    assert n >= 3


def test_state_full_seek_loop(model, speech):
    """A 45-s segment: two 30-s windows, seek advanced by the segment-end rules (whisper.cpp's
    seek loop; VAD-merged segments and the whole-file branch hit it, src/vad.rs:49-63,
    src/engine.rs:141-147).  base.en only (the oracle's large-v3 encoder takes ~20 s a window)."""
    name, ctx, hp, W, m = model
    if name != "base.en":
        pytest.skip("seek loop checked on base.en (oracle cost)")
    pcm, _ = speech
    x = pcm_i16_to_f32(pcm[16000:46 * 16000])
    opts = wdr.TranscribeOptions(lang="en", advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    got, _ = ctx.state_full(x, opts, initial_prompt=" hello there")
    p = _greedy_params("en")
    p.initial_prompt = " hello there"
    st = WhisperState(m, Vocab(hp.n_vocab), name)
    st.full(x, p)
    assert len(st.result_all) == 2 and st.stats["encode"] == 2
    n = _compare_results(got, st.result_all, name, "seek-loop")
    _report(test="seek_loop", model=name, tokens_compared=n, windows=len(st.result_all))


def test_c1_whole_file_transcribe_audio(tmp_path):
    """configs[0] (C1): base.en, 30-s mono 16 kHz WAV, enable_vad=false, enable_diarize=false,
    default options (beam search 5, lang auto, fallback thresholds active) through
    Engine::transcribe_audio's whole-file branch (src/engine.rs:141-147) and the subtitle
    formatting on the output path (src/engine.rs:179-199), against the oracle's output committed
    as a fixture (tests/golden/c1_base_en_30s.json, alignment-conditioned weights N(0, 0.05)):
    every cue's text equal, every word and cue bound within +-20 ms (north_star)."""
    from tests.test_gpu_configs import fixture_vs_transcribe_audio
    n, dw = fixture_vs_transcribe_audio(tmp_path, "c1_base_en_30s.json")
    _report(test="c1", cues=n, word_max_dt=dw)


def test_c1_flat_alignment_near_ties(tmp_path):
    """C1 on the round-1 weights N(0, 0.02), whose alignment heads attend almost uniformly over
    the 1500 frames (alignment-matrix spread 0.048 against 0.40 at 0.05): token ids, text,
    heuristic times and formatting must still agree exactly; a DTW anchor may move only at a
    near-tie -- where the GPU's path, priced under the ORACLE's own alignment matrix, is within
    the perturbation the capture's f16-rounding-level error puts on the two paths
    (tests/dtw_neartie.py; the round-3 record: 3 tokens, path margin 7.6e-6 on a path cost of
    101, perturbation 2.5, profiles/r04/dtw_diag.jsonl).  The links:
      1. token level (state.full): ids equal, heuristic t0/t1 within 2 cs, DTW anchors compared
         window by window with the near-tie analysis on the same tokens;
      2. transcribe_audio's output == the oracle formatting applied to the GPU pipeline's own
         words, exactly."""
    from oracle import formatting as F
    from oracle.pipeline import write_wav
    from tests.dtw_neartie import analyse, gpu_capture, record_dtw_calls
    pcm, _ = synth_speech(30.0, seed=31)
    path = str(tmp_path / "c1.wav")
    write_wav(path, pcm)
    syn = wdr.Synthetic(weight_std=0.02, emb_std=EMB_STD, force_len_rate=3.3, disable_fallback=False)
    eng = wdr.Engine(wdr.EngineConfig(cache_dir=str(tmp_path / "cache")), synthetic=syn)
    opts = wdr.TranscribeOptions(model="base.en", enable_vad=False)        # src/types.rs:46-61 defaults otherwise
    got = eng.transcribe_audio(path, opts)
    eng.close()
    hp = hparams_for("base.en")
    m = Whisper(hp, synth_weights(hp, std=0.02, emb_std=EMB_STD))
    ctx = wdr.WhisperContext("base.en", synthetic=syn)
    x = pcm_i16_to_f32(pcm)
    toks_got, _ = ctx.state_full(x, opts)
    st = WhisperState(m, Vocab(hp.n_vocab), "base.en")
    calls = record_dtw_calls(st, m)
    st.full(x, FullParams(language="auto", force_len_rate=3.3))
    ref = st.result_all
    assert len(toks_got) == len(ref)
    moved = ties = 0
    for g, r in zip(toks_got, ref):
        assert [t["id"] for t in g["tokens"]] == [t.id for t in r.tokens] and g["text"] == r.text
        for tg, tr in zip(g["tokens"], r.tokens):
            assert abs(tg["t0"] - tr.t0) <= 2 and abs(tg["t1"] - tr.t1) <= 2, (tg, tr)
    for c in calls:
        a = analyse(c["qk_o"], gpu_capture(ctx, x, c, len(st.aheads)), c["n_frames"], c["sot_len"], c["seek"])
        if a["moved"]:
            moved += len(a["moved"])
            assert a["path_margin"] <= a["perturbation"], ("anchor moved off a near-tie", a["moved"],
                                                           a["path_margin"], a["perturbation"])
            ties += 1
        _report(test="c1_flat_dtw", seek=c["seek"], moved=a["moved"], path_margin=a["path_margin"],
                perturbation=a["perturbation"], path_cost=a["path_cost"], x_spread=a["x_spread"])
    # the pipeline's own anchors against the oracle's: a moved one must be one the seam showed
    d = [abs(tg["t_dtw"] - tr.t_dtw) for g, r in zip(toks_got, ref) for tg, tr in zip(g["tokens"], r.tokens)]
    assert sum(v > 0 for v in d) <= moved, (d, moved)
    # 2. formatting of the GPU's own words == transcribe_audio's output
    seg = [wdr.SpeechSegment(0.0, len(pcm) / 16000.0, pcm)]
    raw_got, lang_got = ctx.run_pipeline(seg, opts)
    ctx.close()
    want = F.process_segments([F.Seg(s.start, s.end, s.text, None if s.words is None else
                                     [F.Word(w.text, w.start, w.end, w.probability) for w in s.words], None)
                               for s in raw_got], F.config_for_language(lang_got or "auto"))
    assert len(got) == len(want) >= 1
    for g, w in zip(got, want):
        assert (g.text, g.start, g.end) == (w.text, w.start, w.end)
        assert [(a.text, a.start, a.end) for a in g.words] == [(b.text, b.start, b.end) for b in w.words]
    _report(test="c1_flat", windows=len(calls), anchors_moved=moved, windows_at_near_tie=ties)


@pytest.mark.parametrize("strategy", ["beam_search", "greedy"])
def test_fallback_ladder_default_thresholds(strategy):
    """whisper.cpp's default thresholds active (logprob -1.0, entropy 2.4, no-speech 0.6): with
    near-uniform logits (emb_std 0.02) every temperature's avg logprob is far below -1.0, so
    the ladder runs t = 0 (beam 5 / greedy), 0.2, ..., 1.0 (best_of 5 sampling decoders,
    std::mt19937 + std::discrete_distribution) and keeps the last -- all of it compared with
    the oracle on base.en."""
    name = "base.en"
    hp = hparams_for(name)
    syn = wdr.Synthetic(weight_std=0.02, emb_std=0.02, force_len_rate=3.3, disable_fallback=False)
    ctx = wdr.WhisperContext(name, synthetic=syn)
    st = WhisperState(Whisper(hp, synth_weights(hp, std=0.02, emb_std=0.02)), Vocab(hp.n_vocab), name)
    pcm, spurts = synth_speech(20.0, seed=41)
    a = spurts[0][0]
    x = pcm_i16_to_f32(pcm[int(a * 16000):int((a + 4.0) * 16000)])
    opts = wdr.TranscribeOptions(lang="en", advanced=wdr.AdvancedTranscribe(sampling_strategy=strategy))
    got, _ = ctx.state_full(x, opts)
    p = FullParams(strategy="greedy" if strategy == "greedy" else "beam", language="en", force_len_rate=3.3)
    st.full(x, p)
    ctx.close()
    assert st.stats["fallbacks"] == 5, st.stats      # t = 0 .. 0.8 failed, 1.0 kept
    ref = st.result_all
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        assert [t["id"] for t in g["tokens"]] == [t.id for t in r.tokens]
        assert g["text"] == r.text
        for tg, tr in zip(g["tokens"], r.tokens):
            assert abs(tg["t_dtw"] - tr.t_dtw) <= 2 and abs(tg["t0"] - tr.t0) <= 2 and abs(tg["t1"] - tr.t1) <= 2


def _no_speech_model(W, v):
    """Final decoder LayerNorm that makes <|nospeech|> dominate every logit row: gamma small,
    beta along the nospeech embedding (logit_nosp ~ 40, every other ~ 40 * cos ~ N(0, 1.8)).
    The decoded text tokens then have avg logprob far below -1.0, so the window is a no-speech
    skip (no_speech_prob > 0.6 and avg_logprob < -1.0)."""
    e = W["decoder.token_embedding.weight"][v.nosp].astype(np.float64)
    W["decoder.ln.weight"] = np.full_like(W["decoder.ln.weight"], 0.02)
    W["decoder.ln.bias"] = (40.0 * e / (e @ e)).astype(np.float32)


@pytest.mark.parametrize("name", ["tiny-test", "base.en"])
def test_no_speech_skip_default_thresholds(tmp_path, name):
    """The no-speech skip (whisper.cpp: no_speech_prob > 0.6 and avg_logprob < -1.0 -> the
    window yields no segment, its tokens do not enter the prompt, seek advances): weights from
    a whisper.cpp ggml file whose final LayerNorm makes <|nospeech|> win the prefill.  A
    45-s segment skips both windows.  GPU and oracle must agree on all of it."""
    from tests.ggml_writer import write_ggml
    hp = hparams_for(name)
    v = Vocab(hp.n_vocab)
    path = str(tmp_path / ("ggml-%s.bin" % name))
    _, _, _, W = write_ggml(path, name, std=0.02, emb_std=EMB_STD, mutate=lambda W: _no_speech_model(W, v))
    syn = wdr.Synthetic(weight_std=0.02, emb_std=EMB_STD, force_len_rate=3.3, disable_fallback=False)
    ctx = wdr.WhisperContext(name, model_path=path, synthetic=syn)
    st = WhisperState(Whisper(hp, W), v, name)
    pcm, _ = synth_speech(50.0, seed=43)
    x = pcm_i16_to_f32(pcm[:45 * 16000])
    opts = wdr.TranscribeOptions(lang="en", advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    got, _ = ctx.state_full(x, opts, initial_prompt=" so")
    p = FullParams(strategy="greedy", language="en", force_len_rate=3.3, initial_prompt=" so")
    st.full(x, p)
    ctx.close()
    assert st.stats["no_speech_skips"] == 2 and st.result_all == [], st.stats
    assert got == []
