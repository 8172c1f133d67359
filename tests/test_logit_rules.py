"""Known-answer tests of whisper.cpp's logit rules and greedy pick (SURVEY.md Appendix A.4,
whisper.cpp whisper_process_logits / whisper_sample_token as the reference drives them through
WhisperState::full, src/transcribe.rs:20-87 and :389).

Every case is a crafted logit vector with a hand-derived answer (the comment of each case says
why); the same cases run on the CPU restatement (oracle/whisper_full.py process_logits +
sample_greedy, not GPU-marked) and on the GPU kernel (k_logits_process through the C ABI seam
wdr_dbg_logits).  Vocabulary: the english layout (eot 50256, beg 50363, 1 501 timestamps) and the
large-v3 layout (eot 50257, beg 50365, 100 language tokens).
"""
import types

import numpy as np
import pytest

from oracle.vocab import Vocab
from oracle.whisper_full import FullParams, Token, WhisperState

MODELS = {"tiny-test": 51864, "tiny-test-ml": 51866}
A, B = 100, 200          # two ordinary text tokens
BASE = -3.0


def _cases(v):
    """(name, logits, history ids, has_ts, seek_delta, force, temperature, max_initial_ts,
    suppress_blank, expected id, extra expectations)."""
    V = v.n_vocab
    out = []

    def lg():
        return np.full(V, BASE, np.float32)

    # 1. initial step: EOT and " " suppressed (suppress_blank) -> the best remaining text token
    x = lg(); x[v.eot] = 9; x[v.token_to_id[" "]] = 8; x[A] = 5
    out.append(("initial_suppress_blank", x, [], False, 0, None, 0.0, 1.0, True, A, {}))
    # 1b. the same without suppress_blank: EOT wins (the initial-step timestamp cap does not
    #     matter: no timestamp is high)
    out.append(("initial_no_suppress_blank", x.copy(), [], False, 0, None, 0.0, 1.0, False, v.eot, {}))
    # 2. sot / not / prev / solm / nosp / translate / transcribe (and language tokens) are never
    #    sampled, whatever their logits
    x = lg()
    for t in (v.sot, v.not_, v.prev, v.solm, v.nosp, v.translate, v.transcribe):
        x[t] = 9
    if v.multilingual:
        x[v.token_lang(3)] = 9
    x[B] = 5
    out.append(("specials_never", x, [A], False, 0, None, 0.0, 1.0, True, B, {}))
    # 3. last two tokens timestamps -> every timestamp masked: text wins over a higher timestamp
    x = lg(); x[v.beg + 20] = 9; x[B] = 5
    out.append(("ts_ts_masks_ts", x, [A, v.beg + 10, v.beg + 12], True, 24, None, 0.0, 1.0, True, B, {}))
    # 4. last token a timestamp after text -> every text token masked (EOT stays allowed); the
    #    timestamp beats EOT
    x = lg(); x[A] = 9; x[v.eot] = 2; x[v.beg + 30] = 4
    out.append(("text_ts_masks_text", x, [B, v.beg + 12], True, 24, None, 0.0, 1.0, True, v.beg + 30, {}))
    # 4b. ... and EOT beats a lower timestamp when the other timestamps carry no mass (at -30:
    #     at the -3 baseline the 1 488 allowed timestamps' log-sum-exp, 4.4, would beat EOT's 4
    #     and mask it with the text -- rule 6)
    x = np.full(V, -30.0, np.float32); x[A] = 9; x[v.eot] = 4; x[v.beg + 30] = 2
    out.append(("text_ts_eot", x, [B, v.beg + 12], True, 24, None, 0.0, 1.0, True, v.eot, {}))
    # 5. initial step: timestamps above beg + round(1.0 / 0.02) = beg + 50 masked; the timestamp
    #    mass (log-sum-exp ~ 6) beats the best text log-prob (~1), so text is masked too
    x = lg(); x[v.beg + 51] = 9; x[v.beg + 50] = 6; x[A] = 1
    out.append(("max_initial_ts", x, [], False, 0, None, 0.0, 1.0, True, v.beg + 50, {}))
    # 5b. max_initial_ts 0 (disabled): beg + 51 is allowed
    out.append(("max_initial_ts_off", x.copy(), [], False, 0, None, 0.0, 0.0, True, v.beg + 51, {}))
    # 6. monotone timestamps: after a timestamp at seek_delta 100, timestamps below beg + 50 are
    #    masked
    x = lg(); x[v.beg + 40] = 9; x[v.beg + 60] = 5
    out.append(("monotone_ts", x, [A, B], True, 100, None, 0.0, 1.0, True, v.beg + 60, {}))
    # 7. timestamp probability mass beats the best single text token: 100 timestamps at 0
    #    (log-sum-exp = ln 100 = 4.61) vs a text token at 2 -> text masked; ties pick the first
    #    index (beg).  The probabilities are NOT renormalised after the mask (whisper.cpp keeps
    #    the log-softmax taken before it): ptsum = 100 / (100 + e^2) = 0.9312, pt = 1 / 100
    x = np.full(V, -30.0, np.float32); x[A] = 2.0; x[v.beg:v.beg + 100] = 0.0
    out.append(("ts_mass_beats_text", x, [B], False, 0, None, 0.0, 1.0, True, v.beg,
                {"pt": 0.01, "ptsum": 100.0 / (100.0 + np.exp(2.0)), "p": 1.0 / (100.0 + np.exp(2.0))}))
    # 7b. a text token at 6 > 4.61 keeps text: it wins
    x = x.copy(); x[A] = 6.0
    out.append(("text_beats_ts_mass", x, [B], False, 0, None, 0.0, 1.0, True, A, {}))
    # 8. synthetic pin "only": the forced token whatever the logits
    x = lg(); x[A] = 9
    out.append(("force_only", x, [B], False, 0, (1, v.beg + 7), 0.0, 1.0, True, v.beg + 7, {}))
    # 9. synthetic pin "text only": EOT and timestamps masked
    x = lg(); x[v.eot] = 9; x[v.beg + 3] = 9; x[A] = 2
    out.append(("force_text", x, [B], False, 0, (2, 0), 0.0, 1.0, True, A, {}))
    # 10. temperature 0.5 divides the logits: same argmax, p = softmax(x / 0.5)[A]
    x = np.full(V, -30.0, np.float32); x[A] = 1.0; x[B] = 0.5
    p_a = 1.0 / (1.0 + np.exp(-1.0))          # (1 - 0.5) / 0.5 = 1 nat apart; the rest ~ 0
    out.append(("temperature", x, [B], False, 0, None, 0.5, 1.0, True, A, {"p": p_a}))
    # 11. no-speech probability = softmax(raw logits)[nosp]: two tokens at 0, the rest at -20
    x = np.full(V, -20.0, np.float32); x[v.nosp] = 0.0; x[A] = 0.0
    out.append(("no_speech_prob", x, [], False, 0, None, 0.0, 1.0, True, A, {"nosp": 0.5}))
    return out


def _ctl(v, hist, has_ts, seek_delta, force):
    last_ts = len(hist) > 0 and hist[-1] >= v.beg
    pen_ts = len(hist) < 2 or hist[-2] >= v.beg
    c = dict(n_tokens=len(hist), last_ts=int(last_ts), pen_ts=int(pen_ts), has_ts=int(has_ts), seek_delta=seek_delta)
    if force is not None:
        c["force_kind"], c["force_tok"] = force
    return c


def _oracle(v, case):
    name, x, hist, has_ts, seek_delta, force, temp, mit, sb, _, _ = case
    st = WhisperState.__new__(WhisperState)
    st.v = v
    st.m = types.SimpleNamespace(hp=types.SimpleNamespace(n_audio_ctx=1500))
    p = FullParams(strategy="greedy", max_initial_ts=mit, suppress_blank=sb)
    f = None
    if force is not None:
        f = ("only", force[1]) if force[0] == 1 else ("text", None)
    toks = [Token(id=t) for t in hist]
    _, lps, probs = st.process_logits(x, toks, has_ts, seek_delta, p, temp, f)
    tok = st.sample_greedy(probs, lps)
    lp = x.astype(np.float64) - x.max()
    nosp = float(np.exp(lp[v.nosp]) / np.exp(lp).sum())
    return dict(id=tok.id, tid=tok.tid, p=tok.p, pt=tok.pt, ptsum=tok.ptsum, nosp=nosp)


def _check(name, got, want_id, extra):
    assert got["id"] == want_id, (name, got["id"], want_id)
    for k, v in extra.items():
        assert abs(got[k] - v) < 2e-3, (name, k, got[k], v)


@pytest.mark.parametrize("model", sorted(MODELS))
def test_logit_rules_known_answers_oracle(model):
    v = Vocab(MODELS[model])
    for case in _cases(v):
        _check(case[0], _oracle(v, case), case[9], case[10])


@pytest.mark.gpu
@pytest.mark.parametrize("model", sorted(MODELS))
def test_logit_rules_known_answers_gpu(model):
    import wdr
    v = Vocab(MODELS[model])
    ctx = wdr.WhisperContext(model, synthetic=wdr.Synthetic())
    cases = _cases(v)
    for i in range(0, len(cases), 8):   # up to 8 rows per call, each row its own rule state
        chunk = cases[i:i + 8]
        # rows of one call share (max_initial_ts, suppress_blank): split where they differ
        groups = {}
        for c in chunk:
            groups.setdefault((c[7], c[8]), []).append(c)
        for (mit, sb), cs in groups.items():
            got = ctx.logit_rules(np.stack([c[1] for c in cs]), [_ctl(v, c[2], c[3], c[4], c[5]) for c in cs],
                                  [c[6] for c in cs], max_initial_ts=mit, suppress_blank=sb)
            for c, g in zip(cs, got):
                _check(c[0], g, c[9], c[10])
                # and the same as the CPU restatement
                o = _oracle(v, c)
                assert g["tid"] == o["tid"], (c[0], g["tid"], o["tid"])
    ctx.close()
