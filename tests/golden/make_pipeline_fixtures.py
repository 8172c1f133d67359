"""Oracle outputs of BASELINE configs[0..2] at sizes the GPU box should not recompute (VERDICT r3
"next round" item 1): the oracle runs HERE, once, and the GPU tests only compare.

Each fixture is data -- the configuration (synthetic audio seed / length, synthetic weights,
options) and the oracle's outputs on it:
  * the VAD mask and merged speech segments (oracle/vad.py + src/vad.rs:33-84 restated);
  * the raw pipeline segments (src/transcribe.rs:323-535 restated: text, bounds, token spans);
  * the formatted cues (src/formatting.rs:240-313 restated, with the VAD mask oracle).

Weights: seeded N(0, WSTD) with WSTD = 0.05, embeddings N(0, 0.5) -- "alignment-conditioned":
at the round-1 std of 0.02 the cross-attention of the alignment heads is almost uniform over
the 1500 frames (alignment-matrix spread 0.048 against 0.40 at 0.05, tools/dtw_diag.py,
profiles/r04/dtw_diag.jsonl), and the DTW path there has competitors within 8e-8 of its cost,
so anchors flip on f32 rounding alone; trained alignment heads are peaked, as at 0.05.

  c1_base_en_30s.json    configs[0]: base.en, 30 s, whole file, default options (beam 5, lang
                         auto, temperature fallback active)
  c2_base_en_600s.json   configs[1]: base.en, 600 s (its full size), Silero VAD, DTW, beam 5,
                         lang auto, fallback off (synthetic decode-length pin)
  c3_large_v3_120s.json  configs[2]: large-v3, 120 s, VAD, DTW, greedy, lang auto, fallback off
  c3_large_v3_900s.json  configs[2] at a real size: 900 s, 35 VAD segments,
                         ~50 windows, same options
  c3_large_v3_beam5_120s.json  configs[2]'s audio with the reference's default beam-5 decode
  c3_large_v3_beam5_300s.json  the same decode on 300 s of another recording (seed 53)
  c4_large_v3_diarize_300s[_w02].json  configs[3] diarized (DIAR / DIAR_W02 below)

Usage:  python tests/golden/make_pipeline_fixtures.py [c1|c2|c3|c3l|c3b|c3b3|c4d|c4dw02 ...]
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "whisper-diarize-rs_amd"))

WSTD = 0.05
EMB_STD = 0.5
FORCE_LEN = 3.3

CONFIGS = {
    "c1": dict(file="c1_base_en_30s.json", model="base.en", seconds=30.0, seed=31, vad=False, greedy=False,
               fallback=True),
    "c2": dict(file="c2_base_en_600s.json", model="base.en", seconds=600.0, seed=51, vad=True, greedy=False,
               fallback=False),
    "c3": dict(file="c3_large_v3_120s.json", model="large-v3", seconds=120.0, seed=52, vad=True, greedy=True,
               fallback=False),
    "c3l": dict(file="c3_large_v3_900s.json", model="large-v3", seconds=900.0, seed=52, vad=True, greedy=True,
                fallback=False),
    # the reference's default decode (beam 5, src/transcribe.rs:22-33) at large-v3 over several
    # VAD segments (VERDICT r5 missing 4): c3's audio with the default strategy
    "c3b": dict(file="c3_large_v3_beam5_120s.json", model="large-v3", seconds=120.0, seed=52, vad=True, greedy=False,
                fallback=False),
    "c3b3": dict(file="c3_large_v3_beam5_300s.json", model="large-v3", seconds=300.0, seed=53, vad=True, greedy=False,
                 fallback=False),
}

# configs[3] (C4) diarized: large-v3, 300 s, 3 speakers, seed 1, greedy, lang auto, DTW, speaker
# assignment with max_speakers 3, on the bench's segmentation pin (in synthetic
# mode the segment list passed downstream is the generator's ground-truth spurt table; the
# pyannote kernels are compared with the oracle in tests/test_gpu_diarize.py).  Two weight sets:
#   c4d     the alignment-conditioned N(0, 0.05) / N(0, 0.5) of the other fixtures: words held to
#           north_star's +-20 ms;
#   c4dw02  the bench's own N(0, 0.02) / N(0, 0.02): the alignment heads
#           attend near-uniformly, DTW anchors move on near-ties (words up to 1.7 s apart on the
#           GPU), so text and speakers are held exact and word times reported.
# Speakers: c4d runs the reference's defaults -- threshold 0.5 (src/engine.rs:103), max_speakers
# None (usize::MAX, src/engine.rs:108-111) -- on the speaker-conditioned CAM++
# (make_cam_conditioning.py: the synthetic network with a last layer fitted on a calibration
# recording; the GPU loads it from an ONNX file, tests/model_writers.py): the 54 spurts come out
# as their 3 ground-truth speakers with decision margins >= 1e-2.  c4dw02 keeps the plain synthetic
# CAM++, which puts every embedding within cosine 0.9997-1.0 of every other, at threshold 0.9999
# and max_speakers 3 (margins down to 7.7e-7).  The fixture records each assignment's margin.
DIAR = dict(file="c4_large_v3_diarize_300s.json", model="large-v3", seconds=300.0, seed=1, n_speakers=3,
            weight_std=WSTD, emb_std=EMB_STD, max_speakers=None, threshold=0.5, cam="conditioned")
DIAR_W02 = dict(DIAR, file="c4_large_v3_diarize_300s_w02.json", weight_std=0.02, emb_std=0.02, max_speakers=3,
                threshold=0.9999, cam="synthetic")
CAM_COND = os.path.join(HERE, "cam_conditioning.npz")


def _seg(s):
    return dict(start=s.start, end=s.end, text=s.text,
                words=None if s.words is None else [[w.text, w.start, w.end] for w in s.words])


def make_diarized(c):
    from oracle import diarize as D
    from oracle.model import Whisper
    from oracle.pipeline import SpeechSegment as OSeg
    from oracle.pipeline import run_transcription_pipeline
    from oracle.vocab import Vocab
    from oracle.weights import hparams_for, synth_weights
    from oracle.whisper_full import WhisperState
    from wdr.synth import synth_speech

    t0 = time.time()
    pcm, spurts = synth_speech(c["seconds"], seed=c["seed"], n_speakers=c["n_speakers"])
    segs = [OSeg(a, b, pcm[int(round(a * 16000)):int(round(b * 16000))]) for a, b, _ in spurts]
    W = D.cam_weights_conditioned(CAM_COND) if c.get("cam") == "conditioned" else D.cam_weights()
    embs = [D.compute_embedding(s.samples, W) for s in segs]
    mgr = D.EmbeddingManager(c["max_speakers"] or 2 ** 64 - 1)   # None / Some(0) -> usize::MAX
    margins = []

    def speaker_of(i):
        e = embs[i]
        if e is not None and mgr.speakers:
            sims = sorted((float(D.EmbeddingManager.cosine(e, v)) for v in mgr.speakers.values()), reverse=True)
            full = len(mgr.speakers) == mgr.max_speakers
            # distance of the decision from flipping: best vs runner-up, and (search) best vs threshold
            m = sims[0] - sims[1] if len(sims) > 1 else np.inf
            if not full:
                m = min(m, abs(sims[0] - c["threshold"]))
            margins.append(m)
        else:
            margins.append(None)
        return mgr.assign(e, c["threshold"])

    hp = hparams_for(c["model"])
    st = WhisperState(Whisper(hp, synth_weights(hp, std=c["weight_std"], emb_std=c["emb_std"])),
                      Vocab(hp.n_vocab), c["model"])
    o = dict(lang="auto", advanced=dict(sampling_strategy="greedy"),
             synthetic=dict(force_len_rate=FORCE_LEN, logprob_thold=-np.inf, entropy_thold=-1.0))
    raw, lang = run_transcription_pipeline(st, segs, o, speaker_of=speaker_of)
    out = dict(config=dict(c, force_len_rate=FORCE_LEN, lang="auto", greedy=True, fallback=False,
                           segmentation="ground-truth spurts"),
               spurts=[[a, b, k] for a, b, k in spurts], lang=lang,
               raw=[dict(_seg(s), speaker_id=s.speaker_id) for s in raw],
               speaker_margins=[None if m is None or not np.isfinite(m) else m for m in margins],
               oracle_seconds=round(time.time() - t0, 1))
    with open(os.path.join(HERE, c["file"]), "w") as f:
        json.dump(out, f, indent=0)
    print("c4d", c["file"], "segments", len(raw), "speakers", "".join(s.speaker_id for s in raw),
          "s", out["oracle_seconds"], flush=True)


def make(key):
    from oracle import formatting as F
    from oracle.model import Whisper
    from oracle.pipeline import SpeechSegment as OSeg
    from oracle.pipeline import run_transcription_pipeline
    from oracle.vad import get_segments as oracle_vad
    from oracle.vocab import Vocab
    from oracle.weights import hparams_for, synth_weights
    from oracle.whisper_full import WhisperState
    from wdr.synth import synth_speech

    c = CONFIGS[key]
    t0 = time.time()
    pcm, _ = synth_speech(c["seconds"], seed=c["seed"])
    if c["vad"]:
        mask, vsegs = oracle_vad(pcm)
    else:
        mask, vsegs = None, [OSeg(0.0, len(pcm) / 16000.0, pcm)]
    hp = hparams_for(c["model"])
    st = WhisperState(Whisper(hp, synth_weights(hp, std=WSTD, emb_std=EMB_STD)), Vocab(hp.n_vocab), c["model"])
    syn = dict(force_len_rate=FORCE_LEN)
    if not c["fallback"]:
        syn.update(logprob_thold=-np.inf, entropy_thold=-1.0)
    o = dict(lang="auto", synthetic=syn)
    if c["greedy"]:
        o["advanced"] = dict(sampling_strategy="greedy")
    raw, lang = run_transcription_pipeline(st, [OSeg(s.start, s.end, s.samples) for s in vsegs], o)
    want = F.process_segments([F.Seg(s.start, s.end, s.text, None if s.words is None else
                                     [F.Word(w.text, w.start, w.end, w.probability) for w in s.words], None)
                               for s in raw], F.config_for_language(lang or "auto"), mask)
    out = dict(config=dict(model=c["model"], seconds=c["seconds"], seed=c["seed"], vad=c["vad"],
                           greedy=c["greedy"], fallback=c["fallback"], weight_std=WSTD, emb_std=EMB_STD,
                           force_len_rate=FORCE_LEN, lang="auto"),
               vad_mask=None if mask is None else [[a, b] for a, b in mask],
               vad_segments=[[s.start, s.end] for s in vsegs],
               lang=lang, raw=[_seg(s) for s in raw], formatted=[_seg(s) for s in want],
               oracle_seconds=round(time.time() - t0, 1))
    with open(os.path.join(HERE, c["file"]), "w") as f:
        json.dump(out, f, indent=0)
    print(key, c["file"], "segments", len(raw), "cues", len(want), "s", out["oracle_seconds"], flush=True)


if __name__ == "__main__":
    for k in (sys.argv[1:] or list(CONFIGS) + ["c4d", "c4dw02"]):
        if k in ("c4d", "c4dw02"):
            make_diarized(DIAR if k == "c4d" else DIAR_W02)
        else:
            make(k)
