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

Usage:  python tests/golden/make_pipeline_fixtures.py [c1|c2|c3 ...]
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
}


def _seg(s):
    return dict(start=s.start, end=s.end, text=s.text,
                words=None if s.words is None else [[w.text, w.start, w.end] for w in s.words])


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
    for k in (sys.argv[1:] or list(CONFIGS)):
        make(k)
