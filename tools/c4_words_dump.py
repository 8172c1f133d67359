"""Dump the GPU's diarized-pipeline words for a c4 fixture (the test's run) beside the oracle's,
raw (no overlap clip) and clipped, for the word-time near-tie analysis.
Run on the GPU box: python tools/c4_words_dump.py c4_large_v3_diarize_300s_w02.json
-> gpurun_out/c4_words_<name>.json"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "whisper-diarize-rs_amd"))
import wdr  # noqa: E402
from wdr.synth import synth_speech  # noqa: E402


def main():
    name = sys.argv[1]
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", name)))
    c = fx["config"]
    pcm, spurts = synth_speech(c["seconds"], seed=c["seed"], n_speakers=c["n_speakers"])
    segs = [wdr.SpeechSegment(a, b, pcm[int(round(a * 16000)):int(round(b * 16000))]) for a, b, _ in spurts]
    syn = wdr.Synthetic(weight_std=c["weight_std"], emb_std=c["emb_std"], force_len_rate=c["force_len_rate"],
                        disable_fallback=True)
    ctx = wdr.WhisperContext(c["model"], enable_dtw=True, synthetic=syn)
    opts = wdr.TranscribeOptions(model=c["model"], lang="auto", enable_vad=False,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    raw, _, idx = ctx.run_pipeline_raw(segs, opts)
    out = dict(raw=[dict(i=i, start=s.start, end=s.end, text=s.text,
                         words=[[w.text, w.start, w.end] for w in (s.words or [])]) for s, i in zip(raw, idx)])
    # per-token data of every segment decoded alone from the oracle's prompt
    toks = []
    for i, sg in enumerate(segs):
        prompt = next((w["text"] for w in reversed(fx["raw"][:i]) if w["text"].strip()), None)
        r, _ = ctx.state_full(np.asarray(sg.samples, np.float32) / 32768.0, opts, initial_prompt=prompt)
        toks.append([[dict(id=t["id"], p=t["p"], pt=t["pt"], ptsum=t["ptsum"], t0=t["t0"], t1=t["t1"],
                           t_dtw=t["t_dtw"]) for t in s["tokens"]] for s in r])
    out["tokens"] = toks
    ctx.close()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "c4_words_" + name), "w"))
    print("ok", len(raw))


if __name__ == "__main__":
    main()
