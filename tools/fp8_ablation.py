"""configs[4] fp8 encoder: where the transcript flips come from.

On the C3 900-s fixture's audio and weights (tests/golden/c3_large_v3_900s.json: large-v3,
Silero VAD, greedy, DTW, lang auto, alignment-conditioned N(0, 0.05) weights), for each fp8 plan
(Context::fp8_plan: which projections of which encoder layers run MX e4m3; WDR_FP8_PLAN /
WDR_FP8_PROJ / WDR_FP8_F16_HEAD / WDR_FP8_F16_TAIL):

  * pipeline  -- Engine::transcribe_audio against the fixture's formatted cues (the oracle's):
                 cues with identical text in order, and the word / cue bounds of those within
                 20 ms -- the prompt chain (src/transcribe.rs:384-386,502) carries every flip
                 into the following segments;
  * teacher   -- teacher-forced: every VAD segment decoded alone (wdr_state_full) from the
                 prompt the f16 path leaves before it (the f16 path equals the oracle on this
                 fixture, tests/test_gpu_configs.py), its text compared with the f16 path's --
                 the per-segment flip rate without the chain's amplification.

Appends one JSON record per plan to gpurun_out/fp8_ablation.jsonl.
Run on the GPU box:  python tools/fp8_ablation.py [plan ...]   (plan = name=ENV=VALUE[,ENV=VALUE])
"""
import json
import os
import struct
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "whisper-diarize-rs_amd"))

import wdr  # noqa: E402
from wdr.synth import synth_speech  # noqa: E402

OUT = os.path.join(ROOT, "gpurun_out", "fp8_ablation.jsonl")
TOL = 0.02 + 1e-9
ENVS = ("WDR_FP8_ENCODER", "WDR_FP8_PLAN", "WDR_FP8_PROJ", "WDR_FP8_F16_HEAD", "WDR_FP8_F16_TAIL")

PLANS = [
    ("f16", {"WDR_FP8_ENCODER": "0"}),
    ("all", {}),
    ("qkv", {"WDR_FP8_PROJ": "1"}),
    ("o", {"WDR_FP8_PROJ": "2"}),
    ("fc1", {"WDR_FP8_PROJ": "4"}),
    ("fc2", {"WDR_FP8_PROJ": "8"}),
    ("mlp", {"WDR_FP8_PROJ": "c"}),
    ("all_head8", {"WDR_FP8_F16_HEAD": "8"}),
    ("all_tail8", {"WDR_FP8_F16_TAIL": "8"}),
]


def write_wav(path, samples):
    s = np.asarray(samples, np.int16).tobytes()
    hdr = b"RIFF" + struct.pack("<I", 36 + len(s)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, 1, 1, 16000, 32000, 2, 16) + b"data" + struct.pack("<I", len(s))
    with open(path, "wb") as f:
        f.write(hdr + s)


def set_plan(env):
    for k in ENVS:
        os.environ.pop(k, None)
    os.environ["WDR_FP8_ENCODER"] = "1"
    os.environ.update(env)


def main():
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "c3_large_v3_900s.json")))
    c = fx["config"]
    pcm, _ = synth_speech(c["seconds"], seed=c["seed"])
    syn = wdr.Synthetic(weight_std=c["weight_std"], emb_std=c["emb_std"], force_len_rate=c["force_len_rate"],
                        disable_fallback=True)
    greedy = wdr.AdvancedTranscribe(sampling_strategy="greedy")
    tmp = tempfile.mkdtemp()
    wav = os.path.join(tmp, "a.wav")
    write_wav(wav, pcm)
    _, vsegs = wdr.Vad().get_segments(pcm)
    segs = [wdr.SpeechSegment(s.start, s.end, s.samples) for s in vsegs]
    plans = PLANS
    if len(sys.argv) > 1:
        plans = []
        for a in sys.argv[1:]:
            name, _, kv = a.partition("=")
            plans.append((name, dict(x.split("=", 1) for x in kv.split(",") if x)))

    # the f16 path's per-segment texts and the prompt entering each segment (teacher forcing)
    set_plan({"WDR_FP8_ENCODER": "0"})
    ctx = wdr.WhisperContext(c["model"], enable_dtw=True, synthetic=syn)
    opts = wdr.TranscribeOptions(model=c["model"], lang="auto", advanced=greedy)
    ref, _, index = ctx.run_pipeline_raw(segs, opts)
    ctx.close()
    ref_txt = [[] for _ in segs]
    for s, i in zip(ref, index):
        ref_txt[i].append(s.text.lstrip())
    prompts, prev = [], None
    for i in range(len(segs)):
        prompts.append(prev)
        for t in ref_txt[i]:
            if t.strip():
                prev = t

    for name, env in plans:
        set_plan(env)
        t0 = time.time()
        eng = wdr.Engine(wdr.EngineConfig(cache_dir=os.path.join(tmp, "cache")), synthetic=syn)
        got = eng.transcribe_audio(wav, wdr.TranscribeOptions(model=c["model"], enable_vad=True, advanced=greedy))
        eng.close()
        want = fx["formatted"]
        same = [(g, w) for g, w in zip(got, want) if g.text == w["text"]]
        dts = []
        for g, w in same:
            gw, ww = g.words or [], w["words"] or []
            if [a.text for a in gw] == [b[0] for b in ww]:
                dts += [abs(a.start - b[1]) for a, b in zip(gw, ww)] + [abs(a.end - b[2]) for a, b in zip(gw, ww)]
            dts += [abs(g.start - w["start"]), abs(g.end - w["end"])]
        dts = np.array(dts) if dts else np.zeros(1)
        first_diff = next((k for k, (g, w) in enumerate(zip(got, want)) if g.text != w["text"]), None)
        # teacher-forced
        ctx = wdr.WhisperContext(c["model"], enable_dtw=True, synthetic=syn)
        tf_same, tf_diff = 0, []
        for i, s in enumerate(segs):
            out, _ = ctx.state_full(np.asarray(s.samples, np.float32) / 32768.0, opts, initial_prompt=prompts[i])
            txt = [r["text"].lstrip() for r in out]
            if txt == ref_txt[i]:
                tf_same += 1
            else:
                tf_diff.append(i)
        ctx.close()
        rec = dict(plan=name, env=env, cues=len(got), cues_oracle=len(want), same_text_in_order=len(same),
                   first_cue_diff=first_diff, bounds_within_20ms=float((dts <= TOL).mean()),
                   bound_max_dt=float(dts.max()), teacher_forced_same=tf_same, segments=len(segs),
                   teacher_forced_diff=tf_diff, seconds=round(time.time() - t0, 1))
        print(json.dumps(rec), flush=True)
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        with open(OUT, "a") as f:
            f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
