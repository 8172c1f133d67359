"""configs[2] with the VAD's OWN segments downstream (not the bench's pinned spurts): 1 h of
synthetic speech, Silero VAD, large-v3 + DTW, greedy, lang auto -- long merged segments decoded
window by window through the seek loop, their later windows encoded on demand.  Times one
run_pipeline call after a warmup; for the on-demand knobs (WDR_ODM_POOL, WDR_ODM_ALT).
Run on the GPU box: python tools/vad_segments_bench.py  (one JSON line)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "whisper-diarize-rs_amd"))
import wdr  # noqa: E402
from wdr.synth import synth_speech  # noqa: E402


def main():
    pcm, _ = synth_speech(3600.0, seed=0, n_speakers=1)
    _, vsegs = wdr.Vad().get_segments(pcm)
    syn = wdr.Synthetic(weight_std=0.02, emb_std=0.02, force_len_rate=3.3, disable_fallback=True)
    ctx = wdr.WhisperContext("large-v3", enable_dtw=True, synthetic=syn)
    opts = wdr.TranscribeOptions(model="large-v3", lang="auto", enable_vad=True,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    ctx.run_pipeline(vsegs, opts)
    t = time.perf_counter()
    out, _ = ctx.run_pipeline(vsegs, opts)
    dt = time.perf_counter() - t
    st = ctx.stage_times()
    ctx.close()
    print(json.dumps(dict(xrt=round(3600.0 / dt, 1), wall_s=round(dt, 3), vad_segments=len(vsegs),
                          whisper_segments=len(out), windows=st.get("windows"), encode_s=st.get("encode"),
                          batch_step_s=st.get("batch_step_s"), knobs={k: os.environ.get(k) for k in
                                                                       ("WDR_ODM_POOL", "WDR_ODM_ALT")})))


if __name__ == "__main__":
    main()
