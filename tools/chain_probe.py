"""Multi-chain probe: wall time and phase split of run_pipeline on one GPU for several chain
counts (large-v3 synthetic, bench.py's workload pin).  Prints one JSON line per chain count.
Run with WDR_DECODE_CHAINS >= the largest count asked for."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "whisper-diarize-rs_amd")]
import wdr  # noqa: E402
from wdr.synth import synth_speech  # noqa: E402


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 600.0
    counts = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,4,8").split(",")]
    model = sys.argv[3] if len(sys.argv) > 3 else "large-v3"
    pcm, spurts = synth_speech(seconds, seed=0, n_speakers=3)
    segs = [wdr.SpeechSegment(a, b, pcm[int(round(a * 16000)):int(round(b * 16000))]) for a, b, _ in spurts]
    syn = wdr.Synthetic(weight_std=0.02, emb_std=0.02, force_len_rate=3.3, disable_fallback=True)
    ctx = wdr.WhisperContext(model, enable_dtw=True, synthetic=syn)
    opts = wdr.TranscribeOptions(model=model, lang="auto",
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    ref = None
    for C in counts:
        ctx.set_chains(C)
        ctx.run_pipeline(segs, opts)          # warm-up (graphs, encode ring)
        t = time.perf_counter()
        out, _ = ctx.run_pipeline(segs, opts)
        dt = time.perf_counter() - t
        st = ctx.stage_times()
        texts = [s.text for s in out]
        if ref is None:
            ref = texts
        print(json.dumps({"chains": C, "segments": len(segs), "wall_s": round(dt, 3), "xrt": round(seconds / dt, 1),
                          "same_text": texts == ref,
                          **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()}}), flush=True)


if __name__ == "__main__":
    main()
