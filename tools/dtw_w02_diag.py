"""Word-time near-ties on the bench's N(0, 0.02) weights: for the diarized
w02 fixture's segments with a bound past 20 ms, the GPU's own DTW times (wdr_state_full, the
pipeline's path) beside the GPU DTW kernels run on the debug capture of the same window and
tokens (wdr_dbg_capture + wdr_dbg_dtw), with the capture saved for the CPU-side analysis
(tests/dtw_neartie.py).  Run on the GPU box: python tools/dtw_w02_diag.py 1 13 24 25 42
-> gpurun_out/dtw_w02_diag.npz"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "whisper-diarize-rs_amd"))
import wdr  # noqa: E402
from wdr import _lib as L  # noqa: E402
from wdr.synth import synth_speech  # noqa: E402

SOT, NOT, EOT, LANG0 = 50258, 50364, 50257, 50259   # large-v3 token layout (oracle/vocab.py)


def main():
    idx = [int(a) for a in sys.argv[1:]]
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "c4_large_v3_diarize_300s_w02.json")))
    c = fx["config"]
    pcm, spurts = synth_speech(c["seconds"], seed=c["seed"], n_speakers=c["n_speakers"])
    syn = wdr.Synthetic(weight_std=c["weight_std"], emb_std=c["emb_std"], force_len_rate=c["force_len_rate"],
                        disable_fallback=True)
    ctx = wdr.WhisperContext(c["model"], enable_dtw=True, synthetic=syn)
    opts = wdr.TranscribeOptions(model=c["model"], lang="auto", enable_vad=False,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    lib = L.load()
    out = {}
    for i in idx:
        a, b, _ = spurts[i]
        x = pcm[int(round(a * 16000)):int(round(b * 16000))].astype(np.float32) / np.float32(32768.0)
        prompt = next((w["text"] for w in reversed(fx["raw"][:i]) if w["text"].strip()), None)
        res, lang = ctx.state_full(x, opts, initial_prompt=prompt)
        text = [t["id"] for s in res for t in s["tokens"] if t["id"] < EOT]
        tdtw = [t["t_dtw"] for s in res for t in s["tokens"] if t["id"] < EOT]
        toks = [SOT, LANG0 + lang, NOT] + text + [EOT]
        n_frames = 1 + (x.size + 200 - 400) // 160   # seek_end of a one-window segment
        n_frames = min(n_frames, 3000)
        ctx.encode(ctx.log_mel_window(x, 0))
        na = 16
        cap = ctx.capture(toks, na)
        while na > 1 and not cap[na - 1].any():
            na -= 1
        cap = cap[:na]
        n_audio = n_frames // 2
        xm = np.zeros((len(toks) - 3, n_audio), np.float32)
        t = np.zeros(len(toks) + 8, np.int32)
        nt = C.c_int32()
        F32, I32 = C.POINTER(C.c_float), C.POINTER(C.c_int32)
        capc = np.ascontiguousarray(cap, np.float32)
        L.check(lib.wdr_dbg_dtw(capc.ctypes.data_as(F32), na, len(toks), n_audio, 2, 0, xm.ctypes.data_as(F32),
                                t.ctypes.data_as(I32), C.byref(nt)))
        out["cap_%d" % i] = capc
        out["toks_%d" % i] = np.array(toks, np.int32)
        out["tdtw_pipe_%d" % i] = np.array(tdtw, np.int32)
        out["tdtw_dbg_%d" % i] = t[:nt.value]
        out["meta_%d" % i] = np.array([n_frames, lang], np.int32)
        print(i, "pipe", tdtw, "dbg", list(t[:nt.value]), flush=True)
    ctx.close()
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "dtw_w02_diag.npz"), **out)


if __name__ == "__main__":
    main()
