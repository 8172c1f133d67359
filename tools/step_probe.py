#!/usr/bin/env python3
"""Decode-step probe: large-v3 (synthetic weights), one encoded window, N single-row steps
through the persistent one-launch step and through the per-kernel chain, host-timed
(prefill included; run under rocprofv3 --kernel-trace for kernel durations)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "whisper-diarize-rs_amd")]
import numpy as np  # noqa: E402
import wdr  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "large-v3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
os.environ.setdefault("WDR_PSTEP", "1")   # the persistent step is opt-in
ctx = wdr.WhisperContext(name, synthetic=wdr.Synthetic())
hp = ctx.hparams
mel = (np.random.default_rng(0).standard_normal((hp["n_mels"], 3000)) * 0.4).astype(np.float32)
ctx.encode(mel)
toks = [50258, 50259, 50359, 50364] + list(range(1000, 1040))
for classic in (False, True):
    ctx.step(toks, classic=classic)
    t = time.perf_counter()
    for _ in range(n):
        ctx.step(toks, classic=classic)
    print("%s: %.3f ms per prefill+step" % ("classic" if classic else "persistent", (time.perf_counter() - t) * 1e3 / n))

# timeline of the last persistent step (WDR_STEP_TRACE=1): per layer and event, the spread of
# thread-0 stamps over the workgroups that recorded it, in us from the first workgroup start
if os.environ.get("WDR_STEP_TRACE"):
    import ctypes as C
    ctx.step(toks)
    G = 1024
    buf = np.zeros(67 * G, np.uint64)
    g = C.c_int32()
    wdr._lib.load().wdr_dbg_step_trace(ctx.h, buf.ctypes.data_as(C.POINTER(C.c_uint64)), buf.size, C.byref(g))
    G = g.value
    tr = buf[:67 * G].reshape(67, G).astype(np.int64)
    t0 = tr[64].min()
    names = ["qkv.wait", "qkv.sig", "self.wait", "self.sig", "o.wait", "o.sig", "xq.wait", "xq.sig",
             "xatt.wait", "comb.sig", "xo.wait", "xo.sig", "fc1.wait", "fc1.sig", "fc2.wait", "fc2.sig"]
    print("start spread %.2f us" % ((tr[64].max() - t0) / 100.0))
    for l in range(4):
        for e in range(16):
            v = tr[l * 16 + e]
            v = v[v >= t0]
            if v.size:
                print("L%d %-10s n=%3d  min %8.2f  max %8.2f us" % (l, names[e], v.size, (v.min() - t0) / 100.0,
                                                                    (v.max() - t0) / 100.0))
    for e, nm in ((65, "logits.wait"), (66, "end")):
        v = tr[e][tr[e] >= t0]
        print("%-14s min %8.2f  max %8.2f us" % (nm, (v.min() - t0) / 100.0, (v.max() - t0) / 100.0))
