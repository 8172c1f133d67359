#!/usr/bin/env python3
"""Batched-step probe: host ms per multi-chain step (StepBatcher, graph replay unless
WDR_NO_GRAPH) at R = 1..8 rows on one encoded large-v3 window (synthetic weights).  Run under
rocprofv3 --kernel-trace (WDR_NO_GRAPH=1) for per-kernel durations by row count."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "whisper-diarize-rs_amd")]
import numpy as np  # noqa: E402
import wdr  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "large-v3"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
rows = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2,3,4,5,6,7,8").split(",")]
ctx = wdr.WhisperContext(name, synthetic=wdr.Synthetic())
hp = ctx.hparams
mel = (np.random.default_rng(0).standard_normal((hp["n_mels"], 3000)) * 0.4).astype(np.float32)
ctx.encode(mel)
toks = [50258, 50259, 50359, 50364] + list(range(1000, 1040))
for R in rows:
    ms = ctx.batch_step_ms(toks, R, iters)
    print("R=%d: %.3f ms per step, %.3f ms per row" % (R, ms, ms / R), flush=True)
