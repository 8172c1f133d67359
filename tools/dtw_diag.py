"""DTW anchor-drift diagnosis (VERDICT r3 "next round" item 1): which tokens' DTW anchors move
between the GPU and the oracle, and why (tests/dtw_neartie.py has the analysis).

For every DTW re-forward of a state.full run, on the SAME window and token sequence, the oracle's
alignment-head probabilities (oracle/model.py) against the GPU's (wdr_dbg_capture); the DTW
paths on both alignment matrices; the path margin (the GPU path's extra cost under the ORACLE's
matrix) against the perturbation the capture error puts on the paths.

Run on the GPU box (needs libwdr):  python tools/dtw_diag.py [--std 0.02] [--emb 0.5]
Appends one record per window + a summary to gpurun_out/dtw_diag.jsonl.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "whisper-diarize-rs_amd"))

import wdr  # noqa: E402
from oracle.mel import pcm_i16_to_f32  # noqa: E402
from oracle.model import Whisper  # noqa: E402
from oracle.vocab import Vocab  # noqa: E402
from oracle.weights import hparams_for, synth_weights  # noqa: E402
from oracle.whisper_full import FullParams, WhisperState  # noqa: E402
from tests.dtw_neartie import analyse, gpu_capture, record_dtw_calls  # noqa: E402
from wdr.synth import synth_speech  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="base.en")
    ap.add_argument("--std", type=float, default=0.02)
    ap.add_argument("--emb", type=float, default=0.5)
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--seed", type=int, default=31)
    ap.add_argument("--fallback", type=int, default=1)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "dtw_diag.jsonl"))
    a = ap.parse_args()
    name = a.model
    hp = hparams_for(name)
    m = Whisper(hp, synth_weights(hp, std=a.std, emb_std=a.emb))
    syn = wdr.Synthetic(weight_std=a.std, emb_std=a.emb, force_len_rate=3.3, disable_fallback=not a.fallback)
    ctx = wdr.WhisperContext(name, synthetic=syn)
    pcm, _ = synth_speech(a.seconds, seed=a.seed)
    x = pcm_i16_to_f32(pcm)
    got, _ = ctx.state_full(x, wdr.TranscribeOptions(lang="auto"))
    st = WhisperState(m, Vocab(hp.n_vocab), name)
    calls = record_dtw_calls(st, m)
    fb = dict(logprob_thold=-np.inf, entropy_thold=-1.0) if not a.fallback else {}
    st.full(x, FullParams(language="auto", force_len_rate=3.3, **fb))
    ref_tok = [t for r in st.result_all for t in r.tokens]
    got_tok = [t for g in got for t in g["tokens"]]
    same_ids = [t.id for t in ref_tok] == [t["id"] for t in got_tok]
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    n_anch = n_moved = n_tie = 0
    with open(a.out, "a") as f:
        for c in calls:
            r = analyse(c["qk_o"], gpu_capture(ctx, x, c, len(st.aheads)), c["n_frames"], c["sot_len"], c["seek"])
            tie = bool(r["moved"]) and r["path_margin"] <= r["perturbation"]
            n_anch += len(r["anchors_oracle"])
            n_moved += len(r["moved"])
            n_tie += len(r["moved"]) if tie else 0
            moved = [dict(token=k, id=c["tokens"][c["sot_len"] + 1 + k], oracle_cs=ao, gpu_cs=ag)
                     for k, ao, ag in r["moved"]]
            rec = dict(model=name, std=a.std, emb=a.emb, seek=c["seek"], n_frames=c["n_frames"],
                       tokens=len(c["tokens"]), cap_rel_max=r["cap_rel_max"], x_spread=r["x_spread"],
                       path_cost_oracle=r["path_cost"], path_margin=r["path_margin"],
                       perturbation_on_paths=r["perturbation"], near_tie=tie, moved=moved,
                       max_cs=max([abs(ao - ag) for _, ao, ag in r["moved"]] or [0]))
            f.write(json.dumps(rec) + "\n")
            print(json.dumps(rec))
    d = [abs(g["t_dtw"] - t.t_dtw) for g, t in zip(got_tok, ref_tok)] if same_ids else []
    summ = dict(summary=True, model=name, std=a.std, emb=a.emb, same_ids=same_ids, windows=len(calls),
                anchors=n_anch, moved_seam=n_moved, moved_at_near_tie=n_tie,
                pipeline_max_cs=max(d) if d else None, pipeline_over_2cs=sum(v > 2 for v in d) if d else None)
    with open(a.out, "a") as f:
        f.write(json.dumps(summ) + "\n")
    print(json.dumps(summ))
    ctx.close()


if __name__ == "__main__":
    main()
