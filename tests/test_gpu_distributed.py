"""Multi-GPU one-file path with the HIP pipeline: two ranks (gloo collectives, both on cuda:0 --
the test box has one GPU) run tools/dist_transcribe.py over one file; rank 0's merged result
must equal ONE process's run_pipeline (with diarization: CAM++ embeddings + speaker
assignment in C++) over the same speech segments exactly: text, times, words, speaker ids.
The pyannote window shards + stitching are covered bit-exactly on CPU (test_distributed.py).  The ranks are child processes of
torch.distributed.run (started with subprocess, never exec'd from this GPU-initialised
process)."""
import dataclasses
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import wdr
from wdr.synth import synth_speech

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("seg", ["diarize", "vad"])
def test_two_ranks_match_one_process(tmp_path, seg):
    pcm, spurts = synth_speech(45.0, seed=7, n_speakers=2)
    spurts = [(a, b) for a, b, _ in spurts]
    p = str(tmp_path / "pcm.npy")
    np.save(p, pcm)
    json.dump(spurts, open(p + ".json", "w"))
    out = str(tmp_path / "out.json")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tools", "dist_transcribe.py"), p, "--model", "tiny-test", "--seg", seg,
           "--backend", "gloo", "--device", "0", "--lang", "auto", "--strategy", "greedy", "--emb-std", "0.5",
           "--force-len", "3.3", "--out", out, "--spurts", p + ".json"]
    r = subprocess.run(cmd, timeout=240, capture_output=True, text=True,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.load(open(out))

    syn = wdr.Synthetic(weight_std=0.02, emb_std=0.5, force_len_rate=3.3, disable_fallback=True)
    ctx = wdr.WhisperContext("tiny-test", gpu_device=0, synthetic=syn)
    opts = wdr.TranscribeOptions(model="tiny-test", lang="auto", enable_vad=seg == "vad",
                                 enable_diarize=True if seg == "diarize" else None,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
    # synthetic workload pin (as bench.py): the segmentation kernels run on the ranks, the
    # speech segments handed downstream are the generator's talk spurts
    segs = [wdr.SpeechSegment(a, b, pcm[int(round(a * 16000)):int(round(b * 16000))]) for a, b in spurts]
    ref, lang = ctx.run_pipeline(segs, opts, diarize_options=wdr.DiarizeOptions.from_options(opts)
                                 if seg == "diarize" else None)
    ctx.close()
    assert len(ref) >= 4
    assert got["lang"] == lang
    assert [s["text"] for s in got["segments"]] == [s.text for s in ref]
    for g, r_ in zip(got["segments"], ref):
        rd = dataclasses.asdict(r_)
        assert (g["start"], g["end"], g["speaker_id"]) == (rd["start"], rd["end"], rd["speaker_id"])
        assert g["words"] == rd["words"]
