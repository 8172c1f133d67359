#!/usr/bin/env python3
"""Transcribe ONE file across the GPUs of a node (wdr/distributed.py).

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        tools/dist_transcribe.py audio.wav --model large-v3 --seg diarize > segments.json

One process per GPU (LOCAL_RANK -> device); collectives over RCCL ("nccl") by default, gloo
with --backend gloo (several ranks may then share one GPU, as the GPU test does).  Rank 0
reads the file and prints the segments as JSON.  Weights are the seeded synthetic ones (no
checkpoints on this machine; --emb-std / --force-len as wdr.Synthetic)."""
import argparse
import dataclasses
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "whisper-diarize-rs_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("audio", help=".wav (16 kHz mono int16) or .npy int16 samples")
    ap.add_argument("--model", default="base")
    ap.add_argument("--seg", default="diarize", choices=["diarize", "vad", "none"])
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--device", type=int, default=None, help="GPU for every rank (default LOCAL_RANK)")
    ap.add_argument("--lang", default="auto")
    ap.add_argument("--strategy", default=None, help="greedy | beam_search (reference default)")
    ap.add_argument("--emb-std", type=float, default=0.02)
    ap.add_argument("--force-len", type=float, default=0.0)
    ap.add_argument("--out", default=None, help="write rank 0's JSON here instead of stdout")
    ap.add_argument("--spurts", default=None,
                    help="JSON [[start_s, end_s], ...]: synthetic workload pin -- the segmentation kernels "
                         "still run (sharded), the speech segments handed downstream are these")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist
    import wdr
    from wdr import distributed as D

    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = args.device if args.device is not None else local
    if args.backend == "nccl":
        torch.cuda.set_device(dev)
    dist.init_process_group(backend=args.backend)
    rank = dist.get_rank()
    pcm = None
    if rank == 0:
        pcm = np.load(args.audio) if args.audio.endswith(".npy") else wdr.read_wav(args.audio)
    syn = wdr.Synthetic(weight_std=0.02, emb_std=args.emb_std, force_len_rate=args.force_len,
                        disable_fallback=args.force_len > 0)
    ctx = wdr.WhisperContext(args.model, gpu_device=dev, synthetic=syn)
    dia = wdr.Diarizer(gpu_device=dev) if args.seg == "diarize" else None
    vad = wdr.Vad(gpu_device=dev) if args.seg == "vad" and rank == 0 else None
    opts = wdr.TranscribeOptions(model=args.model, lang=args.lang, enable_vad=args.seg == "vad",
                                 enable_diarize=True if args.seg == "diarize" else None,
                                 advanced=wdr.AdvancedTranscribe(sampling_strategy=args.strategy))
    pin = None
    if args.spurts and rank == 0:
        spurts = json.load(open(args.spurts))

        def pinned(*a):
            if args.seg == "vad":
                vad.get_segments(pcm)   # runs and is discarded (the pin)
            return [wdr.SpeechSegment(x, y, pcm[int(round(x * 16000)):int(round(y * 16000))]) for x, y in spurts]
        pin = pinned
    import time
    dist.barrier()
    t0 = time.perf_counter()
    res = D.transcribe_file(pcm, opts, ctx=ctx, segmentation=args.seg, diarizer=dia, vad=vad,
                            speech_segments_fn=pin)
    dist.barrier()
    wall = time.perf_counter() - t0
    print("rank %d: wall %.3f s, block %s" % (rank, wall, json.dumps(D.last_stats)), file=sys.stderr, flush=True)
    if rank == 0:
        segs, lang = res
        doc = json.dumps({"lang": lang, "segments": [dataclasses.asdict(s) for s in segs]})
        if args.out:
            open(args.out, "w").write(doc)
        else:
            print(doc)
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
