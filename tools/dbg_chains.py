import sys, dataclasses
sys.path[:0]=['/root/repo','/root/repo/whisper-diarize-rs_amd']
import numpy as np, wdr
from wdr.synth import synth_speech
syn = wdr.Synthetic(weight_std=0.02, emb_std=0.5, force_len_rate=3.3, disable_fallback=True)
ctx = wdr.WhisperContext("tiny-test", synthetic=syn)
pcm, spurts = synth_speech(80.0, seed=11, n_speakers=2)
segs=[wdr.SpeechSegment(a, b, pcm[int(round(a*16000)):int(round(b*16000))]) for a,b,_ in spurts]
opts = wdr.TranscribeOptions(lang="auto", advanced=wdr.AdvancedTranscribe(sampling_strategy="greedy"))
res={}
for C in (1,2,1,2):
    ctx.set_chains(C)
    out,lang=ctx.run_pipeline(segs, opts)
    res.setdefault(C,[]).append([dataclasses.asdict(s) for s in out])
print("repeat C1 equal:", res[1][0]==res[1][1], " repeat C2 equal:", res[2][0]==res[2][1])
a,b=res[1][0],res[2][0]
for i,(x,y) in enumerate(zip(a,b)):
    if x!=y:
        print("seg",i, x["start"], y["start"], x["end"], y["end"])
        for w1,w2 in zip(x["words"] or [], y["words"] or []):
            if w1!=w2: print("  ", w1, "\n  ", w2)
