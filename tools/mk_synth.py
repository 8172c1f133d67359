import sys, json, numpy as np
sys.path[:0]=['/root/repo/whisper-diarize-rs_amd']
from wdr.synth import synth_speech
pcm, sp = synth_speech(float(sys.argv[1]), seed=0)
np.save(sys.argv[2], pcm); json.dump([(a,b) for a,b,_ in sp], open(sys.argv[2]+'.json','w'))
