#!/bin/bash
# Round 6 against round 5's HEAD library (e09f746, no ABI change), interleaved on one box: the
# default diarize line and configs[2]'s VAD line, ROUNDS rounds; the libraries are swapped in
# place (tools/_ab/libwdr_r05.so / libwdr_r06.so, built in the container).
set -e -o pipefail
mkdir -p gpurun_out/ab
L=whisper-diarize-rs_amd/libwdr.so
trap 'cp tools/_ab/libwdr_r06.so $L' EXIT
for r in $(seq 1 ${1:-2}); do
  for lib in r06 r05; do
    cp tools/_ab/libwdr_$lib.so $L
    for seg in ${LINES:-diarize vad}; do
      out=gpurun_out/ab/lib_${lib}_${seg}_$r
      timeout -k 10 300 python3 bench.py --seg $seg --no-cpu-baseline --prof none --beam-seconds 0 > $out.json 2> $out.err
      python3 -c "import json;d=json.load(open('$out.json'));s=d['stages_s'];print('$r $lib $seg',d['value'],'batch_step',s.get('batch_step_s'),'launches',d['counts'].get('batch_launches'),'seg_gpu_ms',d['segmentation'].get('gpu_ms'))" | tee -a gpurun_out/ab/lib.txt
    done
  done
done
