#!/bin/bash
# Interleaved A/B of env-knob variants on the default diarize line and configs[2]'s VAD line.
# usage: ab_lines.sh ROUNDS "name:ENV=V,ENV2=V2" ...   (name:- = no env); one bench run per (round,
# variant, line), summary lines in gpurun_out/ab/lines.txt; stops at the first failure
set -e -o pipefail
mkdir -p gpurun_out/ab
R=$1; shift
for r in $(seq 1 $R); do
  for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}; [ "$envs" = "-" ] && envs=""
    for seg in ${LINES:-diarize vad}; do
      out=gpurun_out/ab/${name}_${seg}_$r
      env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python3 bench.py --seg $seg --no-cpu-baseline --prof none --beam-seconds 0 > $out.json 2> $out.err
      python3 -c "import json;d=json.load(open('$out.json'));s=d['stages_s'];print('$r $name $seg',d['value'],'batch_step',s.get('batch_step_s'),'launches',d['counts'].get('batch_launches'))" | tee -a gpurun_out/ab/lines.txt
    done
  done
done
