set -e -o pipefail
mkdir -p gpurun_out/ab
for v in "vad3:vad:3" "dia1:diarize:1" "vad1:vad:1" "dia3:diarize:3"; do
  n=${v%%:*}; r=${v#*:}; seg=${r%%:*}; sp=${r#*:}
  timeout -k 10 300 python3 bench.py --seg $seg --speakers $sp --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/ab/sp_$n.json 2> gpurun_out/ab/sp_$n.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab/sp_$n.json'));s=d['stages_s'];print('$n',d['value'],'batch_step',s.get('batch_step_s'),'launches',d['counts'].get('batch_launches'),'segs',d['config']['global_batch'],'windows',d['counts'].get('windows'))"
done
