set -e -o pipefail
mkdir -p gpurun_out/lines
for v in "fp8:--fp8" "vad:--seg vad" "diarize:--seg diarize" "beam:--strategy beam --seconds 900"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 400 python3 bench.py $a --no-cpu-baseline --beam-seconds 0 > gpurun_out/lines/$n.json 2> gpurun_out/lines/$n.err
  python3 -c "import json;d=json.load(open('gpurun_out/lines/$n.json'));print('$n',d['value'],'batch_step',d['stages_s'].get('batch_step_s'),'frac',d['roofline'].get('frac'))"
done
