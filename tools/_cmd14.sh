set -e -o pipefail
mkdir -p gpurun_out/ab
for v in "vad_ka20k:--seg vad --keepalive 20000" "vad_ka200k:--seg vad --keepalive 200000" "vad:--seg vad"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python3 bench.py $a --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/ab/k_$n.json 2> gpurun_out/ab/k_$n.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab/k_$n.json'));s=d['stages_s'];print('$n',d['value'],'batch_step',s.get('batch_step_s'),'launches',d['counts'].get('batch_launches'))"
done
