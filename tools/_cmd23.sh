set -e -o pipefail
mkdir -p gpurun_out/ab
for v in "vad_mb64:--seg vad --keepalive-mb 64" "vad_mb8:--seg vad --keepalive-mb 8"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python3 bench.py $a --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/ab/m_$n.json 2> gpurun_out/ab/m_$n.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab/m_$n.json'));s=d['stages_s'];print('$n',d['value'],'batch_step',s.get('batch_step_s'),'launches',d['counts'].get('batch_launches'))"
done
