set -e -o pipefail
mkdir -p gpurun_out/sync
for r in 1 2; do
for v in blk spin; do
  e=""; [ $v = spin ] && e="WDR_BLOCKING_EVENTS=0"
  env $e WDR_THREAD_CPU=1 timeout -k 10 300 python3 bench.py --seg diarize --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/sync/$v.json 2> gpurun_out/sync/$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/sync/$v.json'));h=d['host_cpu'];print('$r $v',d['value'],d['stages_s'].get('batch_step_s'),h['cpu_s'],h['cg_throttled'],h['cg_throttled_s'])"
done
done
