set -e -o pipefail
mkdir -p gpurun_out/sync
for v in base blocking yield; do
  e=""; [ $v != base ] && e="WDR_SYNC_MODE=$v"
  env $e timeout -k 10 300 python3 bench.py --seg diarize --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/sync/$v.json 2> gpurun_out/sync/$v.err
  grep "hipSetDeviceFlags" gpurun_out/sync/$v.err || true
  python3 -c "import json;d=json.load(open('gpurun_out/sync/$v.json'));print('$v',d['value'],d['stages_s'].get('batch_step_s'),d['host_cpu'])"
done
