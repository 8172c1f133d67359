set -e -o pipefail
mkdir -p gpurun_out/sync
for v in "base:-" "raw0:ROC_ACTIVE_WAIT_TIMEOUT=0" "raw1k:ROC_ACTIVE_WAIT_TIMEOUT=1000" "blkdev:WDR_SYNC_MODE=blocking"; do
  n=${v%%:*}; e=${v#*:}; [ "$e" = "-" ] && e=""
  env $e timeout -k 10 300 python3 bench.py --seg diarize --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/sync/$n.json 2> gpurun_out/sync/$n.err
  python3 -c "import json;d=json.load(open('gpurun_out/sync/$n.json'));h=d['host_cpu'];print('$n',d['value'],d['stages_s'].get('batch_step_s'),h['cpu_s'],h['cg_throttled'],h['cg_throttled_s'])"
done
