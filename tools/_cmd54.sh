set -e -o pipefail
mkdir -p gpurun_out/sync
for r in 1 2; do
for v in "poll:-" "sync:WDR_READY_POLL_US=0"; do
  n=${v%%:*}; e=${v#*:}; [ "$e" = "-" ] && e=""
  env $e WDR_BENCH_THROTTLE_LOG=1 timeout -k 10 300 python3 bench.py --seg diarize --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/sync/$n.json 2> gpurun_out/sync/$n.err
  python3 -c "import json;d=json.load(open('gpurun_out/sync/$n.json'));h=d['host_cpu'];print('$r $n',d['value'],d['stages_s'].get('batch_step_s'),h['cpu_s'],h['cg_throttled'],h['throttle_at_s'])"
done
done
