# the partial-batch wait with the live profiler on (the headline run's configuration): 1000 (default) vs 300 us
set -e -o pipefail
mkdir -p gpurun_out/abp
for r in 1 2; do
  for v in "" "WDR_BATCH_WAIT_US=300"; do
    env $v timeout -k 10 300 python3 bench.py --no-cpu-baseline --beam-seconds 0 > gpurun_out/abp/run.json 2> gpurun_out/abp/run.err
    python3 -c "import json,sys; d=json.load(open('gpurun_out/abp/run.json')); print('%-28s xRT %7.1f  launches %d' % (sys.argv[1] or '(default)', d['value'], d['counts']['batch_launches']), flush=True)" "$v"
  done
done
