# cost of the live profiler on the headline run: profiler on (default) vs --prof none, 2 rounds
set -e -o pipefail
mkdir -p gpurun_out/abp
for r in 1 2; do
  for v in "" "--prof none"; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --beam-seconds 0 $v > gpurun_out/abp/run.json 2> gpurun_out/abp/run.err
    python3 -c "import json,sys; d=json.load(open('gpurun_out/abp/run.json')); print('%-28s xRT %7.1f  launches %d' % (sys.argv[1] or '(profiler on)', d['value'], d['counts']['batch_launches']), flush=True)" "$v"
  done
done
