set -e -o pipefail
mkdir -p gpurun_out/sync
WDR_BENCH_THROTTLE_LOG=1 timeout -k 10 300 python3 bench.py --seg diarize --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/sync/tl.json 2> gpurun_out/sync/tl.err
python3 -c "import json;d=json.load(open('gpurun_out/sync/tl.json'));print(d['value'],d['host_cpu'])"
