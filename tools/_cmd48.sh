set -e -o pipefail
mkdir -p gpurun_out/sync
WDR_THREAD_CPU=1 WDR_BENCH_THREADS=1 timeout -k 10 300 python3 bench.py --seg diarize --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/sync/thr.json 2> gpurun_out/sync/thr.err
python3 -c "import json;d=json.load(open('gpurun_out/sync/thr.json'));print(d['value']);print(json.dumps(d['host_cpu']))"
grep "wdr-cpu" gpurun_out/sync/thr.err | tail -40 | awk '{u+=$5; s+=$7; v+=$9; iv+=$11} END {print "last40 chains user",u,"sys",s,"vcsw",v,"ivcsw",iv}'
grep "wdr-cpu" gpurun_out/sync/thr.err | tail -3
