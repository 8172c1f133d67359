# the default bench line at HEAD (live roofline from profiled graph replays), then the unlocked
# rocprofv3 kernel trace of the benched configuration (tools/round_profile.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 bench.py > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err || { tail -20 gpurun_out/bench_head.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_head.json')); print(d['value'], json.dumps(d['roofline']))"
LOCK=0 bash tools/round_profile.sh r04 3600
