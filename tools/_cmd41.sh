set -e -o pipefail
LOCK=1 bash tools/round_profile.sh r06 3600
cp gpurun_out/prof_r06/classes.json profiles/r06/prof_graph/classes.json
timeout -k 10 900 python3 bench.py > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err
cat gpurun_out/bench_head.json | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['value'],d['roofline'].get('frac'),d['roofline'].get('trace_frac'),d.get('cpu_baseline',{}).get('value'))"
