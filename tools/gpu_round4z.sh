# HEAD with 40 decode chains by default: the GPU suite + smoke, then the default bench line
set -o pipefail
bash tools/gpu_suite.sh && timeout -k 10 600 python3 bench.py > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err && \
  python3 -c "import json; d=json.load(open('gpurun_out/bench_head.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('beam5') or {}).get('value'))"
