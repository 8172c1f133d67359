# final HEAD check: chain / whisper GPU suites, smoke, the default bench line
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_chains.py tests/test_gpu_whisper.py tests/test_gpu_kernels.py > gpurun_out/t_final.log 2>&1
tail -1 gpurun_out/t_final.log
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_head.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('beam5') or {}).get('value'))"
