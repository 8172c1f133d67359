# partial batches (WDR_BATCH_WAIT_US) + cheaper kernel clock: the chain tests, then the bench with
# the live profiler on (default) and off, and the batch-wait A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_chains.py tests/test_gpu_step.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_h.log 2>&1 || { tail -40 gpurun_out/t_h.log; exit 1; }
tail -2 gpurun_out/t_h.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --beam-seconds 0 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err && python3 -c "
import json; d=json.load(open('gpurun_out/bench_prof.json')); print('prof on', d['value']); [print(k, v['achieved'], v['avg_launch_us']) for k, v in d['roofline_classes'].items()]"
tools/ab_env.sh "" "WDR_BATCH_WAIT_US=-1" "WDR_BATCH_WAIT_US=100" "WDR_BATCH_WAIT_US=1000" "" "WDR_BATCH_WAIT_US=-1" 2>&1 | tee gpurun_out/ab_wait.txt
