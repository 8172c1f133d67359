# fc1 on k_gemm5 tiles + pseudo-random live sampling: kernel tests, A/B, then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_t.log 2>&1 || { tail -30 gpurun_out/t_t.log; exit 1; }
tail -1 gpurun_out/t_t.log
tools/ab_env.sh "" "WDR_GEMM5_WIDE=0" "" "WDR_GEMM5_WIDE=0" 2>&1 | tee gpurun_out/ab_gemm5w.txt
timeout -k 10 500 python3 bench.py > gpurun_out/bench_t.json 2> gpurun_out/bench_t.err && python3 -c "
import json; d=json.load(open('gpurun_out/bench_t.json')); print(d['value']); r=d['roofline']; print({k: r.get(k) for k in ('kernel','achieved','frac','avg_launch_us','flops_per_launch','trace_achieved','trace_frac')})"
