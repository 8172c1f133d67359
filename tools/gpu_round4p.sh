# two row tiles per workgroup above 32 rows: kernel + chain tests, then the A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_chains.py tests/test_gpu_step.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_p.log 2>&1 || { tail -40 gpurun_out/t_p.log; exit 1; }
tail -2 gpurun_out/t_p.log
timeout -k 10 120 ./tools/rows_bench 16 40 56 > gpurun_out/rows_bench_pair.txt 2>&1 && cat gpurun_out/rows_bench_pair.txt
tools/ab_env.sh "" "WDR_ROWS_PAIR=0" "" "WDR_ROWS_PAIR=0" 2>&1 | tee gpurun_out/ab_pair.txt
