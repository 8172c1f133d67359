# decode-step anatomy at HEAD: rows_bench with the weights from HBM (32 copies) and from cache
# (1 copy: the latency floor of the launch chain), and one bench run with the batch log
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/rows_bench 1 8 16 24 32 56 > gpurun_out/rows_bench_hbm.txt 2>&1 && cat gpurun_out/rows_bench_hbm.txt
RB_COPIES=1 timeout -k 10 120 ./tools/rows_bench 1 8 16 24 32 56 > gpurun_out/rows_bench_cache.txt 2>&1 && cat gpurun_out/rows_bench_cache.txt
WDR_BATCH_LOG=gpurun_out/blog_r4.txt timeout -k 10 240 python3 bench.py --no-cpu-baseline --prof none > gpurun_out/bench_blog.json 2> gpurun_out/bench_blog.err && python3 tools/batch_log.py gpurun_out/blog_r4.txt
