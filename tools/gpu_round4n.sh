# o / fc2 on k_gemm4's 120 tiles (one round on the encoder's 224 CUs, ~100 CUs left to decode)
# vs k_gemm5's 240 (two rounds), and a batch log of the default bench
set -o pipefail
mkdir -p gpurun_out
tools/ab_env.sh "" "WDR_GEMM5=0" "" "WDR_GEMM5=0" 2>&1 | tee gpurun_out/ab_gemm5.txt
WDR_BATCH_LOG=gpurun_out/blog_r4b.txt timeout -k 10 240 python3 bench.py --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/bench_blog2.json 2> gpurun_out/bench_blog2.err && python3 tools/batch_log.py gpurun_out/blog_r4b.txt
