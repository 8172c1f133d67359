# k_gemm4 / k_gemm5 / k_gemm2 transposed-accumulator vector epilogue + 7-instruction GELU:
# kernel tests (bit identity with k_gemm), rows_bench from HBM and from cache, the encoder-shape
# microbenchmark, a same-box A/B of the bench (HEAD vs the build before these changes vs the
# round-4 first rows engine), and one bench run with the batch log
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_k.log 2>&1 || { tail -40 gpurun_out/t_k.log; exit 1; }
tail -2 gpurun_out/t_k.log
timeout -k 10 120 ./tools/rows_bench 1 8 16 24 32 56 > gpurun_out/rows_bench_hbm.txt 2>&1 && cat gpurun_out/rows_bench_hbm.txt
RB_COPIES=1 timeout -k 10 120 ./tools/rows_bench 1 8 16 24 32 56 > gpurun_out/rows_bench_cache.txt 2>&1 && cat gpurun_out/rows_bench_cache.txt
timeout -k 10 180 ./tools/gemm_bench 6000 > gpurun_out/gemm_bench_epi4.txt 2>&1 && grep -E "gemm4|gemm5|flash|differ" gpurun_out/gemm_bench_epi4.txt
B1="WDR_AB_LIB=$PWD/tools/_ab/libwdr_93c26ba.so"
B0="WDR_AB_LIB=$PWD/tools/_ab/libwdr_48c4668.so"
tools/ab_env.sh "" "$B1" "$B0" "" "$B1" "$B0" 2>&1 | tee gpurun_out/ab_epi4.txt
WDR_BATCH_LOG=gpurun_out/blog_r4.txt timeout -k 10 240 python3 bench.py --no-cpu-baseline --prof none > gpurun_out/bench_blog.json 2> gpurun_out/bench_blog.err && python3 tools/batch_log.py gpurun_out/blog_r4.txt
