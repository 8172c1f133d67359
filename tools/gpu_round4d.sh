# k_skinny rows engine restored on top of the vector GEMM epilogues + log2 flash: the GPU suites
# touching kernels and the decoder, rows_bench (HBM / cache), the co-scheduling probe, and a
# same-box A/B against the build before the restore (rows v2) and the round-4 k_skinny build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_whisper.py tests/test_gpu_step.py tests/test_gpu_chains.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_d.log 2>&1 || { tail -40 gpurun_out/t_d.log; exit 1; }
tail -2 gpurun_out/t_d.log
timeout -k 10 120 ./tools/rows_bench 1 8 16 24 32 56 > gpurun_out/rows_bench_sk.txt 2>&1 && cat gpurun_out/rows_bench_sk.txt
RB_COPIES=1 timeout -k 10 120 ./tools/rows_bench 16 56 > gpurun_out/rows_bench_sk_cache.txt 2>&1 && cat gpurun_out/rows_bench_sk_cache.txt
timeout -k 10 120 ./tools/cosched_bench 16 > gpurun_out/cosched_sk.txt 2>&1 && cat gpurun_out/cosched_sk.txt
B1="WDR_AB_LIB=$PWD/tools/_ab/libwdr_c82e44a.so"
B0="WDR_AB_LIB=$PWD/tools/_ab/libwdr_48c4668.so"
tools/ab_env.sh "" "$B1" "$B0" "" "$B1" "$B0" 2>&1 | tee gpurun_out/ab_sk.txt
