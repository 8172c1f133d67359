# flash lazy rescale + the configs[3] 8-model test with per-model pools sized for 3 chains, then
# the scheduling A/B at the new kernel speeds (decode chains, encoder CU mask)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_multidevice.py tests/test_gpu_step.py tests/test_gpu_whisper.py -x -q --timeout 400 --timeout-method thread > gpurun_out/t_f.log 2>&1 || { tail -40 gpurun_out/t_f.log; exit 1; }
tail -2 gpurun_out/t_f.log
timeout -k 10 180 ./tools/gemm_bench 6000 > gpurun_out/gemm_bench_f.txt 2>&1 && grep -E "flash" gpurun_out/gemm_bench_f.txt
tools/ab_env.sh "" "WDR_DECODE_CHAINS=32" "WDR_DECODE_CHAINS=40" "WDR_ENC_MASK=16" "WDR_ENC_MASK=48" "" "WDR_DECODE_CHAINS=32" "WDR_ENC_MASK=0" 2>&1 | tee gpurun_out/ab_sched4.txt
