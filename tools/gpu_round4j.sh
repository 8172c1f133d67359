# two-head cross-attention partials: kernel + chain tests, then a same-box A/B against e875423
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_chains.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_j.log 2>&1 || { tail -40 gpurun_out/t_j.log; exit 1; }
tail -2 gpurun_out/t_j.log
B="WDR_AB_LIB=$PWD/tools/_ab/libwdr_e875423.so"
tools/ab_env.sh "" "$B" "" "$B" "WDR_GEMM_CUS=224" 2>&1 | tee gpurun_out/ab_xattn2.txt
