# LayerNorm fused into the row kernel up to 64 rows + k_gemm4 for o / fc2: decoder tests, then
# the A/B against the 32-row threshold
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_whisper.py tests/test_gpu_step.py tests/test_gpu_chains.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_o.log 2>&1 || { tail -40 gpurun_out/t_o.log; exit 1; }
tail -2 gpurun_out/t_o.log
tools/ab_env.sh "" "WDR_ROWS_LN_FUSE=32" "" "WDR_ROWS_LN_FUSE=32" 2>&1 | tee gpurun_out/ab_lnfuse.txt
