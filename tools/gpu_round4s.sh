# diarization GEMM seam test, then shorter encoder tiles (128 x 128 k_gemm2 / k_gemm3 instead of
# the 256 x 256 ping-pong: CUs free up for the decode chain several times as often)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_diarize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_s.log 2>&1 || { tail -30 gpurun_out/t_s.log; exit 1; }
tail -1 gpurun_out/t_s.log
tools/ab_env.sh "" "WDR_GEMM4=0" "WDR_GEMM4=0 WDR_GEMM3=0" "" "WDR_GEMM4=0" "WDR_GEMM4=0 WDR_GEMM3=0" 2>&1 | tee gpurun_out/ab_short_tiles.txt
