# shorter encoder tiles (128 x 128 k_gemm2 / k_gemm3 instead of the 256 x 256 ping-pong: CUs
# free up for the decode chain several times as often)
set -o pipefail
mkdir -p gpurun_out
tools/ab_env.sh "" "WDR_GEMM4=0" "WDR_GEMM4=0 WDR_GEMM3=0" "" "WDR_GEMM4=0" "WDR_GEMM4=0 WDR_GEMM3=0" 2>&1 | tee gpurun_out/ab_short_tiles.txt
