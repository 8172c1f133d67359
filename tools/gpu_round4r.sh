# remaining scheduling knobs at the final kernels: decode chains 28 / 32, encoder GEMM persistent
# grid 192 / 160 workgroups (more CUs left to the decode chain while a GEMM runs)
set -o pipefail
mkdir -p gpurun_out
tools/ab_env.sh "" "WDR_DECODE_CHAINS=32" "WDR_GEMM_CUS=192" "WDR_GEMM_CUS=160" "" "WDR_DECODE_CHAINS=32" "WDR_GEMM_CUS=192" "WDR_DECODE_CHAINS=28" 2>&1 | tee gpurun_out/ab_final_knobs.txt
