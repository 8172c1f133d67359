# the encoder on 240 CUs (mask 16: o / fc2 in one round on k_gemm5) against the default 224 CUs
set -o pipefail
mkdir -p gpurun_out
tools/ab_env.sh "" "WDR_ENC_MASK=16 WDR_GEMM5=1" "WDR_ENC_MASK=16" "" "WDR_ENC_MASK=16 WDR_GEMM5=1" "WDR_ENC_MASK=16" 2>&1 | tee gpurun_out/ab_mask16.txt
