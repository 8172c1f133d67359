# encoder placement A/B: CU mask (32 default / 16 / 0) and 8-window encode batches (M = 12000)
set -o pipefail
mkdir -p gpurun_out
tools/ab_env.sh "" "WDR_ENC_MASK=16" "WDR_ENC_MASK=0" "WDR_ENC_BATCH=8" "WDR_ENC_BATCH=8 WDR_ENC_MASK=0" "" "WDR_ENC_MASK=16" "WDR_ENC_MASK=0" "WDR_ENC_BATCH=8" 2>&1 | tee gpurun_out/ab_enc4.txt
