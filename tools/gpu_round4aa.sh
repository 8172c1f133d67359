# scheduling knobs re-checked at the 40-chain default: partial-batch wait, chain count, encoder CU mask
set -e -o pipefail
for r in 1 2 3; do
  bash tools/ab_env.sh "" "WDR_BATCH_WAIT_US=150" "WDR_BATCH_WAIT_US=600" "WDR_DECODE_CHAINS=36" "WDR_ENC_MASK=16"
done
