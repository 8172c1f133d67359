# decode-chain count A/B with partial batches (3 interleaved rounds)
set -e -o pipefail
for r in 1 2 3; do
  bash tools/ab_env.sh "" "WDR_DECODE_CHAINS=32" "WDR_DECODE_CHAINS=40"
done
