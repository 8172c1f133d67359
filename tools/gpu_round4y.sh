# decode chains beyond 40 with fewer ring slots per chain (16 slots x 245 MB of cross-K/V per chain
# put 48 chains out of memory): 3 interleaved rounds
set -e -o pipefail
for r in 1 2 3; do
  bash tools/ab_env.sh "" "WDR_DECODE_CHAINS=40" "WDR_DECODE_CHAINS=40 WDR_SLOTS=8" "WDR_DECODE_CHAINS=48 WDR_SLOTS=8" "WDR_DECODE_CHAINS=64 WDR_SLOTS=8"
done
