# partial-batch wait at 40 chains: 300 (default) / 600 / 1000 us, 3 interleaved rounds
set -e -o pipefail
for r in 1 2 3; do
  bash tools/ab_env.sh "" "WDR_BATCH_WAIT_US=600" "WDR_BATCH_WAIT_US=1000"
done
