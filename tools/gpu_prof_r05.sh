set -e -o pipefail
LOCK=0 bash tools/round_profile.sh r05 3600
bash tools/pmc_profile.sh r05 600
