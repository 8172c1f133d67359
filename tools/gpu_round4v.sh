# the HEAD trace for profiles/r04 (unlocked; the locked form if the tool faults again)
set -o pipefail
mkdir -p gpurun_out
LOCK=0 bash tools/round_profile.sh r04h 3600 || LOCK=1 bash tools/round_profile.sh r04h 3600
