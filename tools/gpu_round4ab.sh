# the HEAD trace (40 decode chains) for profiles/r04/prof_graph (unlocked; the locked form if the tool faults)
set -o pipefail
mkdir -p gpurun_out
LOCK=0 bash tools/round_profile.sh r04i 3600 || LOCK=1 bash tools/round_profile.sh r04i 3600
