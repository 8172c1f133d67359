# HEAD profile for round 5: the locked kernel trace (LOCK=0 faults inside rocprofiler-sdk's
# dispatch interception, see DESIGN.md "Faults"), then the PMC traffic passes.
set -e -o pipefail
LOCK=1 bash tools/round_profile.sh r05 3600
bash tools/pmc_profile.sh r05 600
