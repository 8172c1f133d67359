# HEAD profile for round 6: the locked kernel trace of the benched command (DESIGN.md "Faults"),
# then the PMC traffic passes.
set -e -o pipefail
LOCK=1 bash tools/round_profile.sh r06 3600
bash tools/pmc_profile.sh r06 600
