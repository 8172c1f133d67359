# HEAD profiles for profiles/r04: the rocprofv3 kernel trace of the benched configuration (launch
# calls serialised: the unlocked trace faults inside librocprofiler-sdk, gpurun_out/prof_r04 of
# the previous call) and the FETCH_SIZE / WRITE_SIZE passes
set -o pipefail
mkdir -p gpurun_out
LOCK=1 bash tools/round_profile.sh r04 3600 || exit 1
bash tools/pmc_profile.sh r04 600
