#!/bin/bash
# Round profile of the BENCHED configuration on the GPU box: rocprofv3 kernel trace + stats of
# the default bench command (1 h of audio, hipGraph replays on, the GPU streams of all decode
# chains concurrent), then the stage grouping.  WDR_LAUNCH_LOCK=1 serialises only the host-side
# launch CALLS of the chain threads: rocprofv3's kernel-trace interception of hipLaunchKernel
# faults (SIGSEGV inside the tool) when several threads launch eagerly at once
# (tools/prof_crash_ab.sh: eager + unlocked faults, every locked or graph-replayed run is clean).
# Every GPU step has its own time limit and the chain stops at the first failure.
#   tools/round_profile.sh TAG [SECONDS]
set -e -o pipefail
TAG=${1:-r02}
SECS=${2:-3600}
export TMPDIR=/tmp
# LOCK=0: unlocked launches (the configuration bench.py measures); WDR_SEGV_TRACE: a fault
# prints its address and a backtrace with library offsets (csrc/prof.cpp)
export WDR_LAUNCH_LOCK=${LOCK:-1}
export WDR_SEGV_TRACE=1
mkdir -p gpurun_out
O=gpurun_out/prof_$TAG
rm -rf $O && mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --seconds $SECS --warmup 1 --steps 1 --no-cpu-baseline --prof none --beam-seconds 0 > $O/bench_trace.json 2> $O/trace.err
python3 tools/kstat_groups.py $(find $O/trace -name "*kernel_stats.csv" | head -1) > $O/stages.txt
python3 tools/busy.py $(find $O/trace -name "*kernel_trace.csv" | head -1) 0.1 >> $O/stages.txt
python3 tools/prof_summary.py $O/trace --json $O/classes.json --drop-trace > $O/summary.txt
head -40 $O/summary.txt
