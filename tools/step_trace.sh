#!/bin/bash
# Step timeline of the benched configuration: rocprofv3 kernel trace of bench.py on a shorter
# shard (SECS, default 900 s: a smaller trace) with host launch calls serialised
# (WDR_LAUNCH_LOCK=1: rocprofv3's launch interception faults under concurrent launching threads,
# DESIGN.md §7), then tools/step_gaps.py on the trace; the trace CSV itself is deleted.
#   tools/step_trace.sh TAG [SECS]
set -e -o pipefail
TAG=${1:-steps}
SECS=${2:-900}
export TMPDIR=/tmp WDR_LAUNCH_LOCK=${LOCK:-1}
O=gpurun_out/trace_$TAG
rm -rf $O && mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- \
  python3 bench.py --seconds $SECS --warmup 1 --steps 1 --no-cpu-baseline --prof none > $O/bench.json 2> $O/trace.err
T=$(find $O/trace -name "*kernel_trace.csv" | head -1)
timeout -k 10 300 python3 tools/step_gaps.py $T > $O/step_gaps.txt
rm -f $T
cat $O/step_gaps.txt
