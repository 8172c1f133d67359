#!/bin/bash
# Round profile on the GPU box: kernel trace + stats of the bench command, separate PMC passes
# for FETCH_SIZE / WRITE_SIZE, then the default (1 h) bench line.  Every GPU step has its own
# time limit and the chain stops at the first failure.
set -e -o pipefail
TAG=${1:-r01}
SECS=${2:-300}
export TMPDIR=/tmp
# rocprofv3's kernel tracing faults on concurrent kernel launches from several host threads
# (the decode chains): serialise the launch calls while profiling (csrc/prof.h)
# and on hipGraph replays: decode steps run their kernels eagerly under the profiler
export WDR_LAUNCH_LOCK=1 WDR_NO_GRAPH=1
mkdir -p gpurun_out
O=gpurun_out/prof_$TAG
rm -rf $O && mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --seconds $SECS --warmup 0 --prof gemv --no-cpu-baseline > $O/bench_trace.json 2> $O/trace.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- \
  python3 bench.py --seconds 30 --warmup 0 --prof gemv --no-cpu-baseline > $O/bench_fetch.json 2> $O/fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- \
  python3 bench.py --seconds 30 --warmup 0 --prof gemv --no-cpu-baseline > $O/bench_write.json 2> $O/write.err
python3 tools/kstat_groups.py $(find $O/trace -name "*kernel_stats.csv" | head -1) > $O/stages.txt
python3 tools/busy.py $(find $O/trace -name "*kernel_trace.csv" | head -1) 0.1 >> $O/stages.txt
python3 tools/prof_summary.py $O/trace --fetch $O/fetch --write $O/write --drop-trace --json $O/pmc.json > $O/summary.txt
rm -f $O/fetch/*/*counter_collection.csv.big 2>/dev/null || true
unset WDR_LAUNCH_LOCK WDR_NO_GRAPH
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
cat $O/summary.txt | head -60
cat $O/bench_default.json
