#!/bin/bash
# PMC passes of the BENCHED configuration (the default bench command: 1 h of audio, hipGraph
# replays on), one counter per rocprofv3 run (FETCH_SIZE and WRITE_SIZE cannot share a pass),
# folded per kernel class into pmc.json (FETCH_SIZE doubled: the gfx950 correction,
# MI355X_MICROARCH.md 'HBM'), which bench.py reads for roofline.traffic.  Launch calls are
# serialised (WDR_LAUNCH_LOCK=1): rocprofv3's queue interception faults on concurrent submissions
# (profiles/r03/rocprof_unlocked_fault.txt).  Every GPU step has its own limit.
#   tools/pmc_profile.sh TAG [SECONDS]   (default a 600-s shard: counter collection serialises
#   every dispatch, ~10x slower than the run itself; the per-dispatch figures are the same launch
#   mix -- encode-ahead batches, batched rows steps with prefills and DTW re-forwards)
set -e -o pipefail
TAG=${1:-r03}
SECS=${2:-600}
export TMPDIR=/tmp WDR_LAUNCH_LOCK=1
O=gpurun_out/pmc_$TAG
rm -rf $O && mkdir -p $O
# counter collection serialises every dispatch: a heartbeat keeps the run visibly alive
( while true; do date >> $O/heartbeat; sleep 50; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 900 rocprofv3 --pmc $c --output-format csv -d $O/$c -o run -- \
    python3 bench.py --seconds $SECS --warmup 0 --steps 1 --prof none --no-cpu-baseline --beam-seconds 0 > $O/bench_$c.json 2> $O/$c.err
done
python3 tools/prof_summary.py $O/FETCH_SIZE --fetch $O/FETCH_SIZE --write $O/WRITE_SIZE --json $O/pmc.json > $O/pmc_summary.txt
find $O -name "*counter_collection.csv" -delete
tail -12 $O/pmc_summary.txt
