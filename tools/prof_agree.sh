#!/bin/bash
# Live HIP-event kernel timing vs rocprofv3 kernel trace on the same bench command: graphs on
# vs every step eager (WDR_NO_GRAPH=1), with and without the live sampling.  Each step has its
# own time limit; the chain stops at the first failure.
set -e -o pipefail
export TMPDIR=/tmp
S=${1:-120}
O=gpurun_out/agree
rm -rf $O && mkdir -p $O
for mode in graph eager; do
  if [ $mode = eager ]; then export WDR_NO_GRAPH=1; else unset WDR_NO_GRAPH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$mode -o run -- \
    python3 bench.py --seconds $S --steps 1 --warmup 1 --prof none --no-cpu-baseline > $O/tr_$mode.json 2> $O/tr_$mode.err
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trl_$mode -o run -- \
    python3 bench.py --seconds $S --steps 1 --warmup 1 --no-cpu-baseline > $O/trl_$mode.json 2> $O/trl_$mode.err
  timeout -k 10 300 python3 bench.py --seconds $S --steps 1 --warmup 1 --no-cpu-baseline > $O/live_$mode.json 2> $O/live_$mode.err
done
for d in $O/tr_graph $O/trl_graph $O/tr_eager $O/trl_eager; do
  echo "== $d"; python3 tools/prof_summary.py $d | sed -n '/kernel classes/,$p'
done
for m in graph eager; do python3 - <<PY
import json
d = json.load(open("$O/live_$m.json"))
print("live $m", d["value"], {k: (v["avg_launch_us"], v["achieved"]) for k, v in d["roofline_classes"].items()})
PY
done
find $O -name "*kernel_trace.csv" -delete
