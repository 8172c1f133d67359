#!/bin/bash
# Which factor makes rocprofv3 --kernel-trace fault on the pipeline: hipGraph replays or
# concurrent launches from the decode-chain threads.  Four 120-s bench runs under the tracer,
# each under its own time limit; every run's exit status is recorded (a fault does not stop the
# script: the faulting process has exited and the next run starts clean).
export TMPDIR=/tmp
O=gpurun_out/crash_ab
rm -rf $O && mkdir -p $O
for cfg in "WDR_NO_GRAPH=1 WDR_LAUNCH_LOCK=1" "WDR_NO_GRAPH=1" "WDR_LAUNCH_LOCK=1" ""; do
  tag=$(echo "${cfg:-default}" | tr ' =' '__')
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o run -- \
    python3 bench.py --seconds 120 --warmup 1 --steps 1 --prof none --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err
  rc=$?
  echo "${cfg:-default (graphs, concurrent launches)}: exit $rc" | tee -a $O/summary.txt
  find $O/$tag -name "*kernel_trace.csv" -delete 2>/dev/null
  if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then break; fi
done
