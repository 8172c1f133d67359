#!/bin/bash
# Locked rocprofv3 kernel traces of short bench runs (600 s), one per "name:line:ENV=V,..." spec,
# analysed by tools/queue_map.py (which kernels share the step batcher's hardware queue).
#   tools/queue_trace.sh "def_vad:vad:-" "own4_vad:vad:WDR_OWN_POOL=4" ...
set -e -o pipefail
export TMPDIR=/tmp WDR_LAUNCH_LOCK=1
mkdir -p gpurun_out/qtrace
for v in "$@"; do
  name=${v%%:*}; rest=${v#*:}; seg=${rest%%:*}; envs=${rest#*:}; [ "$envs" = "-" ] && envs=""
  O=gpurun_out/qtrace/$name
  rm -rf $O && mkdir -p $O
  env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- \
    python3 bench.py --seg $seg --seconds 600 --warmup 0 --steps 1 --no-cpu-baseline --prof none --beam-seconds 0 > $O/bench.json 2> $O/trace.err
  python3 tools/queue_map.py $(find $O/trace -name "*kernel_trace.csv" | head -1) "$name $(python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['stages_s'].get('batch_step_s'))")" $(find $O/trace -name "*memory_copy_trace.csv" | head -1) > gpurun_out/qtrace/$name.txt
  find $O/trace -name "*_trace.csv" -delete
  head -30 gpurun_out/qtrace/$name.txt
done
