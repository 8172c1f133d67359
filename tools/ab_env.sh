#!/bin/bash
# A/B of environment knobs on the default bench (1 h of audio, 1 GPU): one bench run per
# variant, each under its own time limit; the chain stops at the first failure.
#   tools/ab_env.sh "A=1 B=2" "C=3" ...      (an empty string = the default)
#   AB_ARGS="--fp8" tools/ab_env.sh ...       (extra bench.py arguments for every variant)
set -e -o pipefail
mkdir -p gpurun_out/ab
i=0
for v in "$@"; do
  i=$((i + 1))
  env $v timeout -k 10 240 python3 bench.py --no-cpu-baseline --prof none --beam-seconds 0 ${AB_ARGS:-} > gpurun_out/ab/run$i.json 2> gpurun_out/ab/run$i.err
  python3 - "$v" gpurun_out/ab/run$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
s = d["stages_s"]
print("%-40s xRT %7.1f  wall %6.3f s  batch_step %6.3f s  launches %d" % (
    sys.argv[1] or "(default)", d["value"], d["ms_per_step"] / 1e3, s.get("batch_step_s", 0),
    d["counts"].get("batch_launches", 0)), flush=True)
PY
done
