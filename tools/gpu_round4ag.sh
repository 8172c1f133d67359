# the live profiler's cost: on (decode steps 1 in 32 eager) / on with 1 in 64 eager / off, 2 rounds
set -e -o pipefail
mkdir -p gpurun_out/abp
for r in 1 2; do
  for v in "" "WDR_PROF_STEP_EVERY=64" "NONE"; do
    if [ "$v" = NONE ]; then a="--prof none"; e=""; else a=""; e="$v"; fi
    env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --beam-seconds 0 $a > gpurun_out/abp/run.json 2> gpurun_out/abp/run.err
    python3 -c "import json,sys; d=json.load(open('gpurun_out/abp/run.json')); c=d.get('roofline') or {}; print('%-28s xRT %7.1f  launches %d  gemm frac %s' % (sys.argv[1] or '(profiler on)', d['value'], d['counts']['batch_launches'], c.get('frac')), flush=True)" "$v"
  done
done
