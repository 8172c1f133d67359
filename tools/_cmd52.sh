set -e -o pipefail
mkdir -p gpurun_out/sync
for v in "base:-" "blas1:OPENBLAS_NUM_THREADS=1,OMP_NUM_THREADS=1,MKL_NUM_THREADS=1"; do
  n=${v%%:*}; e=${v#*:}; [ "$e" = "-" ] && e=""
  env $(echo "$e" | tr ',' ' ') WDR_BENCH_THREADS=1 timeout -k 10 300 python3 bench.py --seg diarize --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/sync/$n.json 2> gpurun_out/sync/$n.err
  python3 -c "import json;d=json.load(open('gpurun_out/sync/$n.json'));h=d['host_cpu'];print('$n',d['value'],d['stages_s'].get('batch_step_s'),h)"
done
