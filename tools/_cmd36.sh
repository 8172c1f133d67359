set -e -o pipefail
mkdir -p gpurun_out/blog
for v in base sl30; do
  e=""; [ $v = sl30 ] && e="WDR_START_LOAD=30"
  env $e WDR_BATCH_LOG=gpurun_out/blog/$v.batch WDR_CHAIN_LOG=gpurun_out/blog/$v.chain timeout -k 10 300 python3 bench.py --seg vad --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/blog/$v.json 2> gpurun_out/blog/$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/blog/$v.json'));print('$v',d['value'],d['stages_s'].get('batch_step_s'))"
done
