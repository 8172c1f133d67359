# A/B of decode-step GEMV variants on the default bench (1 h large-v3 + DTW + diarize)
set -e -o pipefail
mkdir -p gpurun_out/ab
WDR_MGEMV_STAGED=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab/old.json 2> gpurun_out/ab/old.err
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab/new.json 2> gpurun_out/ab/new.err
WDR_STEP_LN_SPLIT=2 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab/lns2.json 2> gpurun_out/ab/lns2.err
for f in old new lns2; do python -c "import json;d=json.load(open('gpurun_out/ab/$f.json'));print('$f',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'] if d.get('roofline') else None, d['counts']['batch_launches'])"; done
