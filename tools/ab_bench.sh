# A/B of background-stream CU reservation on the default bench (1 h large-v3 + DTW + diarize).
# usage: ab_bench.sh "name:ENV=V,ENV2=V2" ...   (each variant is one bench run; stops at the first failure)
set -e -o pipefail
mkdir -p gpurun_out/ab
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python bench.py --no-cpu-baseline --prof none > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err
  python -c "import json;d=json.load(open('gpurun_out/ab/$name.json'));s=d['stages_s'];print('$name',d['value'],d['ms_per_step'],s.get('batch_step_s'),d['counts']['batch_launches'],s['encode'])" | tee -a gpurun_out/ab/summary.txt
done
