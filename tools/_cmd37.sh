set -e -o pipefail
mkdir -p gpurun_out/clk
timeout 20 rocm-smi --showclocks > gpurun_out/clk/idle.txt 2>&1 || true
cat gpurun_out/clk/idle.txt | tail -15
for v in base sl30 base2; do
  e=""; [ $v = sl30 ] && e="WDR_START_LOAD=30"
  ( while true; do echo "T $(date +%s.%N)"; timeout 5 rocm-smi --showclocks --showpower 2>/dev/null | grep -E "sclk|mclk|fclk|socclk|Power|level" || true; sleep 0.05; done ) > gpurun_out/clk/$v.smi 2>&1 &
  SP=$!
  env $e timeout -k 10 300 python3 bench.py --seg vad --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/clk/$v.json 2> gpurun_out/clk/$v.err || { kill $SP; exit 1; }
  kill $SP || true
  python3 -c "import json;d=json.load(open('gpurun_out/clk/$v.json'));print('$v',d['value'],d['stages_s'].get('batch_step_s'))"
done
