set -e -o pipefail
LINES=vad bash tools/ab_lines.sh 1 "spin1:WDR_HOST_SPIN=1" "spin4:WDR_HOST_SPIN=4"
timeout -k 10 600 python3 bench.py > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err
python3 tools/bench_brief.py gpurun_out/bench_head.json
