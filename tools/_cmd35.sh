set -e -o pipefail
mkdir -p gpurun_out/ab
WDR_EMBED_LOG=1 timeout -k 10 300 python3 bench.py --seg diarize --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/ab/elog_dia.json 2> gpurun_out/ab/elog_dia.err
grep "wdr-embed" gpurun_out/ab/elog_dia.err | tail -30
LINES=vad bash tools/ab_lines.sh 1 "ve2:WDR_VAD_EMBED=2" "ve1:WDR_VAD_EMBED=1"
