set -e -o pipefail
mkdir -p gpurun_out/ab
WDR_STREAM_LOG=1 timeout -k 10 300 python3 bench.py --seg vad --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/ab/slog.json 2> gpurun_out/ab/slog.err
grep -c "state-own->pool" gpurun_out/ab/slog.err || true
grep "state-own->" gpurun_out/ab/slog.err | sort | uniq -c | sort -rn | head -12
LINES=vad bash tools/ab_lines.sh 1 "own4:WDR_OWN_POOL=4" "ou4:-"
