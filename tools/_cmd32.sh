set -e -o pipefail
mkdir -p gpurun_out/im2col
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_diarize.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/im2col/pytest.txt 2>&1
tail -2 gpurun_out/im2col/pytest.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/im2col/prof -o run -- python3 bench.py --seconds 600 --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/im2col/bench600.json 2> gpurun_out/im2col/bench600.err
find gpurun_out/im2col/prof -name "*kernel_stats.csv" | head -1 | xargs grep -i "im2col" || true
LINES=diarize bash tools/ab_lines.sh 1 "im2col:-"
