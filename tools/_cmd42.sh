set -e -o pipefail
timeout -k 10 100 ./tools/dtw_bench
WDR_DTW_WAVE_MAX=4 timeout -k 10 100 ./tools/dtw_bench
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "dtw" 2>&1 | tail -2
