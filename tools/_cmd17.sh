set -o pipefail
bash tools/_cmd16.sh || exit 1
PYT="python3 -u -m pytest -x -v --timeout 1100 --timeout-method thread -m gpu"
timeout -k 10 1000 $PYT -s tests/test_gpu_configs.py -k "w02 or beam5_dtw_300s or c2_one_hour" > gpurun_out/t17.log 2>&1 || { tail -40 gpurun_out/t17.log; exit 1; }
grep -E "c4_diarized|near_tie|c3_beam|c2_vad|passed|failed" gpurun_out/t17.log | tail -20
