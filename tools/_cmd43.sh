set -o pipefail
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread --ignore tests/test_gpu_configs.py --ignore tests/test_gpu_multidevice.py > gpurun_out/t_a2.log 2>&1 || { tail -40 gpurun_out/t_a2.log; exit 1; }
tail -2 gpurun_out/t_a2.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q -s --timeout 400 --timeout-method thread -k "c3_large_v3 or c2_base or c4_diarized" > gpurun_out/t_c.log 2>&1 || { tail -40 gpurun_out/t_c.log; exit 1; }
tail -3 gpurun_out/t_c.log
LINES=diarize bash tools/ab_lines.sh 1 "dtwnew:-" "dtwold:WDR_DTW_DP_OLD=1"
