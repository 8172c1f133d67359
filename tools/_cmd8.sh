set -o pipefail
PYT="python3 -u -m pytest -x -v --timeout 1100 --timeout-method thread -m gpu"
timeout -k 10 600 $PYT tests/test_gpu_diarize.py tests/test_vad.py tests/test_gpu_fp8.py -k "not pipeline_agreement" > gpurun_out/t8a.log 2>&1 || { tail -30 gpurun_out/t8a.log; exit 1; }
tail -3 gpurun_out/t8a.log
timeout -k 10 1000 $PYT -s tests/test_gpu_configs.py -k "c4_diarized or beam5_dtw_120s" > gpurun_out/t8b.log 2>&1 || { tail -40 gpurun_out/t8b.log; exit 1; }
grep -E "c4_diarized|near_tie|c3_beam|passed|failed" gpurun_out/t8b.log | tail -20
