set -e -o pipefail
mkdir -p gpurun_out/im2col
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_whisper.py tests/test_gpu_diarize.py tests/test_gpu_baseline_models.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/im2col/pytest.txt 2>&1
tail -1 gpurun_out/im2col/pytest.txt
bash tools/ab_lines.sh 1 "base:-" "bres:WDR_BATCH_HWQ=2" "bdres:WDR_BATCH_HWQ=2,WDR_DTWQ_HWQ=2"
bash tools/_cmd33b.sh
