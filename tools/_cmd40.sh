set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_multidevice.py -m gpu -x -q -s --timeout 600 --timeout-method thread --durations 10 > gpurun_out/t_b.log 2>&1 || { tail -60 gpurun_out/t_b.log; exit 1; }
tail -14 gpurun_out/t_b.log
