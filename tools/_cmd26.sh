set -o pipefail
timeout -k 10 1150 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_multidevice.py -m gpu -x -q --timeout 900 --timeout-method thread --durations 12 -s > gpurun_out/suite_b.log 2>&1 || { tail -60 gpurun_out/suite_b.log; exit 1; }
grep -E "passed|failed|c4_diarized|near_tie|c3_|c2_|c4_shard" gpurun_out/suite_b.log | tail -30
