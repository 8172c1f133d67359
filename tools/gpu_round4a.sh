# round-4 check on the GPU box: kernel / model / step / chain parity tests, the co-scheduling
# probe, then an A/B of the encoder stream mask on the bench (each step under its own limit)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_whisper.py tests/test_gpu_step.py tests/test_gpu_chains.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_a.log 2>&1 || { tail -40 gpurun_out/t_a.log; exit 1; }
tail -3 gpurun_out/t_a.log
timeout -k 10 120 ./tools/cosched_bench 16 > gpurun_out/cosched2.txt 2>&1 && cat gpurun_out/cosched2.txt
tools/ab_env.sh "" "WDR_ENC_MASK=0" 2>&1 | tee gpurun_out/ab_v2.txt
