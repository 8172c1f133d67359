# prompt prefills on a batcher of their own beside the decode steps: decoder tests, then the A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_chains.py tests/test_gpu_whisper.py tests/test_gpu_step.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_q.log 2>&1 || { tail -40 gpurun_out/t_q.log; exit 1; }
tail -2 gpurun_out/t_q.log
tools/ab_env.sh "" "WDR_PREFILL_SPLIT=0" "" "WDR_PREFILL_SPLIT=0" 2>&1 | tee gpurun_out/ab_psplit.txt
WDR_BATCH_LOG=gpurun_out/blog_r4c.txt timeout -k 10 240 python3 bench.py --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/bench_blog3.json 2> gpurun_out/bench_blog3.err && python3 tools/batch_log.py gpurun_out/blog_r4c.txt | head -8
