# unbiased live sampling (only graph-replayable work draws eager sampled runs): chain / whisper
# suites, the default bench line (live profiler on), then two profiler-off runs for its cost
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_chains.py tests/test_gpu_whisper.py > gpurun_out/t_prof.log 2>&1
tail -1 gpurun_out/t_prof.log
timeout -k 10 600 python3 bench.py > gpurun_out/bench_head2.json 2> gpurun_out/bench_head2.err
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench_head2.json"))
print("value", d["value"], "beam5", (d.get("beam5") or {}).get("value"))
for k, v in d["roofline_classes"].items():
    print(k, v["avg_launch_us"], v["achieved"], v["frac"], v["launches_est"])
print("trace", json.dumps(d["roofline_trace"]))
PY
bash tools/ab_env.sh "" ""
