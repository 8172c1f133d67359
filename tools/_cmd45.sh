set -e -o pipefail
cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cpu.max"
grep -E "throttled" /sys/fs/cgroup/cpu.stat 2>/dev/null || echo "no throttle stats"
timeout -k 10 300 python3 bench.py --seg diarize --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/cg.json 2> gpurun_out/cg.err
grep -E "throttled" /sys/fs/cgroup/cpu.stat 2>/dev/null || true
python3 -c "import json;d=json.load(open('gpurun_out/cg.json'));print(d['value'],d['host_cpu'])"
