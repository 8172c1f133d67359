set -e -o pipefail
mkdir -p gpurun_out/qlog
for v in "vad:--seg vad" "dia:--seg diarize" "dia_noemb:--seg diarize --no-embed"; do
  n=${v%%:*}; a=${v#*:}
  AMD_LOG_LEVEL=3 timeout -k 10 300 python3 bench.py $a --seconds 600 --warmup 0 --steps 1 --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/qlog/$n.json 2> gpurun_out/qlog/$n.raw
  grep -E "Number of allocated hardware queues|Selected queue refCount|acquireQueue|Setting CU mask" gpurun_out/qlog/$n.raw > gpurun_out/qlog/$n.log || true
  rm -f gpurun_out/qlog/$n.raw
  echo "$n $(wc -l < gpurun_out/qlog/$n.log) lines"; grep "Number of allocated" gpurun_out/qlog/$n.log | tail -3
done
