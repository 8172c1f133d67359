set -e -o pipefail
for v in "" "WDR_ODM_ALT=0" "WDR_ODM_POOL=-1 WDR_ODM_ALT=0" ""; do
  env $v timeout -k 10 300 python3 -u tools/vad_segments_bench.py 2> /dev/null | tee -a gpurun_out/vad_segments_bench.jsonl
done
