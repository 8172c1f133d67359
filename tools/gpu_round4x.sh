# flash attention at 4 waves/SIMD (WDR_FLASH_OCC=4, 128 VGPRs) vs 3: kernel tests, microbench, A/B
set -e -o pipefail
mkdir -p gpurun_out
WDR_FLASH_OCC=4 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "flash or attention" > gpurun_out/flash_occ4_tests.txt 2>&1
tail -2 gpurun_out/flash_occ4_tests.txt
for o in 3 4 3 4; do
  WDR_FLASH_OCC=$o timeout -k 10 180 ./tools/gemm_bench 6000 > gpurun_out/gb_occ$o.txt 2>&1
  echo "occ $o: $(grep flash gpurun_out/gb_occ$o.txt)"
done
for r in 1 2 3; do bash tools/ab_env.sh "" "WDR_FLASH_OCC=4" "WDR_DECODE_CHAINS=40" "WDR_DECODE_CHAINS=48" "WDR_DECODE_CHAINS=64"; done
