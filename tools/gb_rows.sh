set -e -o pipefail
mkdir -p gpurun_out
O=gpurun_out/gb.txt; : > $O
for M in 8 16; do
  WDR_MGEMV_STAGED=0 timeout -k 10 60 ./tools/gemv_bench >> /dev/null 2>&1 || true
  echo "== M=$M unstaged" >> $O; GB_ROWS=$M WDR_MGEMV_STAGED=0 timeout -k 10 60 ./tools/gemv_bench >> $O 2>&1
  for R in 1 2 4; do echo "== M=$M staged R=$R" >> $O; GB_ROWS=$M WDR_MGEMV_R=$R timeout -k 10 60 ./tools/gemv_bench >> $O 2>&1; done
done
cat $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_chains.py -x -q --timeout 300 --timeout-method thread > gpurun_out/chains_t.log 2>&1; echo "chains rc=$?"; tail -5 gpurun_out/chains_t.log
