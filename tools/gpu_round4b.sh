# rows_bench (k_rowproj per shape and row count) + same-box A/B: HEAD vs the previous rows
# engine build (tools/_ab, gitignored) vs HEAD with unmasked encode-ahead streams
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/rows_bench > gpurun_out/rows_bench_v2.txt 2>&1 && cat gpurun_out/rows_bench_v2.txt
OLD="WDR_AB_LIB=$PWD/tools/_ab/libwdr_48c4668.so"
tools/ab_env.sh "" "$OLD" "WDR_ENC_MASK=0" "" "$OLD" "WDR_ENC_MASK=0" 2>&1 | tee gpurun_out/ab_v2b.txt
