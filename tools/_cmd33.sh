set -e -o pipefail
mkdir -p gpurun_out/im2col
export TMPDIR=/tmp
L=whisper-diarize-rs_amd/libwdr.so
trap 'cp tools/_ab/libwdr_new.so $L' EXIT
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_whisper.py tests/test_gpu_diarize.py tests/test_gpu_baseline_models.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/im2col/pytest.txt 2>&1
tail -1 gpurun_out/im2col/pytest.txt
for lib in r06 new; do
  cp tools/_ab/libwdr_$lib.so $L
  WDR_LAUNCH_LOCK=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/im2col/p_$lib -o run -- python3 bench.py --seconds 600 --no-cpu-baseline --prof none --beam-seconds 0 > gpurun_out/im2col/b_$lib.json 2> gpurun_out/im2col/b_$lib.err
  f=$(find gpurun_out/im2col/p_$lib -name "*kernel_stats.csv" | head -1)
  echo "== $lib"; grep -i "im2col" $f || true
done
