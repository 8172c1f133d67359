#!/bin/bash
# One parameterised GPU-box driver (replaces round 4's one-off gpu_round4*.sh scripts).
# Usage: bash tools/gpu_run.sh STEP [STEP ...]; each step runs under its own time limit, the
# steps are chained (the first failure ends the call), output goes to gpurun_out/<step>.log.
#   gemm        tools/gemm_bench at M = 6000 (f16 encoder tiles, fp8 MX, flash attention)
#   rows        tools/rows_bench (decoder row projections by row count)
#   kernels     pytest tests/test_gpu_kernels.py
#   fp8         pytest tests/test_gpu_fp8.py
#   whisper     pytest test_gpu_whisper / test_gpu_chains / test_gpu_kernels
#   configs     pytest tests/test_gpu_configs.py (C2 / C3 / C4-shard fixtures)
#   suite       the whole -m gpu suite
#   smoke       __graft_entry__.smoke()
#   bench       python bench.py (default line) -> gpurun_out/bench.json
#   benchfast   python bench.py without the beam-5 and CPU-baseline legs -> gpurun_out/bench_fast.json
#   bench8      the same with --fp8 (configs[4] encoder)
#   xattn       tools/xattn_bench (cross-attention partial + combine by row count), then its
#               rocprofv3 kernel stats -> gpurun_out/xattn$T.log, gpurun_out/xprof$T/
#   fp8abl      tools/fp8_ablation.py (fp8 plans on the C3 900-s fixture; FP8_PLANS = its arguments)
#   cosched     tools/cosched_bench at R = $ROWS (default 56): a decode chain beside the encoder
# TAG=name: suffix of the output files (A/B runs of one step under different env knobs) -> gpurun_out/bench_fp8.json
set -e -o pipefail
mkdir -p gpurun_out
export LD_LIBRARY_PATH=$PWD/whisper-diarize-rs_amd:$LD_LIBRARY_PATH
PYT="python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu"
T=${TAG:+_$TAG}
for step in "$@"; do
  echo "== $step $(date +%T)"
  case "$step" in
    gemm) timeout -k 10 120 ./tools/gemm_bench 6000 > gpurun_out/gemm.log 2>&1; cat gpurun_out/gemm.log ;;
    rows) timeout -k 10 120 ./tools/rows_bench > gpurun_out/rows$T.log 2>&1; tail -40 gpurun_out/rows$T.log ;;
    kernels) timeout -k 10 600 $PYT tests/test_gpu_kernels.py > gpurun_out/kernels.log 2>&1 || { tail -40 gpurun_out/kernels.log; exit 1; }; tail -2 gpurun_out/kernels.log ;;
    fp8) timeout -k 10 900 $PYT -s tests/test_gpu_fp8.py > gpurun_out/fp8.log 2>&1 || { tail -40 gpurun_out/fp8.log; exit 1; }; tail -8 gpurun_out/fp8.log ;;
    whisper) timeout -k 10 900 $PYT tests/test_gpu_whisper.py tests/test_gpu_chains.py tests/test_gpu_kernels.py > gpurun_out/whisper.log 2>&1 || { tail -40 gpurun_out/whisper.log; exit 1; }; tail -2 gpurun_out/whisper.log ;;
    configs) timeout -k 10 1100 $PYT -s tests/test_gpu_configs.py > gpurun_out/configs.log 2>&1 || { tail -40 gpurun_out/configs.log; exit 1; }; tail -8 gpurun_out/configs.log ;;
    suite) timeout -k 10 1150 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread --durations 15 > gpurun_out/suite.log 2>&1 || { tail -60 gpurun_out/suite.log; exit 1; }; tail -22 gpurun_out/suite.log ;;
    smoke) timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; tail -1 gpurun_out/smoke.log ;;
    bench) timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; cat gpurun_out/bench.json ;;
    benchfast) timeout -k 10 400 python3 bench.py --beam-seconds 0 --no-cpu-baseline > gpurun_out/bench_fast$T.json 2> gpurun_out/bench_fast$T.err; python3 tools/bench_brief.py gpurun_out/bench_fast$T.json ;;
    bench8) timeout -k 10 400 python3 bench.py --fp8 --beam-seconds 0 --no-cpu-baseline > gpurun_out/bench_fp8$T.json 2> gpurun_out/bench_fp8$T.err; python3 tools/bench_brief.py gpurun_out/bench_fp8$T.json ;;
    xattn) timeout -k 10 120 ./tools/xattn_bench > gpurun_out/xattn$T.log 2>&1; cat gpurun_out/xattn$T.log
      (cd /tmp && export TMPDIR=/tmp; timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/xprof$T -o x -- $GRAFT_REPO_ROOT/tools/xattn_bench > /dev/null 2>&1)
      python3 tools/prof_summary.py gpurun_out/xprof$T --drop-trace > gpurun_out/xprof$T.txt; head -12 gpurun_out/xprof$T.txt ;;
    fp8abl) timeout -k 10 1100 python3 -u tools/fp8_ablation.py $FP8_PLANS > gpurun_out/fp8abl$T.log 2>&1 || { tail -30 gpurun_out/fp8abl$T.log; exit 1; }; cat gpurun_out/fp8abl$T.log ;;
    cosched) timeout -k 10 200 ./tools/cosched_bench ${ROWS:-56} > gpurun_out/cosched$T.log 2>&1; cat gpurun_out/cosched$T.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
