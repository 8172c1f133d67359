set -o pipefail
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread --durations 10 --ignore=tests/test_gpu_configs.py --ignore=tests/test_gpu_multidevice.py > gpurun_out/suite_a.log 2>&1 || { tail -60 gpurun_out/suite_a.log; exit 1; }
tail -15 gpurun_out/suite_a.log
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log

LINES=vad bash tools/ab_lines.sh 1 "m64:WDR_ENC_MASK_PAT=0,WDR_ENC_MASK=64" "m96:WDR_ENC_MASK_PAT=0,WDR_ENC_MASK=96" "enc1:WDR_ENC_POOL=1" "ahead3:WDR_ENC_AHEAD=4" "base:-"
