set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread --durations 10 --ignore tests/test_gpu_configs.py --ignore tests/test_gpu_multidevice.py > gpurun_out/t_a.log 2>&1 || { tail -60 gpurun_out/t_a.log; exit 1; }
tail -14 gpurun_out/t_a.log
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log
