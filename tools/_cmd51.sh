set -o pipefail
timeout -k 10 700 python -u -m pytest tests/test_gpu_multidevice.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t_md.log 2>&1 || { tail -40 gpurun_out/t_md.log; exit 1; }
tail -2 gpurun_out/t_md.log
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log
