# the round-end GPU checks: the whole -m gpu suite, then smoke(); each under its own limit
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread --durations 15 > gpurun_out/t_full.log 2>&1 || { tail -60 gpurun_out/t_full.log; exit 1; }
tail -22 gpurun_out/t_full.log
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log
