# HEAD profiles, second attempt: the unlocked rocprofv3 kernel trace of the benched configuration
# (the locked one is committed), then the WRITE_SIZE pass over a 120-s shard
set -o pipefail
mkdir -p gpurun_out
LOCK=0 bash tools/round_profile.sh r04u 3600 || true
export TMPDIR=/tmp WDR_LAUNCH_LOCK=1
O=gpurun_out/pmc_r04w; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/WRITE_SIZE -o run -- \
  python3 bench.py --seconds 120 --warmup 0 --steps 1 --prof none --no-cpu-baseline --beam-seconds 0 > $O/bench.json 2> $O/err.txt && echo write-pass-ok
