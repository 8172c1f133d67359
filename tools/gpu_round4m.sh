# front-loading the encoder: encode-ahead depth (WDR_ENC_AHEAD 8 default / 16) and encode stream
# priority (WDR_ENC_PRIO 0 lowest default / 2 highest)
set -o pipefail
mkdir -p gpurun_out
tools/ab_env.sh "" "WDR_ENC_AHEAD=16" "WDR_ENC_PRIO=2" "WDR_ENC_AHEAD=16 WDR_ENC_PRIO=2" "" "WDR_ENC_AHEAD=16" "WDR_ENC_PRIO=2" "WDR_ENC_AHEAD=16 WDR_ENC_PRIO=2" 2>&1 | tee gpurun_out/ab_front.txt
