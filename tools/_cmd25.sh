set -e -o pipefail
LINES=vad bash tools/ab_lines.sh 1 "m64:WDR_ENC_MASK_PAT=0,WDR_ENC_MASK=64" "m96:WDR_ENC_MASK_PAT=0,WDR_ENC_MASK=96" "enc1:WDR_ENC_POOL=1" "ahead3:WDR_ENC_AHEAD=4" "base:-"
