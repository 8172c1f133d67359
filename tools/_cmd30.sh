set -e -o pipefail
LINES=vad bash tools/ab_lines.sh 2 "ou4:-" "ou0:WDR_OWN_UNDIAR=0" "ou4nolq:WDR_LOWQ_AT_PIPE=0"
LINES=diarize bash tools/ab_lines.sh 2 "base:-"
