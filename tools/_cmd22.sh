set -e -o pipefail
bash tools/ab_lines.sh 1 "dtwq0:WDR_DTW_QUEUE=0" "lap:WDR_LOWQ_AT_PIPE=1"
LINES=diarize bash tools/ab_lines.sh 2 "lnf512:WDR_ROWS_LN_FUSE=512" "base:-"
