set -e -o pipefail
LINES=vad bash tools/ab_lines.sh 1 "sl1:WDR_START_LOAD=1" "sl3:WDR_START_LOAD=3" "sl10:WDR_START_LOAD=10" "sl10b256:WDR_START_LOAD=10,WDR_START_BLOCKS=256"
LINES=diarize bash tools/ab_lines.sh 1 "base:-" "sl30d:WDR_START_LOAD=30,WDR_START_LOAD_DIA=1"
