timeout -k 10 300 python3 -u tools/dtw_w02_diag.py 1 13 24 25 42 > gpurun_out/dtw_w02_diag.log 2>&1 || { tail -20 gpurun_out/dtw_w02_diag.log; exit 1; }
cat gpurun_out/dtw_w02_diag.log
bash tools/ab_lines.sh 1 "odm4:-" "odm0:WDR_ODM_POOL=-1" "odm2:WDR_ODM_POOL=2" "odm8:WDR_ODM_POOL=8" "oprio2:WDR_OWN_PRIO=2"
