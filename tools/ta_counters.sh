export GROUPS_LIST="TA_TA_BUSY_sum GRBM_GUI_ACTIVE TD_TD_BUSY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum
TCC_HIT_sum TCC_MISS_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum"
TAG=ta_sphere AB_ARGS="--scene sphere:6 v:" timeout -k 10 400 tools/wf_counters.sh > gpurun_out/ta_sphere.txt 2>&1 || { tail -5 gpurun_out/ta_sphere.txt; exit 1; }
TAG=ta_cloud AB_ARGS="--scene random:10000000 v:" timeout -k 10 500 tools/wf_counters.sh > gpurun_out/ta_cloud.txt 2>&1 || { tail -5 gpurun_out/ta_cloud.txt; exit 1; }
grep wf_trace gpurun_out/ta_sphere.txt gpurun_out/ta_cloud.txt
