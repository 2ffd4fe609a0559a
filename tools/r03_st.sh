set -u
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "wide or wavefront or config" --timeout 200 --timeout-method thread > gpurun_out/st_parity.log 2>&1 || { echo "parity rc=$?"; tail -30 gpurun_out/st_parity.log; exit 1; }
tail -1 gpurun_out/st_parity.log
LIBS="base st" AB_SCENES="sphere:6 random:10000000" AB_ITERS=2 timeout -k 10 500 tools/ab_libs_scenes.sh || exit 1
timeout -k 10 900 tools/ta_counters.sh
