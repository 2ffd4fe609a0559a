set -e
timeout -k 10 600 python3 -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
LIBS="prev new" AB_ARGS="--no-parity n1:lds=1 n2:lds=1,nr=2 n8:lds=1,nr=8" bash tools/ab_libs.sh
