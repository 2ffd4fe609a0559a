set -e
timeout -k 10 600 python3 -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 bench.py --compare-no-cull > gpurun_out/bench_n1.log 2>&1 || { tail -20 gpurun_out/bench_n1.log; exit 1; }
tail -n 1 gpurun_out/bench_n1.log
TAG=r01c bash tools/gpu_profile.sh
