set -e
timeout -k 10 600 python3 -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
LIBS="prev new" AB_ARGS="--no-parity cull:lds=1 s2:lds=1,opt2=2 s8:lds=1,opt2=8" bash tools/ab_libs.sh
PTAMD_LIB=ab/new.so timeout -k 10 120 python3 tools/ab_bench.py --scene box_away --no-parity --reps 10 s1:lds=1,opt2=1 s4:lds=1,opt2=4 f4:lds=1,opt2=4,opt3=1 | tail -n 1
