set -e
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for i in 1 2 3; do
timeout -k 10 120 python3 tools/ab_bench.py --reps 10 cull:lds=1 nocull:lds=1,opt6=0 d0cull:lds=1,depth=0 s1:lds=1,opt2=1 s4:lds=1,opt2=4 > gpurun_out/ab_cull.$i.log 2>&1
python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_cull.$i.log')); print({k: round(v['mean_ms'],4) for k,v in d['results'].items()})"
done
