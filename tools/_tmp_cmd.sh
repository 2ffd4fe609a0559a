set -e
for nr in 1 2 4 8; do
timeout -k 10 180 python3 tools/ab_bench.py --no-parity --reps 10 s1:lds=1,opt2=1,nr=$nr s2:lds=1,opt2=2,nr=$nr s4:lds=1,opt2=4,nr=$nr s8:lds=1,opt2=8,nr=$nr > gpurun_out/ab_spl_nr$nr.log 2>&1
echo "nr=$nr $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_spl_nr$nr.log').read().strip().splitlines()[-1]); print({k: round(v['mean_ms'],4) for k,v in d['results'].items()})")"
done
