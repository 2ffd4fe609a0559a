set -u
mkdir -p gpurun_out
for n in 64 80; do
  timeout -k 10 200 python -u bench.py --scene sphere --steps 2 --warmup 1 --no-cpu-baseline --opt 16=$n > gpurun_out/cnt_$n.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/cnt_$n.log; exit 1; }
  grep '^{' gpurun_out/cnt_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['ms_per_step'], d['config'].get('traced'))"
done
