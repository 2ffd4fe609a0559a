set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rounds
for S in sphere:6 random:10000000; do
  n=${S%%:*}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rounds/tr_$n -o run -- python3 tools/ab_bench.py --scene $S --reps 1 v: > gpurun_out/rounds/$n.log 2>&1 || { echo "rc=$?"; tail gpurun_out/rounds/$n.log; exit 1; }
done
find gpurun_out/rounds -name '*kernel_trace.csv' | head
