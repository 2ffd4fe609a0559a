set -u
cd "${GRAFT_REPO_ROOT}"
for args in "--scene sphere:6 --spp 1" "--scene sphere:6 --spp 8 --w 1920 --h 1080" "--scene sphere:5 --spp 2" "--scene random:100000 --spp 1" "--scene random:1000000 --spp 1"; do
  timeout -k 10 200 python3 tools/ab_bench.py $args --reps 3 rec:opt4=1 wf:opt4=3 > gpurun_out/sel.log 2>&1 || { tail -5 gpurun_out/sel.log; exit 1; }
  echo "$args $(tail -1 gpurun_out/sel.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: round(v["mean_ms"],2) for k,v in d["results"].items()})')"
done
for nr in 2 4 8; do
  timeout -k 10 200 python3 tools/ab_bench.py --scene sphere:6 --spp 8 --reps 3 rec:opt4=1,nr=$nr wf:opt4=3,nr=$nr > gpurun_out/sel.log 2>&1 || { tail -5 gpurun_out/sel.log; exit 1; }
  echo "sphere:6 8spp nr=$nr $(tail -1 gpurun_out/sel.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: round(v["mean_ms"],2) for k,v in d["results"].items()})')"
done
