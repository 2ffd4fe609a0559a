set -e
for args in "--scene sphere:6 --refcam --grid 30" "--scene sphere:6 --grid 100" "--scene sphere:6 --refcam --grid 100" "--scene random:10000000 --refcam --grid 33" "--scene random:10000000 --grid 100"; do
  PTAMD_LIB=ab/probe.so timeout -k 10 200 python3 tools/wide_probe.py $args | tail -1
done
