#!/bin/bash
# (writes gpurun_out/calib_<TAG>/fetch_calibration.json; copy it to profiles/<TAG>/)
# FETCH_SIZE calibration for the large-scene access patterns (tools/fetch_calib.hip,
# built in the container: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/calib_${TAG:-x}
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc -o run -- ./tools/fetch_calib > $OUT/calib.log 2>&1 \
  || { echo "calib rc=$?"; tail -20 $OUT/calib.log; exit 1; }
cat $OUT/calib.log
python3 - "$OUT" "${TAG:-x}" <<'PY'
import csv, glob, json, os, sys
out, tag = sys.argv[1], sys.argv[2]
known = {}
for l in open(os.path.join(out, "calib.log")):
    if l.startswith("{"):
        d = json.loads(l)
        known[d["kernel"]] = d
res = {}
for f in glob.glob(out + "/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        for k, d in known.items():
            if k in r["Kernel_Name"]:
                res[k] = {"algorithmic_bytes": d["bytes"], "fetch_size_bytes": float(r["Counter_Value"]) * 1024,
                          "ms": d["ms"], "GBps": d["bytes"] / d["ms"] / 1e6}
for k, v in res.items():
    v["fetch_over_algorithmic"] = v["fetch_size_bytes"] / v["algorithmic_bytes"]
json.dump(res, open(os.path.join(out, "fetch_calibration.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
PY
