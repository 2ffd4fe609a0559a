#!/usr/bin/env python3
"""Condense a tools/gpu_profile.sh run (gpurun_out/prof_<tag>/) into
profiles/<tag>_summary.json + copies of the rocprofv3 stats CSV.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB, collected in separate passes; on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced read, so it is doubled."""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag, kernel_substr="render_kernel<false, "):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats_csv = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats_csv, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    kern = {}
    for row in csv.DictReader(open(stats_csv)):
        kern[row["Name"]] = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                             "min_ns": float(row["MinNs"]), "max_ns": float(row["MaxNs"]),
                             "percent": float(row["Percentage"])}
    pmc = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        path = os.path.join(src, f"pmc_{c}", "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
                if kernel_substr in r["Kernel_Name"] and r["Counter_Name"] == c]
        if vals:
            pmc[c] = sum(vals) / len(vals)
    sq = {}
    path = os.path.join(src, "pmc_SQ_INSTS_VALU", "run_counter_collection.csv")
    if os.path.exists(path):
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES"):
            vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
                    if kernel_substr in r["Kernel_Name"] and r["Counter_Name"] == c]
            if vals:
                sq[c] = sum(vals) / len(vals)
    import hashlib
    src_hash = hashlib.sha1(open(os.path.join(ROOT, "discovering-path-tracer_amd", "csrc", "pt_device.hip"),
                                 "rb").read()).hexdigest()
    out = {"tag": tag, "kernels": kern, "kernel": kernel_substr, "pt_device_hip_sha1": src_hash}
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        fetch = pmc["FETCH_SIZE"] * 1024 * 2      # gfx950: FETCH_SIZE counts half of wide reads
        write = pmc["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch"] = {"fetch_corrected": fetch, "write": write, "total": fetch + write,
                                       "raw_fetch_kib": pmc["FETCH_SIZE"], "raw_write_kib": pmc["WRITE_SIZE"]}
    if sq:
        out["sq_per_launch"] = sq
    for log in ("bench_trace.log",):
        p = os.path.join(src, log)
        if os.path.exists(p):
            lines = [l for l in open(p) if l.startswith("{")]
            if lines:
                out["bench_line"] = json.loads(lines[-1])
    json.dump(out, open(os.path.join(dst, f"{tag}_summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1)[:3000])


if __name__ == "__main__":
    main(*sys.argv[1:])
