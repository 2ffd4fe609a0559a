#!/usr/bin/env python3
"""Condense a tools/profile_workload.sh run (gpurun_out/prof_<tag>_<workload>/)
into profiles/<tag>/<workload>_summary.json + the rocprofv3 stats CSV.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are KiB, from separate passes; FETCH_SIZE is doubled.  The guide
calibrates x2 for 16-B/lane streaming reads; profiles/r02/fetch_calibration.json
(tools/fetch_calib.hip + request counters) shows it holds for the random
32-B/48-B gathers of the traversal too: every fabric read request is a 128-B
line and FETCH_SIZE tallies 64 B per request.  Raw readings are kept.

box: the dominant kernel is one render_kernel launch per frame (averaged over
its dispatches).  sphere/synthetic: a frame is the wavefront pipeline
(wf_gen, wf_trace x rays, wf_shade x rays, wf_fold, fill_culled): per-frame
bytes = the sum over every dispatch of those kernels / frames."""
import csv
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BOX_KERNEL = "render_kernel<false, true, false>"
KERNEL_SOURCES = ("pt_device.hip", "pt_device.h", "pt_isect.h", "wide_walk.h", "pt_math.h", "scene/wide_bvh.cpp",
                  "../Makefile")   # the Makefile: the device build flags   # == bench.py
WF_KERNELS = ("wf_gen_kernel", "wf_trace_kernel", "wf_trace_wide_kernel", "wf_trace_pairs_kernel", "wf_tail_kernel", "wf_shade_kernel",
              "wf_fold_kernel", "fill_culled_kernel")


def main(tag, workload, frames):
    frames = int(frames)
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_{workload}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    stats_csv = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats_csv, os.path.join(dst, f"{workload}_kernel_stats.csv"))
    kern = {}
    for row in csv.DictReader(open(stats_csv)):
        kern[row["Name"]] = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                             "total_ns": float(row["TotalDurationNs"]), "percent": float(row["Percentage"])}
    box = workload == "box"
    match = (lambda k: BOX_KERNEL in k) if box else (lambda k: any(w in k for w in WF_KERNELS))

    def per_launch(path, names):
        if not os.path.exists(path):
            return {}
        vals = {}
        for r in csv.DictReader(open(path)):
            if match(r["Kernel_Name"]) and r["Counter_Name"] in names:
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        return {c: (sum(v) / len(v) if box else sum(v) / frames) for c, v in vals.items()}

    pmc = {}
    pmc.update(per_launch(os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv"), ("FETCH_SIZE",)))
    # per kernel family (FETCH_SIZE KiB per frame): where the reads come from
    fam_fetch = {}
    fpath = os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv")
    if os.path.exists(fpath) and not box:
        for r in csv.DictReader(open(fpath)):
            if match(r["Kernel_Name"]) and r["Counter_Name"] == "FETCH_SIZE":
                f = next(w for w in WF_KERNELS if w in r["Kernel_Name"])
                fam_fetch[f] = fam_fetch.get(f, 0.0) + float(r["Counter_Value"]) / frames
    pmc.update(per_launch(os.path.join(src, "pmc_WRITE_SIZE", "run_counter_collection.csv"), ("WRITE_SIZE",)))
    sq = per_launch(os.path.join(src, "pmc_SQ_INSTS_VALU", "run_counter_collection.csv"),
                    ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES"))
    # the kernel source: pt_device.hip, the headers its kernels are built from and the Makefile (build flags)
    h = hashlib.sha1()
    for name in KERNEL_SOURCES:
        h.update(open(os.path.join(ROOT, "discovering-path-tracer_amd", "csrc", name), "rb").read())
    src_hash = h.hexdigest()
    if box:
        ns = [v["avg_ns"] for k, v in kern.items() if BOX_KERNEL in k]
        kernel_ms = ns[0] / 1e6 if ns else None
    else:
        kernel_ms = sum(v["total_ns"] for k, v in kern.items() if match(k)) / frames / 1e6
    out = {"tag": tag, "workload": workload, "unit": "per launch" if box else f"per frame ({frames} frames)",
           "kernel": BOX_KERNEL if box else "+".join(WF_KERNELS), "pt_device_hip_sha1": src_hash,
           "kernel_ms_per_launch": kernel_ms, "kernels": kern}
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        fetch = pmc["FETCH_SIZE"] * 1024 * 2
        write = pmc["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch"] = {"fetch_corrected": fetch, "write": write, "total": fetch + write,
                                       "raw_fetch_kib": pmc["FETCH_SIZE"], "raw_write_kib": pmc["WRITE_SIZE"]}
        if fam_fetch:
            out["fetch_kib_by_kernel"] = fam_fetch
        if kernel_ms:
            out["hbm_GBps"] = {"x2_corrected": (fetch + write) / kernel_ms / 1e6,
                               "raw": (pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024 / kernel_ms / 1e6}
    cal = os.path.join(ROOT, "profiles", "r02", "fetch_calibration.json")
    if os.path.exists(cal):
        out["fetch_calibration"] = {k: v["fetch_over_algorithmic"] for k, v in json.load(open(cal)).items()
                                    if isinstance(v, dict) and "fetch_over_algorithmic" in v}
        out["fetch_calibration"]["source"] = "profiles/r02/fetch_calibration.json (x2 holds for 128-B line requests)"
    if sq:
        out["sq_per_launch"] = sq
    # L2 hits and misses of the traversal kernel alone (its node fetches, ray
    # and triangle loads): the hit fraction the gather ceiling of a partly
    # L2-resident tree is priced with (bench.py gather_roofline)
    tpath = os.path.join(src, "pmc_TCC_HIT_sum", "run_counter_collection.csv")
    if os.path.exists(tpath):
        tcc = {}
        for r in csv.DictReader(open(tpath)):
            k = r["Kernel_Name"]
            fam = "trace" if ("wf_trace_wide_kernel" in k or (box and BOX_KERNEL in k)) else None
            if fam and r["Counter_Name"] in ("TCC_HIT_sum", "TCC_MISS_sum"):
                tcc[r["Counter_Name"]] = tcc.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"]) / frames
        if tcc.get("TCC_HIT_sum", 0.0) + tcc.get("TCC_MISS_sum", 0.0) > 0:
            tot = tcc.get("TCC_HIT_sum", 0.0) + tcc.get("TCC_MISS_sum", 0.0)
            out["trace_kernel_l2"] = {"hits_per_frame": tcc.get("TCC_HIT_sum", 0.0),
                                      "misses_per_frame": tcc.get("TCC_MISS_sum", 0.0),
                                      "hit_fraction": tcc.get("TCC_HIT_sum", 0.0) / tot}
    p = os.path.join(src, "bench_trace.log")
    if os.path.exists(p):
        lines = [l for l in open(p) if l.startswith("{")]
        if lines:
            out["bench_line"] = json.loads(lines[-1])
    json.dump(out, open(os.path.join(dst, f"{workload}_summary.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k not in ("kernels", "bench_line")}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
