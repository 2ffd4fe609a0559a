#!/usr/bin/env python3
"""Benchmark: Mrays/s of the path-tracing pixel kernel on box.obj at
1920x1080, 8 spp, 4 bounces (BASELINE.json configs[1]), on 1..N GPUs.

A step is one frame.  It renders the 8 sample batches from a fresh
accumulator in one fused launch, bit-identical to 8 progressive 1-spp
dispatches after a clear.  For N > 1 the frame is split into 16x16 screen
tiles (tile b on rank b % N).  Every rank packs the tile parts that can
hold a live pixel (primary culling) and the root assembles them with one
RCCL gather, rebuilding the culled parts.  The gather of frame k overlaps the
render of frame k+1 (double-buffered); the timed region ends only after the
last frame is assembled.

Mrays/s counts the reference's traceRay invocations of all kinds: light
pre-pass, primary/bounce, shadow, SSS and SSS-shadow.  A stats-mode pass of
the same frame, run before the timed region, measures them.

The kernel skips work the reference does without changing a bit of the
output (culled primary rays, shadow rays whose answer cannot change the
image, the repeated pre-pass ray): a counting pass of the fast kernel
(PT_OPT_COUNT_TRACED, untimed) reports the walks it really starts as
config.rays_traced next to the reference-equivalent rays_per_frame.

roofline (the dominant kernel): HBM bytes per launch from the committed
rocprofv3 FETCH_SIZE/WRITE_SIZE summary of this exact kernel source
(profiles/, matched by SHA-1 of pt_device.hip and by workload) over the
kernel time measured here with HIP events.  The algorithmic bytes of
SURVEY §8d (exhaustive reference counts) over the same time are reported as
effective_GBps: on box.obj the scene is staged in LDS, so that figure is far
above the HBM peak and is not a bandwidth.

At N = 1 the line also carries `configs`: config 3 (the level-6 displaced
icosphere standing in for the missing Sylveon.obj) at 1920x1080x8spp,
config 4 (the same mesh at 3840x2160x16spp, 8 bounces) and config 5 (10M
random triangles, 1920x1080x8spp), each timed, counted and roofline-priced
the same way.  At N > 1 `configs` holds configs 4 and 5 split across the N
GPUs (screen tiles, RCCL SUM reduce of the accumulation buffer), each
checked bitwise against a one-GPU render of the same frame on rank 0
(--no-scene-legs skips the legs).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run, one process per GPU.  Rank 0 prints one JSON line.
Other workloads: --scene sphere (the labelled Sylveon substitute) or
--scene synthetic:<T> (SURVEY §8d config 5 cloud, camera at z=2.2).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

T_START = time.perf_counter()
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "discovering-path-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_ACHIEVABLE_GBS = 6300.0    # the guide's measured achievable HBM rate (MI355X_MICROARCH.md §HBM)
# VALU issue peak: 1024 SIMDs x 2.4 GHz, one wave64 f32 instruction per 2
# cycles per SIMD (MI355X_MICROARCH.md constants: v_fma_f32 2 cyc on SIMD-32)
VALU_PEAK_GINST = 1024 * 2.4 / 2


def algorithmic_bytes(st):
    """32 B per BVH node visited + 48 B per leaf triangle test
    (12 B indices + 36 B vertices) under the reference's exhaustive traversal,
    + 32 B accumulation read-modify-write per pixel-sample."""
    return 32 * st["nodes"] + 48 * st["leaf_tests"] + 32 * st["samples"]


def build_threads():
    """Host threads for one process's BVH build: its usable CPUs shared by
    the processes of this node (LOCAL_WORLD_SIZE ranks build at once)."""
    return max(1, cpu_threads() // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1"))))


def load_scene(name):
    import ptamd
    import scenes
    if name == "box":
        s = ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh()
        return s, scenes.DEFAULT_CAMERA, False, "box.obj, camera (0,0,5) fov 60"
    if name == "sphere":
        v, i = scenes.displaced_sphere(6)
        s = ptamd.Scene.from_arrays(v, i).build_bvh(threads=build_threads())
        return (s, scenes.camera((0.0, 0.5, 3.0)), False,
                f"displaced icosphere ({i.size // 3} tris, Sylveon substitute), camera (0,0.5,3) fov 60")
    if name.startswith("synthetic:"):
        t = int(name.split(":")[1])
        v, i = scenes.random_triangles(t, seed=42)
        big = 2 * t - 1 >= (1 << 24)
        s = ptamd.Scene.from_arrays(v, i).build_bvh(int_bits=big, threads=build_threads())
        return s, scenes.camera((0.0, 0.0, 2.2)), big, f"synthetic {t} random triangles, camera (0,0,2.2) fov 60"
    raise SystemExit(f"unknown scene {name}")


KERNEL_SOURCES = ("pt_device.hip", "pt_device.h", "pt_isect.h", "wide_walk.h", "pt_math.h", "scene/wide_bvh.cpp",
                  "../Makefile")   # the Makefile: the device build flags


def kernel_sha1():
    """SHA-1 of the kernel source (pt_device.hip, the headers its kernels
    are built from and the Makefile that holds the device build flags), as
    tools/summarize_profile.py records it."""
    import hashlib
    h = hashlib.sha1()
    for f in KERNEL_SOURCES:
        h.update(open(os.path.join(ROOT, "discovering-path-tracer_amd", "csrc", f), "rb").read())
    return h.hexdigest()


def leg_traffic(workload):
    """The committed profile of a leg's workload taken in the configuration
    the leg times (`<workload>_leg`, bench.py --leg), else the one-context
    profile of the same workload."""
    return profiled_traffic(workload + "_leg") or profiled_traffic(workload)


def profiled_traffic(workload=None):
    """HBM bytes per launch (per frame for the wavefront pipeline) of the
    current kernel source from the newest committed rocprofv3 PMC summary
    (tools/profile_workload.sh ->
    tools/summarize_profile.py) whose pt_device.hip SHA-1 and workload match.
    None if there is none.  Returns the summary dict and its path."""
    import glob
    h = kernel_sha1()
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "*_summary.json"), recursive=True)):
        try:
            d = json.load(open(p))
        except ValueError:
            continue
        if d.get("pt_device_hip_sha1") != h or "hbm_bytes_per_launch" not in d:
            continue
        if workload is not None and d.get("workload") != workload:
            continue
        if workload is None and d.get("workload") not in (None, "box"):
            continue
        best = (os.path.relpath(p, ROOT), d)
    return best


def cpu_threads():
    """Cores this process can actually use: its sched affinity, capped by the
    cgroup CPU quota (the GPU box shows all 256 host CPUs but grants 16 --
    256 threads on a 16-CPU quota measured 22 Mrays/s against 33 on 16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    q = cpu_quota()
    if q is not None:
        n = min(n, max(1, int(-(-q // 1))))
    return n


def cpu_quota():
    """cgroup v2 CPU quota in CPUs (None when unlimited or unreadable)."""
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(v, i, n, cam, light, W, H, spp, DEPTH, SSS):
    """The oracle (scalar C++ restatement of raytrace_comp.comp) on this host,
    on every CPU the process may use, on a bounded sample of the same
    workload, plus the same traversal on one core.  Returns the baseline
    block and the oracle's image when the sample is the whole frame (else
    None): main() checks the timed GPU frame against it bit for bit."""
    import oracle_lib
    threads = cpu_threads()
    stride = 1 if W * H <= 1920 * 1080 else 4
    oracle_lib.render(v, i, n.reshape(-1), cam, light, 64, 64, n_batches=1, nthreads=threads)   # warm
    t0 = time.perf_counter()
    img, st = oracle_lib.render(v, i, n.reshape(-1), cam, light, W, H, n_batches=spp, max_depth=DEPTH,
                              sss_bounces=SSS, row_stride=stride, row_phase=0, nthreads=threads)
    dt = time.perf_counter() - t0
    image = img if stride == 1 else None   # the whole frame: the timed frame is checked against it
    # the scalar traversal on one core, on every 16th row of those
    s1 = stride * 16
    t1 = time.perf_counter()
    _, st1 = oracle_lib.render(v, i, n.reshape(-1), cam, light, W, H, n_batches=spp, max_depth=DEPTH,
                               sss_bounces=SSS, row_stride=s1, row_phase=0, nthreads=1)
    dt1 = time.perf_counter() - t1
    return {"value": round(float(st[0]) / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"rows y%{stride}==0 of the same {W}x{H}x{spp}spp frame ({H // stride} rows, "
                      f"{int(st[0])} rays, {dt:.2f} s, {threads} std::threads, oracle/pt_oracle.cpp)",
            "host_cpus_visible": os.cpu_count(), "cpus_allowed": threads, "cgroup_cpu_quota": cpu_quota(),
            "single_thread": {"value": round(float(st1[0]) / dt1 / 1e6, 3), "unit": "Mrays/s", "cores": 1,
                              "sample": f"rows y%{s1}==0 ({int(st1[0])} rays, {dt1:.2f} s)"}}, image


KERNEL_NAMES = {1: "render_kernel<false,*>",
                3: "wavefront pipeline (wf_gen + wf_trace/wf_shade x rays + wf_fold), per frame"}

TRACED_KEYS = ("closest_walks", "shadow_walks", "nodes", "tri_tests", "primaries")


def reference_and_traced_counts(r, spp):
    """One untimed frame in stats mode (the reference-exhaustive traversal:
    every traceRay with its exhaustive node and leaf counts) and one with the
    fast kernel's counters on (PT_OPT_COUNT_TRACED: the walks, node visits
    and triangle tests it really performs).  Both frames are bit-identical
    to the timed ones."""
    import ptamd
    r.set_stats_mode(True)
    r.reset_stats()
    r.clear()
    r.render(0, spp)
    st = r.stats()
    r.set_stats_mode(False)
    r.set_option(ptamd.PT_OPT_COUNT_TRACED, 1)
    r.reset_stats()
    r.render(0, spp)
    traced = r.traced()
    r.set_option(ptamd.PT_OPT_COUNT_TRACED, 0)
    return np.array([st["rays"], st["nodes"], st["leaf_tests"], st["samples"]], np.float64), traced


def add_traced(cfg, traced, seconds_per_frame):
    """config.rays_traced (walks the kernel really starts: closest-hit plus
    shadow) beside the reference-equivalent rays_per_frame, and its rate."""
    rays = traced["closest_walks"] + traced["shadow_walks"]
    cfg["rays_traced"] = int(rays)
    cfg["rays_traced_per_s_M"] = round(rays / seconds_per_frame / 1e6, 3)
    cfg["traced"] = {k: int(traced[k]) for k in TRACED_KEYS}
    if cfg.get("rays_per_frame"):
        cfg["rays_traced_frac_of_reference"] = round(rays / cfg["rays_per_frame"], 4)


def roofline_block(prof, time_ms, alg_bytes, kernel, kernel_ms, interval_ms, n_timed, time_basis):
    """The HBM roofline of the dominant kernel: committed-profile HBM bytes per
    launch (FETCH_SIZE x2 per the guide's gfx950 correction, + WRITE_SIZE)
    over the kernel time measured in this run.  The algorithmic bytes of
    SURVEY §8d over the same time are `effective_GBps`."""
    traffic = None if prof is None else prof[1]["hbm_bytes_per_launch"]["total"]
    achieved = None if traffic is None else traffic / (time_ms * 1e-3) / 1e9
    eff = alg_bytes / (time_ms * 1e-3) / 1e9 if alg_bytes else None
    out = {"bound": "hbm",
           "achieved": None if achieved is None else round(achieved, 2),
           "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": None if achieved is None else round(achieved / HBM_PEAK_GBS, 5),
           "traffic": None if traffic is None else int(traffic),
           "traffic_source": None if prof is None else prof[0],
           "kernel": kernel, "kernel_ms": round(kernel_ms, 4), "launch_interval_ms": round(interval_ms, 4),
           "timed_launches": n_timed, "time_basis": time_basis,
           "algorithmic_bytes_per_launch": None if not alg_bytes else int(alg_bytes),
           "effective_GBps": None if eff is None else round(eff, 2),
           "frac_of_achievable": None if achieved is None else round(achieved / HBM_ACHIEVABLE_GBS, 5),
           "achievable_GBps": HBM_ACHIEVABLE_GBS,
           "traffic_basis": "rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per launch (every gfx950 fabric read request is a "
                            "128-B line tallied at 64 B: profiles/r02/fetch_calibration.json)",
           "traffic_label": "L2-miss fabric bytes: HBM plus Infinity-Cache (MALL) hits, which FETCH_SIZE counts "
                            "(MI355X_MICROARCH.md, HBM section); an upper bound on HBM bytes, so frac bounds the HBM "
                            "fraction from above"}
    if prof is not None:
        hb = prof[1]["hbm_bytes_per_launch"]
        if "raw_fetch_kib" in hb:
            raw = (hb["raw_fetch_kib"] + hb["raw_write_kib"]) * 1024
            out["traffic_raw_counters"] = int(raw)
            out["frac_raw_counters"] = round(raw / (time_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
        if "fetch_calibration" in prof[1]:
            out["fetch_calibration"] = prof[1]["fetch_calibration"]
    if traffic is None:
        out["note"] = "no committed rocprofv3 summary of this kernel source and workload: traffic unmeasured"
    elif eff is not None and eff > HBM_PEAK_GBS:
        out["note"] = ("effective_GBps counts the reference's exhaustive node/triangle bytes (SURVEY 8d) over the "
                       "kernel time; the kernel serves them from LDS/L2/MALL and skips exact no-op work, so it can "
                       "exceed the HBM peak.  frac is the measured HBM traffic over the kernel time")
    return out


# The BASELINE configs the default run reports beside the headline, one GPU
# each: (key, scene, W, H, spp, MAX_DEPTH, timed frames, profile workload,
# (contexts, grid %) at BASELINE's camera, (contexts, grid %) at the
# frame-filling camera).  Frames alternate over that many contexts (own
# stream, accumulation and wavefront buffers each), each context's
# traversal launches on `grid` % of a full persistent grid (PT_OPT_WF_GRID):
# with C contexts at 100/C % every frame's rounds run side by side with more
# rays per lane, instead of each launch taking the whole GPU and leaving its
# drain to the others.  Measured one variant per process (profiles/r05c,
# profiles/r05d, r05g, r05l; with the split grid's refill at 8 idle lanes):
# config 3 at (0,0,5) 3 contexts 15.7 ms -> 4 at 25 % 13.2; config 4 at
# (0,0,5) 1 context 141.5 -> 2 at 50 % 131.3 (3 at 33 % ~132-135, 4 at 25 %
# 151); config 5 at (0,0,5) 1 context 23.3 -> 3 at 33 % 17.7.  At the
# frame-filling cameras config 3 36.1 -> 34.7 (4 at 25 %), config 4 360.4 ->
# 351.4 (2 at 50 %), config 5 111.1 -> 110.3 (2 at 100 %; 2 at 50 % 112.9).
# Config 3 at 4 x 30 % (shares overlapping by a fifth) rather than 25: at the
# frame-filling camera 33.3 -> 32.95 ms, at (0,0,5) 12.72 -> 12.68
# (profiles/r05z/c3ff_grid.log, six runs each, the final build).
# Config 4 times runs of 6 frames: with 3 the runs were mostly the pipeline's
# fill and drain.  A run's frame count is a multiple of the contexts at both
# cameras, so its last frames do not run on part of the grid alone: config 5
# at (0,0,5) (3 x 33 %) measured 18.4 ms per frame in runs of 5 frames, 18.9
# in runs of 10 and 17.4 in runs of 20 (profiles/r05w/frames.log); configs 3
# and 4, whose runs already were such multiples, within 0.4 % at 2-4 times
# the frames.
SCENE_LEGS = (("config3", "sphere", 1920, 1080, 8, 4, 12, "sphere_1080p8", (4, 30), (4, 30)),
              ("config4", "sphere", 3840, 2160, 16, 8, 6, "sphere_4k16_d8", (2, 50), (2, 50)),
              ("config5", "synthetic:10000000", 1920, 1080, 8, 4, 12, "synthetic10M_1080p8", (3, 33), (2, 100)))


# Which measured gather ceiling bounds each leg's trace kernel: the 2.6-MB
# wide tree of the displaced sphere (configs 3, 4) is L2-resident; the 10M
# cloud's 313-MB tree is not (its leg keeps the fabric-bytes roofline primary,
# the gather ceiling beside it).  The ceiling is the best rate of 64-B record
# fetches (four 16-B loads per record per lane, the trace kernel's own access)
# over every memory-level parallelism measured at the trace kernel's
# occupancy -- 1, 2 or 4 dependent chains per lane, 2, 4 or 8 independent
# records in flight per lane (tools/gather_roof.hip mlp) -- so no kernel
# fetching such records at that occupancy can beat it (VERDICT r04 item 4:
# the one-chain figure alone was beaten).
GATHER_CASES = {"sphere_1080p8": ("l2_gather", "l2_4MB"), "sphere_4k16_d8": ("l2_gather", "l2_4MB"),
                "synthetic10M_1080p8": ("hbm_gather", "hbm1GB")}
GATHER_FILE = os.path.join("profiles", "r05", "gather_roof_mlp.jsonl")


def gather_rows(case):
    """The measured 64-B record gather rates of one table case, or []."""
    try:
        rows = [json.loads(x) for x in open(os.path.join(ROOT, GATHER_FILE)) if x.strip().startswith("{")]
    except (OSError, ValueError):
        return []
    return [d for d in rows if d.get("case") == case and d.get("record_B") == 64]


def _pattern(d):
    return (f"chains{d['chains_per_lane']}" if d["pattern"] == "dependent_chains"
            else f"independent{d['records_in_flight_per_lane']}")


def gather_roofline(workload, prof=None):
    """The fetch-rate ceiling of the wide walk's node fetches for a leg.
    l2_gather (configs 3/4, a 2.6-MB tree): the best rate any measured
    pattern reaches from an L2-resident table.  hbm_gather (config 5, a
    313-MB tree whose upper levels stay in L2): with h the trace kernel's L2
    hit fraction (TCC_HIT / (TCC_HIT + TCC_MISS), committed profile), a frame
    of N fetches needs at least h N / R_L2 of L2 service and (1 - h) N /
    R_miss of miss service, so its rate is at most min(R_L2 / h, R_miss /
    (1 - h)) -- a ceiling even if both overlap perfectly (without h: R_L2)."""
    base = workload[:-len("_refcam")] if workload.endswith("_refcam") else workload
    if base not in GATHER_CASES:
        return None
    bound, case = GATHER_CASES[base]
    l2 = gather_rows("l2_4MB")
    if not l2:
        return None
    best_l2 = max(l2, key=lambda d: d["Grec_per_s"])
    pats = {"l2_4MB": {_pattern(d): d["Grec_per_s"] for d in l2}}
    if bound == "l2_gather":
        return {"bound": bound, "Grec_per_s": best_l2["Grec_per_s"], "patterns": pats,
                "basis": f"tools/gather_roof.hip mlp: the best of {len(l2)} access patterns of 64-B records (four "
                         f"16-B loads each) from a {best_l2['table_MB']}-MB table at 6 workgroups of 256 per CU "
                         f"({_pattern(best_l2)}; {GATHER_FILE})"}
    miss = gather_rows(case)
    if not miss:
        return None
    best_miss = max(miss, key=lambda d: d["Grec_per_s"])
    pats[case] = {_pattern(d): d["Grec_per_s"] for d in miss}
    h = None if prof is None else prof[1].get("trace_kernel_l2", {}).get("hit_fraction")
    r_l2, r_miss = best_l2["Grec_per_s"], best_miss["Grec_per_s"]
    if h is None:
        ceil, how = r_l2, "no L2 hit fraction in the committed profile: the L2-resident ceiling"
    else:
        ceil = min(r_l2 / h if h > 0 else float("inf"), r_miss / (1.0 - h) if h < 1 else float("inf"))
        how = (f"min(R_L2 / h, R_miss / (1 - h)) with h = {h:.3f} (the trace kernel's L2 hit fraction, "
               f"{prof[0]}), R_L2 = {r_l2} ({_pattern(best_l2)}, 4-MB table), R_miss = {r_miss} "
               f"({_pattern(best_miss)}, {best_miss['table_MB']}-MB table)")
    return {"bound": bound, "Grec_per_s": round(ceil, 2), "patterns": pats, "l2_hit_fraction": h,
            "basis": f"tools/gather_roof.hip mlp, 64-B records at 6 workgroups of 256 per CU: {how} "
                     f"({GATHER_FILE})"}


def trace_share(prof):
    """wf_trace_wide_kernel's share of the frame's kernel time in a committed
    rocprofv3 summary (None without one)."""
    if prof is None:
        return None
    ks = prof[1].get("kernels", {})
    tot = sum(v.get("total_ns", 0.0) for k, v in ks.items() if "ptd::" in k)
    tr = sum(v.get("total_ns", 0.0) for k, v in ks.items() if "wf_trace_wide_kernel" in k)
    return tr / tot if tot > 0 and tr > 0 else None


def time_frames(r, spp, steps):
    """`steps` timed frames, one at a time (each synchronized): wall ms per
    frame and the kernel ms of each frame's launches (HIP events)."""
    walls = []
    r.reset_launch_times()
    for _ in range(steps):
        t0 = time.perf_counter()
        r.render(0, spp)
        r.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3)
    return np.array(walls), r.launch_times_ms()


def hip_runtime():
    """The HIP runtime already mapped into this process (torch's, which
    libptamd binds to by SONAME), opened with RTLD_NOLOAD: a stream made
    through another copy of the runtime would not be valid in torch's or
    libptamd's."""
    import ctypes
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 6 and os.path.basename(parts[-1]).startswith("libamdhip64.so"):
                return ctypes.CDLL(parts[-1], mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL)
    raise RuntimeError("the HIP runtime is not loaded (import torch and initialise its device first)")


class HipStream:
    """A HIP stream made for one context of a frames-in-flight run
    (non-blocking, the least priority), with a torch view of it
    (ExternalStream) for collectives that must follow its work.  The HIP
    runtime gives streams hardware queues as they are created, up to
    GPU_MAX_HW_QUEUES (4 here) per priority, then shares the least-used one;
    torch's pool streams, handed out round-robin, were seen to put two busy
    contexts on one queue in later legs of a run (config 3: 38.3 ms per frame
    in the first leg, 40.5 in a later one; two contexts 38.9 vs 43.6).  Each
    context of a leg gets a stream of the least priority created for it --
    a queue pool no other stream of the process uses -- released with the
    leg, so a leg's (at most three) streams get queues of their own."""

    def __init__(self, device):
        import ctypes
        import torch
        self._hip = hip_runtime()
        self._hip.hipSetDevice(ctypes.c_int(device))
        least, greatest = ctypes.c_int(0), ctypes.c_int(0)
        self._hip.hipDeviceGetStreamPriorityRange(ctypes.byref(least), ctypes.byref(greatest))
        h = ctypes.c_void_p()
        # the least priority: a queue pool of its own, away from torch's
        # (normal) and RCCL's (high-priority) streams
        rc = self._hip.hipStreamCreateWithPriority(ctypes.byref(h), ctypes.c_uint(1), least)
        if rc != 0:
            raise RuntimeError(f"hipStreamCreateWithPriority: error {rc}")
        self.handle = h.value
        self.torch = torch.cuda.ExternalStream(self.handle, device=torch.device("cuda", device))

    def close(self):
        import ctypes
        if self.handle:
            self._hip.hipStreamSynchronize(ctypes.c_void_p(self.handle))
            self._hip.hipStreamDestroy(ctypes.c_void_p(self.handle))
            self.handle = None


def time_frames_pipelined(ctxs, spp, steps, groups=3):
    """`groups` runs of `steps` frames alternating between the contexts with
    no wait in between (frames overlap on the GPU): wall ms per frame of each
    run."""
    import torch
    walls = []
    for _ in range(groups):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            ctxs[k % len(ctxs)].render(0, spp)
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3 / steps)
    return np.array(walls)


def spread(ms):
    return {"min": round(float(np.min(ms)), 3), "median": round(float(np.median(ms)), 3),
            "max": round(float(np.max(ms)), 3), "frames": int(ms.size)}


def price_leg(out, workload, traced, kernel_ms, alg, ref_rays):
    """The leg's rooflines from the committed profile of `workload` (this
    kernel source and camera): HBM (roofline_block), the wide walk's node
    fetches against the measured gather ceiling (configs 3/4 primary, config
    5 beside HBM) and VALU issue."""
    prof = leg_traffic(workload)
    gather = gather_roofline(workload, prof)
    if gather is not None:
        # the wide walk's node fetches against the measured ceiling of
        # dependent 64-B gathers from a table of the tree's size at the trace
        # kernel's occupancy and memory-level parallelism (tools/gather_roof.hip)
        visits = float(traced["nodes"])
        ach = visits / (kernel_ms * 1e-3) / 1e9
        roof = {"bound": gather["bound"], "achieved": round(ach, 3), "peak": gather["Grec_per_s"],
                "unit": "G wide-node fetches/s", "frac": round(ach / gather["Grec_per_s"], 4),
                "node_visits_per_frame": int(visits), "peak_basis": gather["basis"],
                "peak_patterns_Grec_per_s": gather.get("patterns"),
                "time_basis": out["roofline"]["time_basis"] + "; every kernel of the frame"}
        share = trace_share(prof)
        if share is not None:
            # the trace kernel's own time: its share of the frame's kernel
            # time in the committed profile of this source and workload
            roof["trace_kernel_share"] = round(share, 4)
            roof["achieved_trace_kernel"] = round(ach / share, 3)
            roof["frac_trace_kernel"] = round(ach / share / gather["Grec_per_s"], 4)
        if gather["bound"] == "hbm_gather":
            out["roofline_gather"] = roof   # beside the fabric-bytes roofline (config 5)
        else:
            roof["traffic"] = out["roofline"]["traffic"]
            roof["hbm"] = {k: out["roofline"][k] for k in ("achieved", "peak", "unit", "frac", "traffic",
                                                           "traffic_source", "traffic_label")}
            out["roofline"] = roof
    if prof is not None and prof[1].get("sq_per_launch", {}).get("SQ_INSTS_VALU"):
        # the same frame against the VALU issue peak (committed PMC profile)
        valu = prof[1]["sq_per_launch"]["SQ_INSTS_VALU"]
        gi = valu / (kernel_ms * 1e-3) / 1e9
        out["roofline_valu"] = {"achieved": round(gi, 2), "peak": VALU_PEAK_GINST, "unit": "G wave-instr/s",
                                "frac": round(gi / VALU_PEAK_GINST, 4), "valu_wave_instr_per_frame": int(valu),
                                "source": prof[0],
                                "peak_basis": "1024 SIMDs x 2.4 GHz / 2 cycles per wave64 f32 instruction"}


def leg_contexts(scene_name, W, H, depth, sss, device, contexts):
    """A scene leg's contexts on one GPU: each with the scene, the reference
    light and params, its own least-priority stream when there are several
    (HipStream), launch timing on the first only.  Returns (contexts, their
    HipStreams, the scene's frame-filling camera, int_bits, description,
    triangles)."""
    import ptamd
    import scenes
    scene, cam, int_bits, desc = load_scene(scene_name)
    v, i, n, _, _ = scene.arrays()
    del scene
    ctxs = []
    hip_streams = []
    for _ in range(contexts):
        x = ptamd.Renderer(device)
        x.upload_scene(v, i, n, int_bits=int_bits)
        x.upload_lights(scenes.REFERENCE_LIGHT)
        x.set_params(depth, sss)
        if contexts > 1:
            hs = HipStream(device)
            hip_streams.append(hs)
            x.set_stream(hs.handle)
        x.set_option(ptamd.PT_OPT_LAUNCH_TIMING, 0 if ctxs else 1)
        if ctxs:
            x.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
        for kv in filter(None, os.environ.get("PT_BENCH_LEG_OPTS", "").split(",")):   # A/B of leg options
            k, _, val = kv.partition("=")
            x.set_option(int(k), int(val))
        x.resize_and_clear(W, H)
        ctxs.append(x)
    return ctxs, hip_streams, cam, int_bits, desc, i.size // 3


def leg_profile(key, which, device, steps):
    """--leg KEY --leg-camera ref|ff: only the timed frames of one scene leg
    at one camera, with the leg's own contexts and traversal grid (SCENE_LEGS)
    -- one warmup frame per context, then `steps` frames alternating between
    them -- for rocprofv3 (tools/profile_workload.sh, workloads *_leg): the
    counters then come from the configuration the leg times (VERDICT r05
    item 6).  Prints one line with the frame count the summary divides by."""
    import ptamd
    import scenes
    import torch
    entry = next(e for e in SCENE_LEGS if e[0] == key)
    _, scene_name, W, H, spp, depth, _, workload, s_ref, s_ff = entry
    nctx, grid = s_ref if which == "ref" else s_ff
    ctxs, hip_streams, cam, _, _, _ = leg_contexts(scene_name, W, H, depth, 3, device, nctx)
    camera = scenes.DEFAULT_CAMERA if which == "ref" else cam
    for x in ctxs:
        x.set_camera(camera)
        x.set_option(ptamd.PT_OPT_WF_GRID, grid)
        x.set_option(ptamd.PT_OPT_WF_TAIL, 0 if nctx > 1 else -1)
        x.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
    for x in ctxs:
        x.render(0, spp)
    torch.cuda.synchronize()
    walls = time_frames_pipelined(ctxs, spp, steps, groups=1)
    print(json.dumps({"leg": key, "camera": which, "workload": workload + ("_refcam" if which == "ref" else ""),
                      "contexts": nctx, "wf_grid_percent": grid, "frames": nctx + steps,
                      "ms_per_step": round(float(np.median(walls)), 3)}), flush=True)
    del ctxs
    torch.cuda.synchronize()
    for hs in hip_streams:
        hs.close()


def scene_leg(scene_name, W, H, spp, depth, sss, steps, device, workload, exhaustive_too=False, contexts=1,
              setup_ref=None, setup_ff=None):
    """One BASELINE config on one GPU (N = 1 only), at two cameras: BASELINE's
    (0,0,5) (Camera.cpp:7-9, Camera.h:34-36) leads -- its
    numbers are the leg's `value` and `roofline`, priced from the committed
    profile of `workload + "_refcam"` -- and the scene's frame-filling camera
    (load_scene) follows as `frame_filling_camera`, priced from `workload`.
    At each: the reference rays of a stats-mode frame, the walks of a
    counting frame, `steps` timed frames after one warmup frame per context.
    exhaustive_too: one more frame at the frame-filling camera with
    PT_OPT_WIDE 0 -- the threaded exhaustive walk, the reference's own
    traversal shape -- reported as `exhaustive_walk` (workload +
    "_exhaustive").  setup_ref / setup_ff: (contexts, grid %) at each camera
    (default (contexts, 100)); with more than one context the timed frames
    alternate between them (own stream, accumulation and wavefront buffers
    each), frames in flight; ms per frame is then the wall time of a run over
    its frames, and the contexts' frames are checked bitwise equal."""
    import ptamd
    import scenes
    import torch
    t_setup = time.perf_counter()
    setup_ref = setup_ref or (contexts, 100)
    setup_ff = setup_ff or (contexts, 100)
    contexts = max(setup_ref[0], setup_ff[0])
    ctxs, hip_streams, cam, int_bits, desc, ntri = leg_contexts(scene_name, W, H, depth, sss, device, contexts)
    r = ctxs[0]
    setup_s = time.perf_counter() - t_setup
    base = desc.split(", camera")[0]

    def measure(camera, cam_desc, wl, setup):
        nctx, grid = setup
        use = ctxs[:nctx]
        for x in use:
            x.set_camera(camera)
            x.set_option(ptamd.PT_OPT_WF_GRID, grid)
            # with frames in flight the other frames fill a frame's last ray
            # rounds: the tail kernel (PT_OPT_WF_TAIL, for a frame alone) then
            # costs more than it saves
            x.set_option(ptamd.PT_OPT_WF_TAIL, 0 if nctx > 1 else -1)
        t0 = time.perf_counter()
        r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 0)
        ref, traced = reference_and_traced_counts(r, spp)
        counts_s = time.perf_counter() - t0
        r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
        for x in use:
            x.render(0, spp)
        torch.cuda.synchronize()
        if nctx > 1:
            walls = time_frames_pipelined(use, spp, steps)
            kt = walls
            want = r.read_accum().view(np.uint32).copy()
            for x in use[1:]:
                if not np.array_equal(x.read_accum().view(np.uint32), want):
                    raise SystemExit(f"bench: {scene_name} leg: the pipelined contexts' frames differ")
        else:
            walls, kt = time_frames(r, spp, steps)
            want = r.read_accum().view(np.uint32).copy()
        # The timed frame against the same frame through the exhaustive
        # threaded walk (PT_OPT_WIDE 0: every box a ray passes, in the
        # reference's visit order, raytrace_comp.comp:159-204), bit for bit;
        # the GPU tests pin that walk to the oracle's rows (test_gpu_configs).
        for x in use[1:]:
            x.synchronize()
        r.set_option(ptamd.PT_OPT_WIDE, 0)
        r.reset_launch_times()
        t_ex = time.perf_counter()
        r.render(0, spp)
        r.synchronize()
        ex_s = time.perf_counter() - t_ex
        ex_kt = r.launch_times_ms()
        r.set_option(ptamd.PT_OPT_WIDE, 1)
        ex_bad = int(np.count_nonzero(r.read_accum().view(np.uint32) != want))
        exhaustive = {"ms": ex_s * 1e3, "kernel_ms": float(np.sum(ex_kt)) if ex_kt.size else float("nan"),
                      "launches": int(ex_kt.size), "mismatched_floats": ex_bad}
        dt = float(np.median(walls)) * 1e-3   # the median frame (min/max beside it)
        kernel_ms = float(np.median(kt)) if kt.size else float("nan")
        alg = algorithmic_bytes({"nodes": ref[1], "leaf_tests": ref[2], "samples": ref[3]})
        cfg = {"workload": f"{base}, {cam_desc} {W}x{H} {spp}spp {depth} bounces {sss} sss", "triangles": int(ntri),
               "int_bits_nodes": bool(int_bits), "rays_per_frame": int(ref[0]), "profile_workload": wl}
        add_traced(cfg, traced, dt)
        kname = KERNEL_NAMES.get(r.last_kernel(), "?")
        out = {"metric": "Mrays/s (reference-equivalent traceRay calls)", "value": round(ref[0] / dt / 1e6, 3),
               "unit": "Mrays/s", "ms_per_step": round(dt * 1e3, 2), "steps": steps, "warmup": 1,
               "ms_per_frame": spread(walls), "kernel_ms_per_frame": spread(kt) if kt.size else None,
               "kernel": kname, "config": cfg,
               "roofline": roofline_block(leg_traffic(wl), kernel_ms, alg, kname, kernel_ms, kernel_ms,
                                          int(kt.size),
                                          f"median wall ms per frame of runs of {steps} frames alternating over "
                                          f"{nctx} contexts (frames overlap)" if nctx > 1 else
                                          "median kernel_ms (HIP events around each frame's launches on the render "
                                          "stream)"),
               "contexts": nctx, "wf_grid_percent": grid, "counting_passes_s": round(counts_s, 2),
               "verified_vs_exhaustive": ex_bad == 0,
               "verified_vs_exhaustive_basis": f"the last timed frame (context 0) bitwise against the same frame "
                                               f"through the exhaustive walk (PT_OPT_WIDE 0): {ex_bad} floats differ"}
        price_leg(out, wl, traced, kernel_ms, alg, ref[0])
        prof = leg_traffic(wl)
        if prof is not None and prof[1].get("bench_line"):
            # the committed counters' run against the timed one: same
            # contexts and grid
            bl = prof[1]["bench_line"]
            out["profile_parallelism"] = {"contexts": bl.get("contexts"), "grid": bl.get("wf_grid_percent")}
            out["profile_parallelism_matches"] = (bl.get("contexts") == nctx and bl.get("wf_grid_percent") == grid)
        return out, ref, alg, exhaustive

    out, _, _, _ = measure(scenes.DEFAULT_CAMERA, "camera (0,0,5) fov 60 (BASELINE.md §3)", workload + "_refcam",
                           setup_ref)
    out["setup_s"] = round(setup_s, 2)
    ff, ref_ff, alg_ff, ex = measure(cam, "camera" + desc.split(", camera")[1], workload, setup_ff)
    ff["note"] = "the scene's frame-filling camera (more pixels on geometry than BASELINE's (0,0,5))"
    if exhaustive_too:
        # the exhaustive frame measure() just checked against the timed frame
        dt0 = ex["ms"] * 1e-3
        k0 = ex["kernel_ms"]
        name0 = "wavefront pipeline, threaded exhaustive walk (PT_OPT_WIDE 0), per frame"
        ff["exhaustive_walk"] = {
            "value": round(ref_ff[0] / dt0 / 1e6, 3), "unit": "Mrays/s", "ms_per_step": round(dt0 * 1e3, 2),
            "steps": 1, "note": "the reference's traversal shape (every box a ray passes, visit order kept); "
                                "compared bitwise with the timed frame (verified_vs_exhaustive)",
            "roofline": roofline_block(profiled_traffic(workload + "_exhaustive"), k0, alg_ff, name0, k0, k0,
                                       ex["launches"], "kernel_ms (HIP events around the frame's launches)")}
    out["frame_filling_camera"] = ff
    del r, ctxs
    torch.cuda.synchronize()
    for hs in hip_streams:
        hs.close()
    return out


# the BASELINE configs that name a multi-GPU run (configs[3]: the Sylveon
# substitute at 4K 16 spp D8 tile-split with an RCCL accumulation reduce;
# configs[4]: the 10M cloud's 8-GPU report), timed at N > 1 beside the box
# runs of 9 / 12 frames: with three in flight, the first frame of a run
# starts alone and the last drains alone
DIST_SCENE_LEGS = (("config4", "sphere", 3840, 2160, 16, 8, 9),
                   ("config5", "synthetic:10000000", 1920, 1080, 8, 4, 12))


def dist_scene_leg(dist, backend, device, world, rank, scene_name, W, H, spp, depth, sss, steps, contexts=3,
                   grid=33):
    """One multi-GPU BASELINE config at N = world: every rank renders its
    screen tiles (pt_set_partition) of the frame with the kernel the library
    picks for its share, then one RCCL SUM reduce of the accumulation buffer
    to rank 0 (owned pixels +0-cleared, the others -0: the sum is bit-exact,
    DESIGN §5).  Frames alternate between `contexts` contexts per rank (own
    stream, accumulation and wavefront buffers each), so a frame's ray rounds
    run beside the previous frames' drains and reduces (a 1/8 tile share of
    config 4 takes 64.0 ms per frame alone, 56.7 ms two in flight, 55.3
    three; config 5 21.9 / 18.7 / 17.7; tools/scene_streams.py).  Timed: runs of `steps` frames after one warmup
    frame per context, each run bracketed by barrier + synchronize on every
    rank; ms per frame = the run's wall time over its frames, the maximum over
    ranks, median over runs.  Rank 0 then renders the whole frame alone and
    checks every context's last reduced frame against it bit for bit.
    Returns the leg's dict on rank 0 (None elsewhere), or {"error": ...} if
    any rank failed its setup (then no rank runs a collective of the leg)."""
    import ptamd
    import scenes
    import torch
    t_setup = time.perf_counter()
    dev = torch.device("cuda", device)
    coll = dev if backend == "nccl" else "cpu"
    err = ""
    ctxs = []   # (renderer, stream, accumulation buffer)
    hip_streams = []
    try:
        scene, _, int_bits, desc = load_scene(scene_name)
        # BASELINE's camera for every config (Camera.cpp:7-9)
        cam = scenes.DEFAULT_CAMERA
        desc = desc.split(", camera")[0] + ", camera (0,0,5) fov 60"
        v, i, n, _, _ = scene.arrays()
        del scene
        for _ in range(contexts):
            r = ptamd.Renderer(device)
            r.upload_scene(v, i, n, int_bits=int_bits)
            r.upload_lights(scenes.REFERENCE_LIGHT)
            r.set_camera(cam)
            r.set_params(depth, sss)
            hs = HipStream(device)   # released with the leg (HipStream)
            hip_streams.append(hs)
            stream = hs.torch
            r.set_stream(hs.handle)
            r.set_partition(world, rank)
            if contexts > 1:
                # frames in flight fill each other's last ray rounds: no tail
                # kernel (1/8 sphere share, three contexts: 8.89 -> 7.37 ms per
                # frame without it; 10M cloud 17.81 -> 17.62)
                r.set_option(ptamd.PT_OPT_WF_TAIL, 0)
            # each context's traversal on 1/C of the GPU (PT_OPT_WF_GRID):
            # emulated 1/8 shares at (0,0,5), three contexts, 100 -> 33 %:
            # config 4 23.7 -> 20.7 ms, config 5 5.07 -> 4.22 (profiles/r05d)
            r.set_option(ptamd.PT_OPT_WF_GRID, grid)
            if ctxs:
                r.set_option(ptamd.PT_OPT_LAUNCH_TIMING, 0)
            frame = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
            r.bind_accum(frame.data_ptr(), W, H)
            ctxs.append((r, stream, frame))
        ntri = i.size // 3
        del v, i, n
    except Exception as e:   # noqa: BLE001 -- reported in the line, never a hang of the other ranks
        err = f"rank {rank}: {type(e).__name__}: {e}"
    ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=coll)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) == 0:
        if err:
            print(f"bench: {scene_name} leg: {err}", file=sys.stderr, flush=True)
        return {"error": err or "another rank failed its setup"} if rank == 0 else None
    setup_s = time.perf_counter() - t_setup
    r0 = ctxs[0][0]

    def reduce_sum(r, stream, t):
        if backend == "nccl":
            with torch.cuda.stream(stream):   # the reduce follows this context's render
                dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)
        else:
            # gloo (the one-GPU rehearsal): the render is waited for on its own
            # stream, then the buffer is staged through the host by the
            # renderer (pt_read_accum), with no torch stream in between
            c = torch.from_numpy(r.read_accum())
            dist.reduce(c, dst=0, op=dist.ReduceOp.SUM)
            if rank == 0:
                with torch.cuda.stream(stream):
                    t.view(-1).copy_(c.to(dev))
                stream.synchronize()

    def allreduce(vals, op):
        t = torch.tensor(np.asarray(vals, np.float64), dtype=torch.float64, device=coll)
        dist.all_reduce(t, op=op)
        return t.cpu().numpy()

    # reference traceRay calls of the whole frame: each rank counts its share
    log(f"{scene_name} leg: counting passes")
    t0 = time.perf_counter()
    mine, traced = reference_and_traced_counts(r0, spp)
    ref = allreduce(mine, dist.ReduceOp.SUM)
    traced = dict(zip(TRACED_KEYS, (int(x) for x in allreduce([traced[k] for k in TRACED_KEYS],
                                                                 dist.ReduceOp.SUM))))
    counts_s = time.perf_counter() - t0

    def frame_once(j):
        r, stream, frame = ctxs[j % len(ctxs)]
        r.clear()                       # +0 owned, -0 elsewhere
        r.render(0, spp)
        reduce_sum(r, stream, frame)

    log(f"{scene_name} leg: warmup")
    for j in range(len(ctxs)):   # warmup
        frame_once(j)
    torch.cuda.synchronize(dev)
    log(f"{scene_name} leg: timed runs")
    walls = []
    for _ in range(3):
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for j in range(steps):
            frame_once(j)
        torch.cuda.synchronize(dev)
        dist.barrier()
        walls.append((time.perf_counter() - t0) * 1e3 / steps)
    wmax = allreduce(walls, dist.ReduceOp.MAX)
    wmin = allreduce(walls, dist.ReduceOp.MIN)
    out = None
    if rank == 0:
        log(f"{scene_name} leg: whole-frame check on rank 0")
        got = [f.cpu().numpy().reshape(-1).copy() for _, _, f in ctxs]
        # the whole frame on this GPU alone, same context and kernels
        r0.set_partition(1, 0)
        r0.clear()
        r0.render(0, spp)
        r0.synchronize()
        want = r0.read_accum().view(np.uint32)
        same = all(bool(np.array_equal(g.view(np.uint32), want)) for g in got)
        out = dist_leg_record(f"{desc} {W}x{H} {spp}spp {depth} bounces {sss} sss", ntri, int_bits, ref, traced,
                              world, len(ctxs), grid, steps, np.asarray(wmax), np.asarray(wmin), same,
                              KERNEL_NAMES.get(r0.last_kernel(), "?"), setup_s, counts_s)
    del r0, ctxs
    torch.cuda.synchronize(dev)
    for hs in hip_streams:
        hs.close()
    dist.barrier()
    return out


def dist_leg_record(workload, ntri, int_bits, ref, traced, world, nctx, grid, steps, wmax, wmin, same, kernel,
                    setup_s, counts_s):
    """The full record of one N > 1 scene leg (rank 0): ms per frame = the
    slowest rank's run wall time over its frames, median over runs."""
    dt = float(np.median(wmax)) * 1e-3
    cfg = {"workload": workload, "triangles": int(ntri), "int_bits_nodes": bool(int_bits),
           "rays_per_frame": int(ref[0]),
           "parallelism": f"tiles{world}-reduce (RCCL SUM of the accumulation buffer to rank 0); "
                          f"{nctx} frames in flight per rank, traversal grid {grid} %"}
    add_traced(cfg, traced, dt)
    return {"metric": "Mrays/s (reference-equivalent traceRay calls)", "value": round(ref[0] / dt / 1e6, 3),
            "unit": "Mrays/s", "n_gpus": world, "ms_per_step": round(dt * 1e3, 2), "steps": steps,
            "warmup": nctx, "ms_per_frame": spread(wmax),
            "rank_ms_per_frame": {"slowest": spread(wmax), "fastest": spread(wmin),
                                  "note": "per run of frames, the slowest and the fastest rank"},
            "kernel": kernel, "config": cfg, "contexts": nctx, "verified_bitwise_vs_single_gpu": bool(same),
            "setup_s": round(setup_s, 2), "counting_passes_s": round(counts_s, 2)}


def group_record(devs, setup_s, state, ms_peer, ms_staged, peer):
    """The pt_create_multi leg's header: devices, the peer-store probe's
    outcome (pt_group_check) and the exchange in force (pt_group_info)."""
    return {"devices": devs, "setup_s": round(setup_s, 2),
            "peer_store_check": {"state": {-1: "not run", 0: "matched", 1: "mismatch: staged copies in force",
                                           2: "probe failed: staged copies in force", -2: "armed"}.get(state, state),
                                 "probe_ms_peer": round(ms_peer, 3), "probe_ms_staged": round(ms_staged, 3)},
            "peer_stores_in_force": bool(peer),
            "note": "one process, one thread, pt_create_multi over the devices (the reference's single-thread "
                    "drop-in); frames whole from batch 0, enqueued back to back, synchronized at the end"}


def group_exchange_record(peer, dt, steps, rays_per_frame, same):
    return {"exchange": "peer stores into the first device's frame" if peer else
            "staged packed copies (pt_tiles_pack, hipMemcpyPeerAsync, pt_tiles_unpack)",
            "ms_per_step": round(dt * 1e3, 4), "steps": steps,
            "value": None if rays_per_frame != rays_per_frame else round(rays_per_frame / dt / 1e6, 3),
            "unit": "Mrays/s", "verified_bitwise_vs_single_gpu": bool(same)}


class IpcFrames:
    """--collective ipc: the root's frame buffers shared with every rank
    through HIP IPC (one hipMalloc of `nbuf` W x H float4 frames on the
    root, its handle broadcast, hipIpcOpenMemHandle elsewhere).  Each rank's
    contexts bind a buffer as their accumulation buffer and render their own
    tiles straight into it -- over xGMI on a multi-GPU node, as the one-process
    group's peer stores do -- so no gather, no assembly and no RCCL call per
    frame.  Disjoint tiles: the ranks never write the same pixel."""

    def __init__(self, dist, rank, W, H, nbuf, coll_dev):
        import ctypes
        import torch
        self.hip = hip_runtime()
        self.rank, self.nbuf = rank, nbuf
        self.frame_bytes = W * H * 16
        self.ptr = None
        self.opened = False
        class IpcHandle(ctypes.Structure):   # hipIpcMemHandle_t: 64 opaque bytes, passed by value to open
            _fields_ = [("reserved", ctypes.c_ubyte * 64)]
        err = 0
        handle = IpcHandle()
        if rank == 0:
            p = ctypes.c_void_p()
            err = self.hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(self.frame_bytes * nbuf))
            if err == 0:
                self.ptr = p.value
                err = self.hip.hipIpcGetMemHandle(ctypes.byref(handle), ctypes.c_void_p(self.ptr))
        t = torch.tensor([err] + list(handle.reserved), dtype=torch.int32, device=coll_dev)
        dist.broadcast(t, 0)
        if int(t[0].item()) != 0:
            raise RuntimeError(f"hipMalloc / hipIpcGetMemHandle on the root: error {int(t[0].item())}")
        if rank != 0:
            h = IpcHandle()
            h.reserved[:] = [int(x) & 0xff for x in t[1:].tolist()]
            p = ctypes.c_void_p()
            # hipIpcMemLazyEnablePeerAccess = 1
            self.hip.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), IpcHandle, ctypes.c_uint]
            e = self.hip.hipIpcOpenMemHandle(ctypes.byref(p), h, ctypes.c_uint(1))
            if e != 0:
                raise RuntimeError(f"hipIpcOpenMemHandle: error {e}")
            self.ptr = p.value
            self.opened = True

    def buffer(self, j):
        return self.ptr + j * self.frame_bytes

    def read(self, j):
        """Root: frame buffer j on the host."""
        import ctypes
        out = np.empty(self.frame_bytes // 4, np.float32)
        e = self.hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(self.buffer(j)),
                               ctypes.c_size_t(self.frame_bytes), ctypes.c_int(2))   # hipMemcpyDeviceToHost
        if e != 0:
            raise RuntimeError(f"hipMemcpy: error {e}")
        return out

    def close(self):
        import ctypes
        if self.opened:
            self.hip.hipIpcCloseMemHandle(ctypes.c_void_p(self.ptr))
        elif self.rank == 0 and self.ptr:
            self.hip.hipFree(ctypes.c_void_p(self.ptr))
        self.ptr = None


def setup_ipc(dist, device, world, rank, W, H, spp, v, i, n, int_bits, light, cam, depth, sss, opts, coll_dev,
              want=None, nbuf=3):
    """--collective ipc: `nbuf` contexts per rank (own stream each), context j
    bound to the root's frame buffer j (IpcFrames) with this rank's tiles of a
    world-way partition; frame k renders on context k % nbuf.  Self-check
    first: every rank renders one frame per buffer, then the root compares
    each buffer with `want` (its single-GPU frame) bit for bit.  Every rank
    returns the same answer: the contexts, or None (the caller then runs the
    gather), with the reason."""
    import ptamd
    import torch
    ok, why = 1, ""
    frames = ctxs = None
    streams = []
    try:
        frames = IpcFrames(dist, rank, W, H, nbuf, coll_dev)
        ctxs = []
        for j in range(nbuf):
            x = ptamd.Renderer(device)
            x.upload_scene(v, i, n, int_bits=int_bits)
            x.upload_lights(light)
            x.set_camera(cam)
            x.set_params(depth, sss)
            x.set_partition(world, rank)
            x.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
            x.set_option(ptamd.PT_OPT_LAUNCH_TIMING, 0)
            for kv in opts:
                k, _, val = kv.partition("=")
                x.set_option(int(k), int(val))
            hs = HipStream(device)
            streams.append(hs)
            x.set_stream(hs.handle)
            x.bind_accum(frames.buffer(j), W, H)
            ctxs.append(x)
        for x in ctxs:
            x.render(0, spp)
        torch.cuda.synchronize(device)
    except Exception as e:   # noqa: BLE001 -- every rank must reach the vote below
        ok, why = 0, f"rank {rank}: {type(e).__name__}: {e}"
    dist.barrier()   # every rank's frames are complete before the root reads them
    if ok and rank == 0 and want is not None:
        for j in range(nbuf):
            got = frames.read(j).view(np.uint32)
            if not np.array_equal(got, want.view(np.uint32)):
                ok, why = 0, f"ipc self-check: buffer {j} differs from the single-GPU frame in " \
                             f"{int(np.count_nonzero(got != want.view(np.uint32)))} floats"
                break
    flag = torch.tensor([ok], dtype=torch.int32, device=coll_dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 0:
        if why:
            print(f"bench: ipc exchange unavailable, gathering instead: {why}", file=sys.stderr, flush=True)
        torch.cuda.synchronize(device)
        if ctxs:
            for x in ctxs:
                x.close()
        for hs in streams:
            hs.close()
        if frames is not None and rank != 0:   # mappings dropped before the root frees the buffers
            frames.close()
        dist.barrier()
        if frames is not None and rank == 0:
            frames.close()
        return None, why or "another rank failed its ipc setup or self-check"
    return {"frames": frames, "ctxs": ctxs, "streams": streams}, ""


def setup_native(r, dist, dev, world, rank, W, H, spp, v, i, n, int_bits, light, cam, depth, sss, coll_dev,
                 n_streams=2):
    """RCCL communicator for pt_dist_run and a 6-frame bitwise self-check on
    the root against a single-GPU render; None (every rank) if anything
    fails, so the caller keeps the Python step.  coll_dev: where the
    torch.distributed process group wants its tensors (the GPU for nccl, the
    host for gloo -- the one-GPU rehearsal with PT_RCCL_LIB)."""
    import ptamd
    import torch
    ok = 1
    uid = bytes(128)
    if rank == 0:
        try:
            uid = ptamd.Renderer.dist_unique_id()
        except ptamd.PTError as e:
            print(f"bench: native step loop unavailable: {e}", file=sys.stderr, flush=True)
            ok = 0
    t = torch.tensor([ok] + list(uid), dtype=torch.uint8, device=coll_dev)
    dist.broadcast(t, 0)   # the id, and whether rank 0 could make one
    if int(t[0].item()) == 0:
        return None
    frames = None
    try:
        r.dist_init(bytes(t[1:].cpu().tolist()), world, rank)
        frames = torch.full((3, H, W, 4), float("nan"), dtype=torch.float32, device=dev)   # up to 3 in flight
        # six frames on the streams the timed run uses; the last three land in
        # buffers 0-2 and are each checked below
        r.dist_run(spp, 6, frames.data_ptr(), 3, n_streams=n_streams)
        try:
            r.dist_wait(30000)   # a hung gather must not hang the bench: abort and fall back
        except ptamd.PTError:
            r.dist_abort()
            raise
        r.synchronize()
        if rank == 0:
            ref = ptamd.Renderer(dev.index)
            ref.upload_scene(v, i, n, int_bits=int_bits)
            ref.upload_lights(light)
            ref.set_camera(cam)
            ref.set_params(depth, sss)
            ref.resize_and_clear(W, H)
            ref.render(0, spp)
            want = ref.read_accum().view(np.uint32)
            del ref
            for f in range(3):
                if not np.array_equal(frames[f].cpu().numpy().reshape(-1).view(np.uint32), want):
                    ok = 0
    except ptamd.PTError as e:
        print(f"bench: native step loop unavailable: {e}", file=sys.stderr, flush=True)
        ok = 0
    flag = torch.tensor([ok], dtype=torch.int32, device=coll_dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 0:
        print("bench: native step loop failed its self-check; using the Python step", file=sys.stderr, flush=True)
        try:
            r.dist_abort()
        except ptamd.PTError:
            pass
        return None
    return {"frames": frames, "outs": list(frames)}


class _StreamWork:
    """Stand-in for an async collective's Work in the rank emulation: wait()
    orders the caller's current stream after what `stream` had queued when
    the work was issued (as ProcessGroupNCCL's Work.wait does)."""

    def __init__(self, stream):
        import torch
        self.ev = torch.cuda.Event()
        self.ev.record(stream)

    def wait(self):
        import torch
        torch.cuda.current_stream().wait_event(self.ev)


# --- the printed line -------------------------------------------------------
# The driver parses the LAST stdout line and reads only its tail: round 5's
# 21.5-KB line could not be parsed (BENCH_r05.parsed null).  The full record
# (per-leg spreads, gather-pattern tables, calibration, basis prose) goes to a
# detail file that the line names; the line keeps the measured numbers, one
# compact entry per leg, and every verification flag, within LINE_MAX_BYTES.
LINE_MAX_BYTES = 6144
DETAIL_DEFAULT = os.path.join("gpurun_out", "bench_detail.json")


def _r(x, nd):
    return None if x is None else round(float(x), nd)


def compact_roofline(rf):
    """bound/achieved/peak/unit/frac/traffic/source of a full roofline block,
    plus the HBM fraction beside a non-HBM primary bound."""
    if not rf:
        return None
    out = {k: rf.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic")}
    out["source"] = rf.get("source") or rf.get("traffic_source")
    if isinstance(rf.get("hbm"), dict):
        out["hbm_frac"] = rf["hbm"].get("frac")
    if "frac_raw_counters" in rf:
        out["frac_raw_counters"] = rf["frac_raw_counters"]
    return out


def _leg_camera(leg):
    """value / ms / primary frac / verification of one camera of an N=1 leg."""
    rf = leg.get("roofline") or {}
    out = {"value": leg.get("value"), "ms_per_step": leg.get("ms_per_step"), "bound": rf.get("bound"),
           "frac": rf.get("frac"), "contexts": leg.get("contexts"), "grid": leg.get("wf_grid_percent"),
           "verified": leg.get("verified_vs_exhaustive")}
    if leg.get("roofline_gather"):
        out["gather_frac"] = leg["roofline_gather"].get("frac")
    if leg.get("roofline_valu"):
        out["valu_frac"] = leg["roofline_valu"].get("frac")
    if leg.get("profile_parallelism_matches") is not None:
        out["profile_matches_timed"] = leg["profile_parallelism_matches"]
    return out


def compact_leg(leg):
    """One compact entry per leg: N=1 legs at BASELINE's camera with the
    frame-filling camera nested (`ff`); N>1 legs value/ms/verified/error."""
    if leg is None:
        return None
    if "error" in leg and "value" not in leg:
        return {"error": str(leg["error"])[:300]}
    if "n_gpus" in leg:   # a distributed leg
        out = {"value": leg.get("value"), "ms_per_step": leg.get("ms_per_step"), "n_gpus": leg.get("n_gpus"),
               "verified": leg.get("verified_bitwise_vs_single_gpu")}
        if leg.get("error"):
            out["error"] = str(leg["error"])[:300]
        return out
    out = _leg_camera(leg)
    ff = leg.get("frame_filling_camera")
    if ff:
        out["ff"] = _leg_camera(ff)
        ex = ff.get("exhaustive_walk")
        if ex:
            out["ff"]["exhaustive_ms"] = ex.get("ms_per_step")
    return out


def compact_group(g):
    """The pt_create_multi leg: devices, the peer-store probe's state, each
    exchange's time and bitwise check, or a short error."""
    if g is None:
        return None
    out = {"devices": g.get("devices")}
    if g.get("skipped"):
        out["skipped"] = str(g["skipped"])[:200]
    if g.get("error"):
        out["error"] = str(g["error"])[:300]
    if isinstance(g.get("peer_store_check"), dict):
        out["peer_store_check"] = g["peer_store_check"].get("state")
    if "peer_stores_in_force" in g:
        out["peer_stores_in_force"] = g["peer_stores_in_force"]
    for k in ("exchange0", "exchange1"):
        if isinstance(g.get(k), dict):
            e = g[k]
            out[k] = {"ms_per_step": e.get("ms_per_step"), "value": e.get("value"),
                      "verified": e.get("verified_bitwise_vs_single_gpu"),
                      "peer": e.get("exchange", "").startswith("peer")}
    return out


def _finite(x):
    """NaN / inf -> None, recursively: the line is strict JSON."""
    if isinstance(x, dict):
        return {k: _finite(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_finite(v) for v in x]
    if isinstance(x, float) and (x != x or x in (float("inf"), float("-inf"))):
        return None
    return x


def compact_line(full, detail_path=None):
    """The line bench.py prints: the driver's contract keys, a short config,
    the headline roofline and CPU baseline, every verification, one compact
    entry per leg.  Raises if it would exceed LINE_MAX_BYTES."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "verified_vs_oracle", "verified_bitwise_vs_single_gpu",
            "emulated_ranks", "bench_wall_s", "dry_run", "ranks_seen", "launcher", "backend_requested")
    out = {k: full[k] for k in keep if k in full}
    c = full.get("config", {})
    out["config"] = {k: c[k] for k in ("workload", "parallelism", "kernel_options", "step_loop", "rays_per_frame",
                                       "rays_traced", "msamples_per_s", "rays_traced_per_s_M", "rccl_comm_ranks",
                                       "partition_slots", "lane_schedule", "exchange_fallback")
                     if c.get(k) is not None}
    out["roofline"] = compact_roofline(full.get("roofline"))
    cb = full.get("cpu_baseline")
    if cb:
        out["cpu_baseline"] = {"value": cb.get("value"), "unit": cb.get("unit"), "cores": cb.get("cores"),
                               "kind": cb.get("kind"), "sample": str(cb.get("sample", ""))[:160]}
        if isinstance(cb.get("single_thread"), dict):
            out["cpu_baseline"]["single_thread_value"] = cb["single_thread"].get("value")
    sc = full.get("single_context")
    if sc:
        out["single_context"] = {k: sc.get(k) for k in ("value", "ms_per_step", "steps", "kernel_ms", "schedule",
                                                        "verified_vs_oracle", "error") if sc.get(k) is not None}
    if full.get("primary_cull_off"):
        out["primary_cull_off_ms"] = full["primary_cull_off"].get("ms_per_step")
    if full.get("configs"):
        out["configs"] = {k: compact_leg(v) for k, v in full["configs"].items()}
    if "group_leg" in full:
        out["group_leg"] = compact_group(full["group_leg"])
    if detail_path:
        out["detail_file"] = detail_path
    out = _finite(out)
    s = json.dumps(out, separators=(",", ":"), allow_nan=False)
    if len(s) > LINE_MAX_BYTES:
        raise ValueError(f"bench line is {len(s)} bytes (> {LINE_MAX_BYTES})")
    return out


def emit_line(full, detail_path=None):
    """Write the full record to `detail_path` (and one stderr line), print the
    compact line on stdout as the process's last stdout line."""
    detail_path = detail_path if detail_path is not None else os.environ.get("PT_BENCH_DETAIL", DETAIL_DEFAULT)
    written = None
    if detail_path:
        try:
            d = os.path.dirname(detail_path)
            if d:
                os.makedirs(d, exist_ok=True)
            with open(detail_path, "w") as f:
                json.dump(full, f, indent=1)
            written = detail_path
        except OSError as e:
            log(f"detail file {detail_path} not written: {e}")
    print("bench detail: " + json.dumps(full), file=sys.stderr, flush=True)
    line = compact_line(full, written)
    print(json.dumps(line, separators=(",", ":"), allow_nan=False), flush=True)
    return line


def log(msg):
    """A progress line on stderr, tagged with the rank and the seconds since
    start: a run that stops shows where."""
    print(f"bench[{os.environ.get('RANK', '0')}] {time.perf_counter() - T_START:7.1f}s: {msg}", file=sys.stderr,
          flush=True)


def spawn_ranks(n):
    """`python bench.py --gpus N` without a launcher: start N ranks with
    torch.distributed.run as a child process (one process per GPU, rendezvous
    on 127.0.0.1) and return its exit code.  Called before anything touches
    the GPU; the parent never execs (a GPU-initialised process must not be
    replaced) and only waits.  Rank 0's JSON line reaches the parent's stdout
    unchanged."""
    import subprocess
    env = dict(os.environ, PT_BENCH_SPAWNED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--standalone",
           "--local-addr", "127.0.0.1", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"--gpus {n} without a launcher: spawning {n} ranks ({' '.join(cmd[1:6])} ...)")
    return subprocess.call(cmd, env=env)


def dry_run(world, rank, backend):
    """--dry-run: the process-group plumbing of an N-rank run without a GPU
    call -- every rank joins the group and contributes its rank; rank 0
    prints one JSON line (the CPU test of the launcher)."""
    import datetime
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=float(os.environ.get("PT_BENCH_PG_TIMEOUT_S", "60"))))
    if int(os.environ.get("PT_BENCH_DRY_STALL_RANK", "-1")) == rank:
        # test hook: this rank never reaches the collective (a stuck rank);
        # the others must fail within the process-group timeout, not hang
        time.sleep(3600)
    t = torch.zeros(world, dtype=torch.int64)
    t[rank] = rank + 1
    dist.all_reduce(t)
    if rank == 0:
        full = dry_run_record(world, [int(x) - 1 for x in t.tolist()],
                              "spawned" if os.environ.get("PT_BENCH_SPAWNED") == "1" else "external", backend)
        emit_line(full, os.environ.get("PT_BENCH_DETAIL", ""))
    dist.barrier()
    dist.destroy_process_group()


def dry_run_record(world, ranks_seen, launcher, backend):
    """The full record of an N-rank run with every N > 1 field filled --
    the distributed legs and the pt_create_multi leg built by the same
    helpers as a real run, with placeholder numbers, long worst-case error
    strings on one leg -- so the printed line's size and keys are checked
    without a GPU (tests/test_multi.py)."""
    nan = float("nan")
    traced = {k: 10 ** 9 for k in TRACED_KEYS}
    ref = np.array([3.06e7, 9.7e7, 1.7e7, 1.6e7])
    legs = {}
    for key, scene_name, lw, lh, lspp, ldepth, lsteps in DIST_SCENE_LEGS:
        legs[key] = dist_leg_record(f"{scene_name} (0,0,5) {lw}x{lh} {lspp}spp {ldepth} bounces 3 sss", 10 ** 7, True,
                                    ref, traced, world, 3, 33, lsteps, np.array([1.0, 1.1, 1.2]),
                                    np.array([0.9, 1.0, 1.1]), True, KERNEL_NAMES[3], 1.0, 1.0)
    legs["config_failed"] = {"error": "rank 7: PTError: " + "x" * 1000}
    group = group_record(list(range(world)), 1.0, 0, 0.1, 0.2, True)
    for exch in (0, 1):
        group[f"exchange{exch}"] = group_exchange_record(exch == 0, 1e-4, 20, 3.06e7, True)
    line = {"metric": "Mrays/s at 1920x1080x8spp, box.obj BVH", "value": None, "unit": "Mrays/s", "n_gpus": world,
            "steps": 0, "warmup": 0, "ms_per_step": None, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f32",
            "data": "DRY RUN (no GPU call): the process-group plumbing and the line's shape",
            "dry_run": True, "ranks_seen": ranks_seen, "launcher": launcher, "backend_requested": backend,
            "config": {"workload": "box.obj, camera (0,0,5) fov 60 1920x1080 8spp 4 bounces 3 sss",
                       "parallelism": f"tiles{world}-sparse-gather", "kernel_options": [],
                       "step_loop": "native (pt_dist_run, RCCL from C++)", "rays_per_frame": 30586335,
                       "rccl_comm_ranks": world, "partition_slots": [12] + [16] * (world - 1)},
            "roofline": roofline_block(None, nan, 0, KERNEL_NAMES[1], nan, nan, 0, "dry run"),
            "verified_bitwise_vs_single_gpu": None, "configs": legs, "group_leg": group}
    return line


def group_leg(devices, v, i, n, int_bits, light, cam, W, H, spp, depth, sss, steps, rays_per_frame):
    """The drop-in multi-GPU path (SURVEY §8b create(device_ordinals[], n)):
    one process, one context over `devices` (pt_create_multi), driven as the
    reference drives its one GPU from one thread (VulkanRenderer.cpp:643-647,
    mainLoop VulkanRayTracer.cpp:717-865).  Each step is pt_render of the
    whole frame from batch 0; the members' tiles reach the frame on
    devices[0] by peer stores (PT_OPT_GROUP_EXCHANGE 0, after the context's
    own probe check on distinct devices, pt_group_check) and then by staged
    packed copies (exchange 1).  Both are timed over `steps` frames and the
    last frame of each is checked bit for bit against a one-GPU render of the
    same frame on devices[0]."""
    import ptamd
    ref = ptamd.Renderer(devices[0])
    ref.upload_scene(v, i, n, int_bits=int_bits)
    ref.upload_lights(light)
    ref.set_camera(cam)
    ref.set_params(depth, sss)
    ref.resize_and_clear(W, H)
    ref.render(0, spp)
    want = ref.read_accum().view(np.uint32).copy()
    ref.close()
    t_setup = time.perf_counter()
    g = ptamd.Renderer(devices=list(devices))
    g.upload_scene(v, i, n, int_bits=int_bits)
    g.upload_lights(light)
    g.set_camera(cam)
    g.set_params(depth, sss)
    g.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
    g.resize_and_clear(W, H)
    setup_s = time.perf_counter() - t_setup
    g.render(0, spp)   # runs the peer-store probe check first when members span devices
    g.synchronize()
    state, ms_peer, ms_staged = g.group_check()
    devs, peer = g.group_info()
    out = group_record(devs, setup_s, state, ms_peer, ms_staged, peer)
    for exch in (0, 1):
        g.set_option(ptamd.PT_OPT_GROUP_EXCHANGE, exch)
        for _ in range(3):
            g.render(0, spp)
        g.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            g.render(0, spp)
        g.synchronize()
        dt = (time.perf_counter() - t0) / steps
        got = g.read_accum().view(np.uint32)
        same = bool(np.array_equal(got, want))
        _, peer = g.group_info()
        out[f"exchange{exch}"] = group_exchange_record(peer, dt, steps, rays_per_frame, same)
    g.close()
    return out


def group_leg_child(gdevs, args, rays_per_frame):
    """The group leg in a child process of its own (`bench.py --group-only`):
    it opens every device of the group, and whatever happens there -- the
    first cross-device peer stores this build runs -- this run's line is
    still printed.  Returns the child's JSON (or an error record)."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--group-only", "--group-devices", gdevs,
           "--steps", str(max(args.steps, 20)), "--scene", args.scene, "--width", str(args.width),
           "--height", str(args.height), "--spp", str(args.spp), "--depth", str(args.depth), "--sss", str(args.sss),
           "--camera", args.camera, "--group-rays", repr(float(rays_per_frame))]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    log(f"group leg: pt_create_multi over devices {gdevs} (child process)")
    try:
        res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    except subprocess.TimeoutExpired:
        return {"error": "group leg: timed out after 300 s"}
    sys.stderr.write(res.stderr[-4000:])
    lines = [x for x in res.stdout.splitlines() if x.startswith("{")]
    if res.returncode != 0 or not lines:
        return {"error": f"group leg: exit {res.returncode}", "stderr_tail": res.stderr[-1500:]}
    return json.loads(lines[-1])


def group_only(args):
    """--group-only: the one-process pt_create_multi leg alone (run by
    group_leg_child)."""
    import torch  # noqa: F401 -- torch's HIP runtime first (libptamd binds to it)
    import ptamd
    import scenes
    devices = [int(x) for x in args.group_devices.split(",")]
    visible = torch.cuda.device_count()
    if max(devices) >= visible:
        print(json.dumps({"devices": devices, "skipped": f"{visible} devices visible to the group leg's process"}),
              flush=True)
        return
    scene, cam, int_bits, _ = load_scene(args.scene)
    if args.camera == "reference":
        cam = scenes.DEFAULT_CAMERA
    v, i, n, _, _ = scene.arrays()
    try:
        out = group_leg(devices, v, i, n, int_bits, scenes.REFERENCE_LIGHT, cam, args.width, args.height, args.spp,
                        args.depth, args.sss, args.steps, args.group_rays)
    except ptamd.PTError as e:
        out = {"devices": devices, "error": str(e)}
    print(json.dumps(out), flush=True)


def main():
    if os.environ.get("PT_BENCH_TRACEBACK_AFTER_S"):
        # diagnostics of a hung run: every thread's stack to stderr after N s
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["PT_BENCH_TRACEBACK_AFTER_S"]), exit=False)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # a box frame takes ~0.3 ms on one GPU and ~0.05 ms per step on 8: 200
    # steps keep the barrier/synchronize bracket a small part of the region
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--scene", default="box")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--depth", type=int, default=4, help="MAX_DEPTH (reference 4; SURVEY §8d config 4 uses 8)")
    ap.add_argument("--sss", type=int, default=3, help="SSS_MAX_BOUNCES (reference 3)")
    ap.add_argument("--collective", choices=["gather", "reduce", "ipc"], default="gather",
                    help="N > 1 frame exchange: sparse RCCL gather of the live items (default), SUM reduce of "
                         "whole frames, or ipc: every rank renders its tiles straight into the root's frame "
                         "buffers (HIP IPC), falling back to the gather if its self-check fails")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", type=int, choices=[0, 1], default=None, nargs="?", const=1,
                    help="N>1: compare the assembled frame with a 1-GPU render (default on at N > 1)")
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VAL",
                    help="pt_set_option before timing (A/B of output-invariant kernel options)")
    ap.add_argument("--assemble", type=int, choices=[0, 1, 2], default=2,
                    help="N>1 gather: 2 = render_packed assembling frame k-2 in frame k's launch, "
                         "1 = render_packed + assembly launch, 0 = render + pack + assembly launches")
    ap.add_argument("--streams", type=int, choices=[1, 2, 3, 4], default=None,
                    help="gather path: frames alternate between this many streams, so one frame's tail "
                         "overlaps the next frame's head (default 2 for N > 1, 1 at N = 1)")
    ap.add_argument("--timing-every", type=int, default=None,
                    help="HIP event pair around every k-th launch (default 4 on one stream, where a pair "
                         "costs ~7 us of device time per launch, 1 on two streams, where it is hidden)")
    ap.add_argument("--root-slots", type=int, default=-1,
                    help="gather path: partition slots of the root out of 16 per other rank "
                         "(-1 auto: the root gives up the share its frame assembly costs; 0: equal shares)")
    ap.add_argument("--packed", action="store_true", help="N=1: run the gather path (render_packed + assembly)")
    ap.add_argument("--compare-no-cull", type=int, choices=[0, 1], default=None,
                    help="also time the same frames with primary-ray culling off, before the warmup (reported "
                         "as primary_cull_off); default on for the box headline")
    ap.add_argument("--no-cull-min-ms", type=float, default=40.0,
                    help="the culling-off frames run for at least this long (and at least --steps frames)")
    ap.add_argument("--no-scene-legs", action="store_true",
                    help="skip the scene legs (`configs` in the JSON line): configs 3, 4 and 5 on one GPU at "
                         "N=1, configs 4 and 5 across the N GPUs at N>1")
    ap.add_argument("--camera", choices=["scene", "reference"], default="scene",
                    help="reference: BASELINE's camera (0,0,5) fov 60 for any --scene (profile runs of the legs)")
    ap.add_argument("--group-devices", default=None,
                    help="comma-separated ordinals: also run the one-process pt_create_multi leg over them "
                         "(default at N > 1: the N devices, from rank 0; 'none' skips it)")
    ap.add_argument("--leg", default=None, help="only the timed frames of one scene leg (config3/4/5; profiling)")
    ap.add_argument("--leg-camera", choices=["ref", "ff"], default="ref",
                    help="--leg: BASELINE's camera (0,0,5) or the scene's frame-filling one")
    ap.add_argument("--group-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--group-rays", type=float, default=float("nan"), help=argparse.SUPPRESS)
    ap.add_argument("--dry-run", action="store_true",
                    help="the process-group plumbing only (no GPU): every rank joins, rank 0 prints a line")
    ap.add_argument("--profile-run", action="store_true",
                    help="only the warmup and timed frames (no stats/counting passes, legs or CPU baseline): "
                         "the command tools/profile_workload.sh runs under rocprofv3")
    args = ap.parse_args()
    W, H, SPP = args.width, args.height, args.spp
    if args.streams is None:
        # N = 1: the box's 0.27-ms frames alternate between two contexts
        # (double-buffered accumulation, one stream each), so frame k+1 starts
        # while frame k's last workgroups drain (-5.4 %, tools/box_streams.py);
        # the long large-scene frames gain nothing from it and keep one.
        # N > 1: three frames in flight on the native loop's three render
        # streams (emulated root step, DESIGN Appendix A.2: N=8 0.0417 ->
        # 0.0369 ms, N=4 0.0685 -> 0.0648, N=2 0.119 -> 0.1145 against two)
        multi = (int(os.environ.get("WORLD_SIZE", "1")) > 1
                 or int(os.environ.get("PT_BENCH_EMULATE_RANKS", "1")) > 1)
        args.streams = 3 if multi and not args.packed else 2 if (multi or args.packed or args.scene == "box") else 1
    if args.collective == "reduce":
        args.streams = 1   # the reduce path runs on one stream
    if args.timing_every is None:
        args.timing_every = 4 if args.streams == 1 else 1
        # the library keeps the last 512 event pairs
        args.timing_every = max(args.timing_every, -(-args.steps // 400))
    elif args.timing_every > 0:
        args.timing_every = max(args.timing_every, -(-args.steps // 400))
    DEPTH, SSS = args.depth, args.sss

    if args.group_only:
        group_only(args)
        return
    if args.leg:
        import torch  # noqa: F401 -- torch's HIP runtime first (libptamd binds to it)
        leg_profile(args.leg, args.leg_camera, int(os.environ.get("PT_BENCH_DEVICE", "0")), args.steps)
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: N ranks of this same command under torch.distributed.run
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        dry_run(world, rank, os.environ.get("PT_BENCH_BACKEND", "nccl"))
        return
    # PT_BENCH_EMULATE_RANKS=N (1-GPU box only): rank 0's step of an N-GPU
    # gather run -- its tile share, pack, the root's unpack of N slots -- with
    # the collective replaced by a device copy of its own slot.  A rehearsal of
    # the root's critical path, never a multi-GPU result (the line says so).
    emu = int(os.environ.get("PT_BENCH_EMULATE_RANKS", "1"))
    if args.verify is None:
        args.verify = int(world > 1)
    if emu > 1 and world != 1:
        raise SystemExit("PT_BENCH_EMULATE_RANKS needs a 1-process run")
    if emu > 1 and (args.collective != "gather" or args.verify):
        raise SystemExit("PT_BENCH_EMULATE_RANKS rehearses the gather path without --verify")
    # Rehearsal knobs for a 1-GPU box: every rank on one device, gloo staged on the host.
    device = int(os.environ.get("PT_BENCH_DEVICE", local))
    backend = os.environ.get("PT_BENCH_BACKEND", "nccl")

    import torch   # load torch's HIP runtime first so libptamd binds to the same one
    import ptamd
    import scenes

    dist = None
    dev = torch.device("cuda", device)
    torch.cuda.set_device(dev)
    # PT_BENCH_FORCE_DIST=1 runs the N>1 step (pack, RCCL gather, unpack) at
    # N=1 too: measures the exchange's own overhead on a 1-GPU box
    if world > 1 or os.environ.get("PT_BENCH_FORCE_DIST") == "1":
        import torch.distributed as dist
        kw = {}
        if backend == "nccl":
            # the gather's RCCL kernels run on a high-priority stream: they get
            # CUs as soon as render workgroups retire, instead of queueing
            # behind two frames' worth of them
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            kw = {"device_id": dev, "pg_options": opts}
        # a collective that one rank never reaches fails after this long
        # instead of holding every other rank for the default 30 minutes
        # (VERDICT r04 item 1); sized above the longest rank-0-only stretch
        # (a whole-frame check render of config 4, the group leg)
        import datetime
        kw["timeout"] = datetime.timedelta(seconds=float(os.environ.get("PT_BENCH_PG_TIMEOUT_S", "900")))
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
        log(f"process group up ({backend}, {world} ranks)")

    def allreduce_max(t):
        if backend == "nccl":
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return t
        c = t.cpu()
        dist.all_reduce(c, op=dist.ReduceOp.MAX)
        return c

    scene, cam, int_bits, scene_desc = load_scene(args.scene)
    if args.camera == "reference":
        cam = scenes.DEFAULT_CAMERA
        scene_desc = scene_desc.split(", camera")[0] + ", camera (0,0,5) fov 60"
    v, i, n, _, _ = scene.arrays()
    light = scenes.REFERENCE_LIGHT
    r = ptamd.Renderer(device)
    r.upload_scene(v, i, n, int_bits=int_bits)
    r.upload_lights(light)
    r.set_camera(cam)
    r.set_params(DEPTH, SSS)
    # PT_BENCH_EMULATE_RANK=r: emulate rank r's step instead of the root's
    # (its share, no assembly) -- to compare the ranks' loads
    emu_rank = int(os.environ.get("PT_BENCH_EMULATE_RANK", "0")) if emu > 1 else rank
    r.set_partition(max(world, emu), emu_rank)
    r.set_option(ptamd.PT_OPT_LAUNCH_TIMING, args.timing_every)
    # One explicit stream for the renderer and every torch op/collective: the
    # legacy default stream has handle 0, which pt_set_stream reads as "the
    # context's own stream", so it cannot be shared by handle.
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    r.set_stream(stream.cuda_stream)   # order with torch's collectives
    r.resize_and_clear(W, H)

    # Root share (gather path).  The root also assembles every gathered frame
    # (a full-frame write, ~7.5 us at 1080p), so with equal shares it is the
    # slowest rank.  Partition slots: 16 per rank, the root 16*(1 - 0.75*N*A/T1)
    # where A = the root's assembly as a launch of its own, T1 = a full frame
    # on one GPU, both timed here on the root (untimed setup); every rank
    # applies the root's choice.  0.75: the part of a standalone assembly
    # launch the pipelined step pays (emulated root vs other ranks at N=2/4/8:
    # 12 of 16 slots balance them at N=8, 15 at N=2).
    nparts = max(world, emu)
    slots = None
    if nparts > 1 and args.collective == "gather" and args.root_slots != 0:
        s0 = args.root_slots
        if s0 < 0:
            s0 = 16
            if rank == 0:
                def time_ms(fn, reps=5):
                    t_first = time.perf_counter()
                    fn()
                    torch.cuda.synchronize(dev)
                    if time.perf_counter() - t_first > 0.02:
                        reps = 1   # a large scene: one more frame is enough
                    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    ev0.record()
                    for _ in range(reps):
                        fn()
                    ev1.record()
                    ev1.synchronize()
                    return ev0.elapsed_time(ev1) / reps
                r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
                r.set_partition(1, 0)
                t1 = time_ms(lambda: r.render(0, SPP))
                r.set_partition(nparts, 0)
                r.render(0, SPP)
                cnt = max(r.items_live(k)[0] for k in range(nparts)) * r.items_live(0)[1] * 4
                src = torch.zeros((nparts, max(cnt, 4)), dtype=torch.float32, device=dev)
                frm = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
                t_asm = time_ms(lambda: r.items_unpack_all(src.data_ptr(), src.shape[1], frm.data_ptr()))
                del src, frm
                r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 0)
                s0 = int(min(16, max(1, round(16 * (1.0 - 0.75 * nparts * t_asm / t1)))))
                print(f"bench: root share: full frame {t1:.4f} ms, assembly {t_asm:.4f} ms -> "
                      f"{s0} of 16 slots", file=sys.stderr, flush=True)
            if dist is not None:
                t = torch.tensor([s0], dtype=torch.int32, device=dev if backend == "nccl" else "cpu")
                dist.broadcast(t, 0)
                s0 = int(t.item())
        slots = [s0] + [16] * (nparts - 1)
        r.set_partition(nparts, emu_rank, slots)
        r.resize_and_clear(W, H)

    def sum_ranks(x):
        if dist is None:
            return np.asarray(x, np.float64)
        t = torch.tensor(np.asarray(x, np.float64), dtype=torch.float64, device=dev)
        if backend == "nccl":
            dist.all_reduce(t)
        else:
            t = t.cpu()
            dist.all_reduce(t)
        return t.cpu().numpy()

    if args.profile_run:
        mine = np.zeros(4)
        rays_per_frame = float("nan")
        traced = None
    else:
        # Stats pass (untimed): the reference's exact traversal counts for one frame.
        mine, traced = reference_and_traced_counts(r, SPP)
        counts = sum_ranks(mine)
        rays_per_frame = float(counts[0])
        traced = dict(zip(TRACED_KEYS, (int(x) for x in sum_ranks([traced[k] for k in TRACED_KEYS]))))
    # output-invariant kernel options apply to the timed frames (the stats
    # pass above always runs the path-recursive kernel)
    for kv in args.opt:
        k, _, val = kv.partition("=")
        r.set_option(int(k), int(val))

    # --- the step ---------------------------------------------------------
    r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
    pending = []
    finish = None
    ingest = None   # the emulated root's stand-in for the gather's receive traffic
    nparts = max(world, emu)
    ctxs = [r]   # N = 1: the contexts frames alternate between
    mixed_learn = []   # frames each N = 1 context took to measure its lane schedule
    ipc, ipc_error = None, None
    if dist is not None and args.collective == "ipc":
        # the root's single-GPU frame for the exchange's self-check
        want_ref = None
        if rank == 0:
            ref = ptamd.Renderer(device)
            ref.upload_scene(v, i, n, int_bits=int_bits)
            ref.upload_lights(light)
            ref.set_camera(cam)
            ref.set_params(DEPTH, SSS)
            ref.resize_and_clear(W, H)
            ref.render(0, SPP)
            want_ref = ref.read_accum().copy()
            ref.close()
        log("ipc exchange: setup and self-check")
        ipc, ipc_error = setup_ipc(dist, device, world, rank, W, H, SPP, v, i, n, int_bits, light, cam, DEPTH, SSS,
                                   args.opt, dev if backend == "nccl" else "cpu", want=want_ref)
        if ipc is None:
            args.collective = "gather"   # equal shares: the root-slot rule is the gather's, not applied here
    box_streams = []   # HipStreams of the N = 1 contexts, closed before the legs
    if dist is None and emu == 1 and not args.packed:
        # args.streams > 1: frames alternate between that many contexts, each
        # with its own stream and accumulation buffer (the same scene, camera
        # and options), so consecutive frames overlap on the GPU; every frame
        # is still a whole frame from batch 0 (bitwise checked after timing)
        if args.streams > 1:
            # with frames in flight the tail of a frame is filled by the next
            # one, so the work granularity that shortened it no longer pays:
            # one lane per pixel (its samples in order, no colour hand-off
            # between lanes) and items in scan order, unless --opt says
            # otherwise.  Box 1080p8 on two contexts: 0.2466 -> 0.2176 ms
            # (one frame at a time the same options take 0.351 against 0.263)
            given = {int(kv.partition("=")[0]) for kv in args.opt}
            for key, val in ((ptamd.PT_OPT_SAMPLE_LANES, 1), (ptamd.PT_OPT_ITEM_ORDER, 0)):
                if key not in given:
                    args.opt.append(f"{key}={val}")
                    r.set_option(key, val)
            if os.environ.get("PT_BENCH_R_HIPSTREAM", "1") == "1":
                # every context on a stream of the same (least) priority:
                # one queue pool, a queue each, none favoured by the dispatcher
                rs = HipStream(device)
                box_streams.append(rs)
                r.set_stream(rs.handle)
        for _ in range(args.streams - 1):
            x = ptamd.Renderer(device)
            x.upload_scene(v, i, n, int_bits=int_bits)
            x.upload_lights(light)
            x.set_camera(cam)
            x.set_params(DEPTH, SSS)
            x.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
            x.set_option(ptamd.PT_OPT_LAUNCH_TIMING, 0)
            for kv in args.opt:
                k, _, val = kv.partition("=")
                x.set_option(int(k), int(val))
            xs = HipStream(device)
            box_streams.append(xs)
            x.set_stream(xs.handle)
            x.resize_and_clear(W, H)
            ctxs.append(x)
        # the library's measured lane schedule (PT_OPT_MIXED_LANES -1: whole
        # tiles longest first on measured costs), frame by frame until it is
        # in force on every context; untimed, before the clocks' pre-warm
        # (which turns culling off and leaves the schedule alone)
        for c in ctxs:
            k = 0
            while k < 60 and c.mixed_info()[0] != 2:
                c.render(0, SPP)
                c.synchronize()
                k += 1
            mixed_learn.append(k)
        state1 = {"k": 0}

        def step():
            c = ctxs[state1["k"] % len(ctxs)]
            state1["k"] += 1
            c.render(0, SPP)
    elif ipc is not None:
        # every rank renders its tiles of frame k straight into the root's
        # frame buffer k % 3 (IpcFrames): nothing to exchange or assemble
        state_ipc = {"k": 0}

        def step():
            c = ipc["ctxs"][state_ipc["k"] % len(ipc["ctxs"])]
            state_ipc["k"] += 1
            c.render(0, SPP)
    elif args.collective == "reduce":
        r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 0)
        frame = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
        r.bind_accum(frame.data_ptr(), W, H)

        def step():
            r.clear()                   # +0 owned, -0 elsewhere: the SUM is bit-exact
            r.render(0, SPP)
            if backend == "nccl":
                dist.reduce(frame, dst=0, op=dist.ReduceOp.SUM)
            else:
                c = frame.cpu()
                dist.reduce(c, dst=0, op=dist.ReduceOp.SUM)
                if rank == 0:
                    frame.copy_(c)
    else:
        # Sparse gather: each rank ships only its live items (tile parts that
        # can hold a live pixel under primary culling); the root rebuilds the
        # culled ones.  Every rank derives every rank's item count itself.
        # --assemble 2 (default): frame k's render launch (pt_render_packed)
        # also assembles frame k-2 on the root, whose gather ran during frame
        # k-1's render -- one launch per step; 1: render_packed, then a
        # separate assembly launch; 0: render + pack + assembly launches.
        r.render(0, SPP)
        per = r.items_live(0)[1]
        slot = max(r.items_live(k)[0] for k in range(nparts)) * per * 4
        slot = max(slot, 4)
        root = rank == 0 and emu_rank == 0
        # Frame k uses buffer set k % nbuf and, under --assemble 2, assembles
        # frame k - depth from that same set in its own launch; depth = streams,
        # so frame k waits only for frame k - depth's gather (which follows
        # frame k - depth's launch on frame k's stream) and `streams` frames
        # are in flight.  The gather of frame k then overwrites the receive
        # set after the launch that read it, on the same stream.
        depth = max(2, args.streams) if args.assemble == 2 else 1   # frames in flight before assembly
        nbuf = max(2, depth)
        send = [torch.zeros(slot, dtype=torch.float32, device=dev) for _ in range(nbuf)]
        recv_all = [torch.zeros((nparts, slot), dtype=torch.float32, device=dev) for _ in range(nbuf)] if root else None
        recv = [[recv_all[b][k] for k in range(nparts)] for b in range(nbuf)] if root else None
        outs = [torch.empty((H, W, 4), dtype=torch.float32, device=dev) for _ in range(args.streams)] if root else None
        out = outs[0] if root else None
        streams = [stream] + [torch.cuda.Stream(dev) for _ in range(args.streams - 1)]
        state = {"k": 0, "written": set()}   # written: outs indices holding an assembled frame
        # Emulated root (PT_BENCH_EMULATE_RANKS): the other ranks' slots
        # still have to arrive.  A high-priority side stream copies N-1 whole
        # slots into the receive buffer after each render, in one copy as an
        # RCCL gather is one call (device to device: a read and a write of
        # them in this GPU's HBM, at least the write an RCCL receive costs),
        # and the frame's assembly waits for it.
        ingest = None
        if dist is None and emu > 1 and root:
            ingest = {"stream": torch.cuda.Stream(dev, priority=-1),
                      "src": torch.zeros((nparts - 1) * slot, dtype=torch.float32, device=dev),
                      "bytes": 4 * (nparts - 1) * slot}

        def finish(work, buf):   # separate assembly launch of one gathered frame
            if work is not None:
                work.wait()
            if root:
                r.items_unpack_all(recv_all[buf].data_ptr(), slot, out.data_ptr())
                state["written"].add(0)

        def step():
            buf = state["k"] % nbuf
            sid = state["k"] % len(streams)
            state["k"] += 1
            if len(streams) > 1:
                torch.cuda.set_stream(streams[sid])
                r.set_stream(streams[sid].cuda_stream)
            fused = None
            if len(pending) >= depth:
                work, pbuf = pending.pop(0)
                if args.assemble == 2:
                    if work is not None:
                        work.wait()   # gather of frame k-depth: ran during the frames since
                    if root:
                        fused = (recv_all[pbuf].data_ptr(), slot, outs[sid].data_ptr())
                        state["written"].add(sid)
                else:
                    finish(work, pbuf)
            # emulation: the root's own slot is written in place, no transfer
            dst = (recv[buf][0] if root else send[buf]) if dist is None else send[buf]
            if args.assemble == 0:
                r.render(0, SPP)
                r.items_pack(dst.data_ptr())
            elif fused is not None:
                r.render_packed(SPP, dst.data_ptr(), *fused)
            else:
                r.render_packed(SPP, dst.data_ptr())
            if dist is None and ingest is not None:
                side = ingest["stream"]
                side.wait_stream(streams[sid])
                with torch.cuda.stream(side):
                    recv_all[buf][1:].view(-1).copy_(ingest["src"])
                work = _StreamWork(side)
            elif dist is None:
                work = _StreamWork(streams[sid])
            elif backend == "nccl":
                work = dist.gather(send[buf], recv[buf] if root else None, dst=0, async_op=True)
            else:
                host = [torch.empty_like(x, device="cpu") for x in recv[buf]] if root else None
                dist.gather(send[buf].cpu(), host, dst=0)
                if root:
                    for x, h in zip(recv[buf], host):
                        x.copy_(h)
                work = None
            pending.append((work, buf))

    def drain():
        while pending:
            finish(*pending.pop(0))

    # Native step loop (pt_dist_*): the same pipelined sparse gather with the
    # RCCL send/recv issued from C++ -- no Python per frame.  Used for N > 1
    # over RCCL (and PT_BENCH_FORCE_DIST=1 at N = 1) unless PT_BENCH_NATIVE=0.
    # A 6-frame self-check against a single-GPU render runs first; if the root
    # finds any bit different, every rank falls back to the Python step.
    # With PT_RCCL_LIB (the one-GPU rehearsal's stand-in for RCCL's
    # point-to-point calls) it runs beside a gloo process group too.
    native = None
    if (dist is not None and (backend == "nccl" or os.environ.get("PT_RCCL_LIB")) and args.collective == "gather"
            and args.assemble == 2 and os.environ.get("PT_BENCH_NATIVE", "1") != "0"):
        native = setup_native(r, dist, dev, world, rank, W, H, SPP, v, i, n, int_bits, light, cam, DEPTH, SSS,
                              n_streams=min(3, args.streams), coll_dev=
                              dev if backend == "nccl" else "cpu")
        if native is not None:
            outs = native["outs"]
            out = outs[0]
    elif (dist is None and emu > 1 and emu_rank == 0 and args.collective == "gather" and args.assemble == 2
          and os.environ.get("PT_BENCH_NATIVE", "1") != "0"):
        # the emulated root on the native loop: a 1-rank communicator with the
        # N-way partition; the other ranks' slots arrive as a device copy of
        # the same bytes on the high-priority stream (pt_dist_init, emulation)
        r.dist_init(ptamd.Renderer.dist_unique_id(), 1, 0)
        frames_t = torch.empty((3, H, W, 4), dtype=torch.float32, device=dev)   # up to 3 frames in flight
        native = {"frames": frames_t, "outs": list(frames_t), "emulated": True}

    def run_steps(k):
        if native is not None:
            r.dist_run(SPP, k, native["frames"].data_ptr(), native["frames"].shape[0], n_streams=min(3, args.streams))
        else:
            for _ in range(k):
                step()

    if native is not None:
        # an event pair around every 4th launch: the native loop's host cost is
        # a handful of HIP calls per frame, and each event record is one of them
        args.timing_every = max(args.timing_every, 4)
        r.set_option(ptamd.PT_OPT_LAUNCH_TIMING, args.timing_every)
    # Primary-ray culling off, for reference beside the default: the same
    # frames (each rank's tile share at N > 1, rendered alone, no exchange)
    # with every pixel generated and traced, in runs of 16 frames until at
    # least --no-cull-min-ms have passed.  They run here, right before the
    # warmup, so the timed region starts on a GPU that has been busy: from
    # idle the GPU's clocks take ~15 ms of load to ramp up (tools/r04_step_probe.py,
    # profiles/r04/step_probe.log: 20-frame runs 0.2512 ms per frame after 300 ms
    # idle, 0.2374 -> 0.2302 -> 0.2216 in back-to-back runs, 0.2198 over 200).
    no_cull = None
    default_cfg = args.scene == "box" and (W, H, SPP, DEPTH, SSS) == (1920, 1080, 8, 4, 3)
    if args.compare_no_cull is None:
        args.compare_no_cull = int(default_cfg and not args.packed and not args.profile_run)
    if args.compare_no_cull:
        nc = ctxs if (dist is None and emu == 1 and not args.packed) else [r]
        for c in nc:
            c.set_option(ptamd.PT_OPT_PRIMARY_CULL, 0)
        for c in nc:
            c.render(0, SPP)
        torch.cuda.synchronize(dev)
        nc_frames = 0
        t1 = time.perf_counter()
        # bounded: at most 64 runs of 16 frames (a slow or shared GPU still
        # reaches the barrier below)
        for _ in range(64):
            for _ in range(16):
                nc[nc_frames % len(nc)].render(0, SPP)
                nc_frames += 1
            torch.cuda.synchronize(dev)
            dt_nc = time.perf_counter() - t1
            if nc_frames >= args.steps and dt_nc * 1e3 >= args.no_cull_min_ms:
                break
        for c in nc:
            c.set_option(ptamd.PT_OPT_PRIMARY_CULL, 1)
            c.render(0, SPP)   # the item layout the exchange follows is the last render's (culled)
        no_cull = {"ms_per_step": round(dt_nc / nc_frames * 1e3, 4), "frames": nc_frames,
                   "basis": "runs of 16 frames, synchronized after each run" +
                            (f"; rank {emu_rank}'s tile share alone, no exchange" if nparts > 1 else "")}
        if nparts == 1:
            no_cull["value"] = round(rays_per_frame * nc_frames / dt_nc / 1e6, 3)
        log(f"culling-off frames: {nc_frames} in {dt_nc * 1e3:.1f} ms")
    if dist is not None:
        dist.barrier()   # every rank leaves its own pre-warm before the first collective of the step
    log("warmup")
    run_steps(args.warmup)
    drain()
    if native is not None and native.get("emulated"):
        ingest = {"bytes": 4 * (emu - 1) * r.dist_slot_floats()}
    r.synchronize()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    r.reset_launch_times()
    log(f"timed region: {args.steps} steps")
    t0 = time.perf_counter()
    run_steps(args.steps)
    t_enq = time.perf_counter() - t0   # host time to issue the steps (no sync inside)
    drain()
    r.synchronize()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    kt = r.launch_times_ms()
    kernel_ms = float(np.mean(kt)) if kt.size else float("nan")
    # Launches on two streams overlap, so each one's event-measured duration
    # includes time shared with its neighbour: the per-launch figure the
    # roofline divides by is then the busy span over the launches.
    try:
        span_ms, n_launch = r.launch_span_ms()
    except ptamd.PTError:   # launch timing off (--opt 9=0)
        span_ms, n_launch = float("nan"), 1
    interval_ms = span_ms / max(n_launch, 1)
    if dist is not None:
        t = allreduce_max(torch.tensor([dt, kernel_ms, interval_ms], dtype=torch.float64, device=dev))
        dt, kernel_ms, interval_ms = float(t[0]), float(t[1]), float(t[2])
    roof_ms = interval_ms if args.streams > 1 else kernel_ms
    pipelined = len(ctxs) > 1
    # the last timed frame, checked bit for bit against the oracle's frame
    # (cpu_baseline renders the whole frame) before the line is printed
    timed_frame = None
    if world == 1 and emu == 1 and not args.packed and args.collective == "gather":
        timed_frame = ctxs[0].read_accum()
    if pipelined:
        # frames overlap across the contexts: the GPU time per frame is the
        # wall time per step (the launch events of one context span two frames)
        roof_ms = dt / args.steps * 1e3
        for c in ctxs[1:]:
            c.synchronize()
        want = ctxs[0].read_accum().view(np.uint32)
        for c in ctxs[1:]:
            if not np.array_equal(c.read_accum().view(np.uint32), want):
                raise SystemExit("bench: the pipelined contexts' frames differ")

    # The drop-in frame: ONE context at the library's
    # defaults -- no bench-only options, its own stream -- frames one after
    # another as the reference's mainLoop renders them (VulkanRayTracer.cpp:
    # 717-865), `steps` frames after a short warmup, the last one checked
    # against the oracle with the timed frame below.
    single = None
    single_frame = None
    if world == 1 and emu == 1 and not args.packed and args.collective == "gather" and not args.profile_run:
        try:
            sc = ptamd.Renderer(device)
            sc.upload_scene(v, i, n, int_bits=int_bits)
            sc.upload_lights(light)
            sc.set_camera(cam)
            sc.set_params(DEPTH, SSS)
            sc.resize_and_clear(W, H)
            # warmup: frame by frame until the library has measured this
            # frame's block costs and switched to its measured lane schedule
            # (PT_OPT_MIXED_LANES -1; a frame's cost copy lands while the next
            # one is enqueued, so it takes a few frames), then `warmup` more
            learn = 0
            while learn < 60 and sc.mixed_info()[0] != 2:
                sc.render(0, SPP)
                sc.synchronize()
                learn += 1
            # then at least 40 ms of frames back to back and `warmup` more: the
            # frame-by-frame waits above let the GPU's clocks drop
            t_w = time.perf_counter()
            while (time.perf_counter() - t_w) < 0.04:
                for _ in range(8):
                    sc.render(0, SPP)
                sc.synchronize()
            for _ in range(max(3, args.warmup)):
                sc.render(0, SPP)
            sc.synchronize()
            sched = sc.mixed_info()
            t_sc = time.perf_counter()
            for _ in range(args.steps):
                sc.render(0, SPP)
            sc.synchronize()
            dt_sc = time.perf_counter() - t_sc
            single_frame = sc.read_accum()
            single = {"ms_per_step": round(dt_sc / args.steps * 1e3, 4), "steps": args.steps,
                      "value": None if rays_per_frame != rays_per_frame else
                      round(rays_per_frame * args.steps / dt_sc / 1e6, 3),
                      "schedule": {0: "uniform lanes", 1: "static mix", 2: "measured"}.get(sched[0], sched[0]),
                      "frames_to_measure": learn,
                      "basis": "one context, library defaults (no pt_set_option), its own stream; "
                               "pt_render(0, spp) per frame back to back, synchronized at the end, after the frames "
                               "in which the library measured its lane schedule"}
            sc.close()
            log(f"single context: {single['ms_per_step']} ms per frame")
        except ptamd.PTError as e:
            single = {"error": str(e)[:300]}

    verified = None
    verify_error = None
    if args.verify and dist is not None and rank == 0:
        # the assembled frame must be bitwise the single-GPU frame
        ref = ptamd.Renderer(device)
        ref.upload_scene(v, i, n, int_bits=int_bits)
        ref.upload_lights(light)
        ref.set_camera(cam)
        ref.set_params(DEPTH, SSS)
        ref.resize_and_clear(W, H)
        ref.render(0, SPP)
        want = ref.read_accum()
        if ipc is not None:   # the root's frame buffers, every one holding a whole frame
            frames = [ipc["frames"].read(j) for j in range(ipc["frames"].nbuf)]
        else:
            # --assemble 2 assembles frames into outs[stream]; 0 and 1 into outs[0]
            frames = (outs if args.assemble == 2 else [out]) if args.collective == "gather" else [frame]
        if ipc is None and native is None and args.collective == "gather" and args.assemble == 2:
            # the Python step: only the buffers a fused or trailing assembly wrote
            frames = [outs[x] for x in sorted(state["written"])]
            assert frames, "bench --verify: no frame was assembled"
        for f in frames:
            got = f.cpu().numpy().reshape(-1) if ipc is None else f
            verified = bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
            if not verified:
                break
        if not verified:
            # recorded, and the run exits non-zero after the line: the other
            # ranks still reach every collective that follows
            bad = np.flatnonzero(got.view(np.uint32) != want.view(np.uint32))
            verify_error = (f"bench --verify: assembled frame differs from the single-GPU frame in {bad.size} "
                            f"floats; first at pixel {bad[0] // 4} ch {bad[0] % 4}: {got[bad[0]]} vs {want[bad[0]]}")

    box_kernel = KERNEL_NAMES.get(r.last_kernel(), "?")
    comm_ranks = None
    if native is not None and not native.get("emulated"):
        comm_ranks = r.dist_info()[0]   # what RCCL itself reports (ncclCommCount)
    dist_legs = None
    if dist is not None and default_cfg and not (args.no_scene_legs or args.profile_run):
        # configs 4 and 5 across the same N GPUs (every rank takes part)
        torch.cuda.synchronize(dev)
        dist.barrier()
        del r
        dist_legs = {}
        legs = DIST_SCENE_LEGS
        if os.environ.get("PT_BENCH_DIST_LEGS"):
            # smaller legs for the GPU tests: "key scene W H spp depth steps;..."
            legs = [tuple(f if k < 2 else int(f) for k, f in enumerate(e.split()))
                    for e in os.environ["PT_BENCH_DIST_LEGS"].split(";")]
        for key, scene_name, lw, lh, lspp, ldepth, lsteps in legs:
            log(f"{key} leg on {world} GPUs ({scene_name} {lw}x{lh} {lspp}spp D{ldepth})")
            dist_legs[key] = dist_scene_leg(dist, backend, device, world, rank, scene_name, lw, lh, lspp, ldepth,
                                            SSS, lsteps)

    # the one-process drop-in (pt_create_multi) over the N devices: rank 0
    # drives every GPU while the other ranks wait at the barrier
    group = None
    gdevs = args.group_devices
    if gdevs is None and world > 1 and default_cfg and not args.profile_run:
        gdevs = ",".join(str(k) for k in range(world))
    if gdevs is not None and gdevs != "none":
        if dist is not None:
            torch.cuda.synchronize(dev)
            dist.barrier()
        if rank == 0:
            group = group_leg_child(gdevs, args, rays_per_frame)
        if dist is not None:
            dist.barrier()

    if rank == 0:
        ms_per_step = dt / args.steps * 1e3
        value = rays_per_frame * args.steps / dt / 1e6
        value = None if value != value else value
        # per-GPU launch: rank 0's share of the algorithmic bytes over the slowest rank's kernel time
        own_bytes = algorithmic_bytes({"nodes": mine[1], "leaf_tests": mine[2], "samples": mine[3]})
        prof = profiled_traffic() if (world == 1 and emu == 1 and default_cfg and not args.packed) else None
        wl = f"{scene_desc} {W}x{H} {SPP}spp {DEPTH} bounces {SSS} sss"
        out_line = {
            "metric": "Mrays/s at 1920x1080x8spp, box.obj BVH" if default_cfg else f"Mrays/s, {wl}",
            "value": None if value is None else round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "host_issue_ms_per_step": round(t_enq / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference scene, camera and light; progressive sample batches 0-%d)" % (SPP - 1),
            "config": {"workload": wl, "width": W, "height": H, "spp": SPP, "max_depth": DEPTH,
                       "sss_bounces": SSS,
                       "partition_slots": slots,
                       "parallelism": (f"tiles{world}-" + ("ipc-peer-stores" if ipc is not None else
                                                           "sparse-gather" if args.collective == "gather" else "reduce"))
                       if world > 1 else ("single-packed" if args.packed else
                                          f"single, frames alternating over {len(ctxs)} contexts (one stream and "
                                          "accumulation buffer each)" if pipelined else "single"),
                       "streams": args.streams,
                       "kernel_options": list(args.opt),
                       "step_loop": ("python" if native is None else
                                     "native (pt_dist_run, RCCL from C++)" if not os.environ.get("PT_RCCL_LIB")
                                     else "native (pt_dist_run, PT_RCCL_LIB stand-in)"),
                       "rays_per_frame": None if rays_per_frame != rays_per_frame else int(rays_per_frame),
                       "primary_cull": True,
                       "msamples_per_s": round(W * H * SPP * args.steps / dt / 1e6, 3)},
            "roofline": roofline_block(prof, roof_ms, own_bytes, box_kernel,
                                       kernel_ms, interval_ms, int(kt.size),
                                       ("wall ms per frame (frames overlap across the N=1 contexts)" if pipelined
                                        else "launch_interval_ms (busy span / launches; launches overlap on "
                                        f"{args.streams} streams)" if args.streams > 1 else "kernel_ms")),
        }
        if traced is not None:
            add_traced(out_line["config"], traced, dt / args.steps)
        if mixed_learn:
            out_line["config"]["lane_schedule"] = {0: "uniform lanes", 1: "static mix", 2: "measured"}.get(
                ctxs[0].mixed_info()[0], "?") if ctxs else None
            out_line["config"]["frames_to_measure_schedule"] = mixed_learn
        if prof is not None and prof[1].get("sq_per_launch", {}).get("SQ_INSTS_VALU"):
            # the box frame is bound by vector-instruction issue, not HBM (its
            # scene lives in LDS): the primary roofline is VALU
            # wave-instructions per launch from the committed PMC profile over
            # the measured kernel time; the HBM roofline stays beside it
            valu = prof[1]["sq_per_launch"]["SQ_INSTS_VALU"]
            gi = valu / (roof_ms * 1e-3) / 1e9
            hbm = out_line["roofline"]
            out_line["roofline"] = {"bound": "valu_issue", "achieved": round(gi, 2), "peak": VALU_PEAK_GINST,
                                    "unit": "G wave-instr/s", "frac": round(gi / VALU_PEAK_GINST, 4),
                                    "traffic": hbm["traffic"], "valu_wave_instr_per_launch": int(valu),
                                    "source": prof[0], "kernel": hbm["kernel"], "kernel_ms": hbm["kernel_ms"],
                                    "time_basis": hbm["time_basis"],
                                    "peak_basis": "1024 SIMDs x 2.4 GHz / 2 cycles per wave64 f32 instruction",
                                    "hbm": {k: hbm[k] for k in ("achieved", "peak", "unit", "frac", "traffic",
                                                                "traffic_source", "effective_GBps")}}
        if emu > 1:
            out_line["metric"] = f"EMULATED (1 GPU, not a multi-GPU result): rank {emu_rank} of {emu}, " + out_line["metric"]
            out_line["emulated_ranks"] = emu
            if ingest is not None:
                out_line["emulated_ingest_bytes_per_step"] = int(ingest["bytes"])
            out_line["config"]["parallelism"] = f"emulated-tiles{emu}-sparse-gather"
        if no_cull is not None:
            out_line["primary_cull_off"] = no_cull
        if verified is not None:
            out_line["verified_bitwise_vs_single_gpu"] = verified
        oracle_mismatch = verify_error
        if world == 1 and emu == 1 and not args.no_cpu_baseline and not args.profile_run:
            out_line["cpu_baseline"], oracle_img = cpu_baseline(v, i, n, cam, light, W, H, SPP, DEPTH, SSS)
            if oracle_img is not None and timed_frame is not None:
                # raytrace_comp.comp:420-470 as restated by oracle/pt_oracle.cpp,
                # on the same scene, camera, light and batches as the timed frames
                bad = np.flatnonzero(timed_frame.view(np.uint32) != oracle_img.view(np.uint32))
                out_line["verified_vs_oracle"] = bool(bad.size == 0)
                out_line["verified_vs_oracle_basis"] = (
                    f"last timed frame of context 0 ({W}x{H}x{SPP}spp, kernel options {list(args.opt)}) bitwise "
                    "equal to the oracle's whole frame rendered by cpu_baseline")
                if bad.size:
                    oracle_mismatch = (f"bench: the timed frame differs from the oracle in {bad.size} floats; first at "
                                       f"pixel {bad[0] // 4} ch {bad[0] % 4}: {timed_frame[bad[0]]} vs "
                                       f"{oracle_img[bad[0]]}")
            if oracle_img is not None and single_frame is not None and single is not None:
                sbad = int(np.count_nonzero(single_frame.view(np.uint32) != oracle_img.view(np.uint32)))
                single["verified_vs_oracle"] = sbad == 0
                if sbad and oracle_mismatch is None:
                    oracle_mismatch = f"bench: the single-context frame differs from the oracle in {sbad} floats"
        if single is not None:
            out_line["single_context"] = single
        if dist_legs is not None:
            out_line["configs"] = dist_legs
        if group is not None:
            out_line["group_leg"] = group
        if comm_ranks is not None:
            out_line["config"]["rccl_comm_ranks"] = comm_ranks
        if ipc_error:
            out_line["config"]["exchange_fallback"] = ipc_error[:300]
        if world == 1 and emu == 1 and default_cfg and not (args.no_scene_legs or args.profile_run or args.packed):
            torch.cuda.synchronize(dev)
            del r
            for c in ctxs:   # the N = 1 contexts go before the legs make theirs
                c.close()
            ctxs.clear()
            for bs in box_streams:
                bs.close()
            out_line["configs"] = {}
            for key, scene_name, lw, lh, lspp, ldepth, steps, workload, s_ref, s_ff in SCENE_LEGS:
                log(f"{key} leg ({scene_name} {lw}x{lh} {lspp}spp D{ldepth})")
                out_line["configs"][key] = scene_leg(scene_name, lw, lh, lspp, ldepth, SSS, steps, device, workload,
                                                     exhaustive_too=key == "config5", setup_ref=s_ref,
                                                     setup_ff=s_ff)
            for key, leg in out_line["configs"].items():
                for cam_leg in (leg, leg.get("frame_filling_camera") or {}):
                    if cam_leg.get("verified_vs_exhaustive") is False and oracle_mismatch is None:
                        oracle_mismatch = f"bench: {key}: {cam_leg.get('verified_vs_exhaustive_basis')}"
        out_line["bench_wall_s"] = round(time.perf_counter() - T_START, 1)
        emit_line(out_line)
        if oracle_mismatch is not None:
            print(oracle_mismatch, file=sys.stderr, flush=True)
    else:
        oracle_mismatch = None
    if ipc is not None:   # ranks drop their mappings of the root's buffers, then the root frees them
        torch.cuda.synchronize(dev)
        for x in ipc["ctxs"]:
            x.close()
        for hs in ipc["streams"]:
            hs.close()
        if rank != 0:
            ipc["frames"].close()
        dist.barrier()
        if rank == 0:
            ipc["frames"].close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if oracle_mismatch is not None:
        sys.exit(1)   # after the last collective: the other ranks are not left waiting


if __name__ == "__main__":
    main()
