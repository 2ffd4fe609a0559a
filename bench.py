#!/usr/bin/env python3
"""Benchmark: Mrays/s of the path-tracing pixel kernel on box.obj at
1920x1080, 8 spp, 4 bounces (BASELINE.json configs[1]), 1..N GPUs.

A step = one frame: clear the accumulation buffer, run the 8 sample batches
(one fused launch, bit-identical to 8 progressive 1-spp dispatches) and, for
N > 1, combine the ranks' screen tiles on rank 0 with one RCCL reduction.
Mrays/s counts the reference's traceRay invocations (all kinds: light
pre-pass, primary/bounce, shadow, SSS, SSS-shadow), measured by a stats-mode
pass of the same frame before the timed region.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU).  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "discovering-path-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
W, H, SPP, DEPTH, SSS = 1920, 1080, 8, 4, 3


def algorithmic_bytes(st):
    """32 B per BVH node visited + 48 B per leaf triangle test
    (12 B indices + 36 B vertices) under the reference's exhaustive traversal,
    + 32 B accumulation read-modify-write per pixel-sample."""
    return 32 * st["nodes"] + 48 * st["leaf_tests"] + 32 * st["samples"]


def profiled_traffic():
    """HBM bytes per launch of the current kernel source from the newest
    committed rocprofv3 PMC summary (tools/gpu_profile.sh ->
    tools/summarize_profile.py): FETCH_SIZE (x2, gfx950) + WRITE_SIZE.
    None if no summary was taken of this exact pt_device.hip."""
    import glob
    import hashlib
    src = os.path.join(ROOT, "discovering-path-tracer_amd", "csrc", "pt_device.hip")
    h = hashlib.sha1(open(src, "rb").read()).hexdigest()
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json"))):
        try:
            d = json.load(open(p))
        except ValueError:
            continue
        if d.get("pt_device_hip_sha1") == h and "hbm_bytes_per_launch" in d:
            best = (os.path.relpath(p, ROOT), d["hbm_bytes_per_launch"]["total"])
    return best


def cpu_baseline(v, i, n, cam, light):
    """The oracle (scalar C++ restatement of raytrace_comp.comp) on this host,
    all cores, on a bounded sample: every 8th row of the same frame."""
    import oracle_lib
    threads = min(16, os.cpu_count() or 1)
    stride = 1
    oracle_lib.render(v, i, n.reshape(-1), cam, light, 64, 64, n_batches=1, nthreads=threads)   # warm
    t0 = time.perf_counter()
    _, st = oracle_lib.render(v, i, n.reshape(-1), cam, light, W, H, n_batches=SPP, max_depth=DEPTH,
                              sss_bounces=SSS, row_stride=stride, row_phase=0, nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": round(float(st[0]) / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"the full {W}x{H}x{SPP}spp box frame (rows y%{stride}==0, {H // stride} rows, "
                      f"{int(st[0])} rays, {dt:.2f} s, {threads} std::threads)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch   # load torch's HIP runtime first so libptamd shares it
    import ptamd
    import scenes

    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))

    scene = ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh()
    v, i, n, _, _ = scene.arrays()
    cam, light = scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT
    r = ptamd.Renderer(local)
    r.upload_scene(v, i, n)
    r.upload_lights(light)
    r.set_camera(cam)
    r.set_params(DEPTH, SSS)
    r.set_partition(world, rank)
    frame = None
    if world > 1:
        # torch owns the accumulation buffer so RCCL can reduce it in place;
        # the kernel runs on torch's current stream, ordering it with the collective.
        frame = torch.empty((H, W, 4), dtype=torch.float32, device=f"cuda:{local}")
        r.bind_accum(frame.data_ptr(), W, H)
        r.set_stream(torch.cuda.current_stream().cuda_stream)
    else:
        r.resize_and_clear(W, H)

    # Stats pass (untimed): the reference's exact traversal counts for one frame.
    r.set_stats_mode(True)
    r.reset_stats()
    r.clear()
    r.render(0, SPP)
    st = r.stats()
    r.set_stats_mode(False)
    counts = np.array([st["rays"], st["nodes"], st["leaf_tests"], st["samples"]], np.float64)
    if dist is not None:
        t = torch.tensor(counts, dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t)
        counts = t.cpu().numpy()
    rays_per_frame = float(counts[0])
    tot = {"nodes": counts[1], "leaf_tests": counts[2], "samples": counts[3]}

    def step():
        r.clear()
        r.render(0, SPP)
        if dist is not None:
            dist.reduce(frame, dst=0, op=dist.ReduceOp.SUM)

    for _ in range(args.warmup):
        step()
    r.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    r.reset_launch_times()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    r.synchronize()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    kt = r.launch_times_ms()
    kernel_ms = float(np.mean(kt)) if kt.size else float("nan")
    if dist is not None:
        t = torch.tensor([kernel_ms], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        kernel_ms = float(t.item())

    if rank == 0:
        ms_per_step = dt / args.steps * 1e3
        value = rays_per_frame * args.steps / dt / 1e6
        # per-launch algorithmic bytes of one rank's share (the kernel is per-GPU)
        bytes_per_launch = algorithmic_bytes(tot) / world
        achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
        prof = profiled_traffic() if world == 1 else None
        out = {
            "metric": "Mrays/s at 1920x1080x8spp, box.obj BVH",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (scenes/box.obj, reference camera and light, progressive sample batches 0-7)",
            "config": {"workload": "box.obj 1920x1080 8spp 4 bounces 3 sss", "width": W, "height": H,
                       "spp": SPP, "max_depth": DEPTH, "sss_bounces": SSS,
                       "parallelism": f"tiles{world}" if world > 1 else "single",
                       "rays_per_frame": int(rays_per_frame),
                       "msamples_per_s": round(W * H * SPP * args.steps / dt / 1e6, 3)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": None if prof is None else int(prof[1]),
                         "traffic_source": None if prof is None else prof[0],
                         "kernel": "render_kernel<false>", "kernel_ms": round(kernel_ms, 4),
                         "algorithmic_bytes_per_launch": int(bytes_per_launch)},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(v, i, n, cam, light)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
