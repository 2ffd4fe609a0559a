#!/usr/bin/env python3
"""Why does `bench.py --steps 20 --warmup 5` measure more per frame than
`--steps 200 --warmup 10`?  

Replays bench.py's N = 1 box setup (two contexts, one lane per pixel, items
in scan order, least-priority HIP streams; the stats and counting passes on
context 0 first) and then times, in one process:
  A. the driver's block: 5 warmup + 20 timed frames, bracketed as bench.py does;
  B. ten more 20-frame blocks back to back (each bracketed the same way);
  C. a 20-frame block after 300 ms of host idle;
  D. a 200-frame block;
  E. a 20-frame block with a device-event timeline: the start and end of
     every frame on its stream, relative to an event before the first frame.
Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "discovering-path-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import bench  # noqa: E402
import ptamd  # noqa: E402
import scenes  # noqa: E402

SPP = 8


def block(ctxs, steps, warmup=0):
    for k in range(warmup):
        ctxs[k % len(ctxs)].render(0, SPP)
    for c in ctxs:
        c.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        ctxs[k % len(ctxs)].render(0, SPP)
    t_enq = time.perf_counter() - t0
    for c in ctxs:
        c.synchronize()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return dt / steps * 1e3, t_enq / steps * 1e3


def main():
    scene, cam, _, _ = bench.load_scene("box")
    v, i, n, _, _ = scene.arrays()
    streams = []
    ctxs = []
    for k in range(2):
        x = ptamd.Renderer(0)
        x.upload_scene(v, i, n)
        x.upload_lights(scenes.REFERENCE_LIGHT)
        x.set_camera(cam)
        x.set_params(4, 3)
        x.set_option(ptamd.PT_OPT_LAUNCH_TIMING, 1 if k == 0 else 0)
        if k == 0:
            x.resize_and_clear(1920, 1080)
            bench.reference_and_traced_counts(x, SPP)   # as bench.py: the counting passes first
        x.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
        x.set_option(ptamd.PT_OPT_SAMPLE_LANES, 1)
        x.set_option(ptamd.PT_OPT_ITEM_ORDER, 0)
        hs = bench.HipStream(0)
        streams.append(hs)
        x.set_stream(hs.handle)
        x.resize_and_clear(1920, 1080)
        ctxs.append(x)
    out = {}
    out["A_driver_block_ms"], out["A_host_issue_ms"] = block(ctxs, 20, warmup=5)
    out["B_repeat_blocks_ms"] = [round(block(ctxs, 20)[0], 4) for _ in range(10)]
    time.sleep(0.3)
    out["C_after_idle_ms"] = block(ctxs, 20)[0]
    out["D_200_ms"] = block(ctxs, 200)[0]
    # E: timeline
    ev = []
    torch.cuda.synchronize()
    t_start = torch.cuda.Event(enable_timing=True)
    t_start.record(streams[0].torch)
    streams[1].torch.wait_event(t_start)
    for k in range(20):
        s = streams[k % 2].torch
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(s)
        ctxs[k % 2].render(0, SPP)
        b.record(s)
        ev.append((a, b))
    torch.cuda.synchronize()
    out["E_timeline_ms"] = [(round(t_start.elapsed_time(a), 4), round(t_start.elapsed_time(b), 4)) for a, b in ev]
    out["E_total_ms"] = round(t_start.elapsed_time(ev[-1][1]), 4)
    # F: a single frame alone, and 20 frames one at a time on one context
    out["F_single_frames_ms"] = [round(block(ctxs[:1], 1)[0], 4) for _ in range(5)]
    print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()
    for s in streams:
        s.close()


if __name__ == "__main__":
    main()
