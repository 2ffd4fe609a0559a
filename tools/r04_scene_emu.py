#!/usr/bin/env python3
"""Emulated N-GPU scene legs on one GPU, with the collective in (VERDICT r03
item 7).

For one BASELINE config, times on one GPU, in one process, the same loop
bench.py's dist_scene_leg runs on every rank at N > 1:
  full  : the whole frame, frames alternating over C contexts (own stream,
          accumulation buffer and wavefront buffers each), each frame
          followed by the reduce stand-in;
  share : rank 0's 1/N tile share (pt_set_partition(N, 0), +0/-0 clear),
          the same C contexts, each frame followed by the reduce stand-in.
The reduce stand-in is what rank 0's RCCL SUM reduce of the accumulation
buffer at least costs on its own GPU: a device-to-device copy of the whole
W x H x 16-B frame (a read and a write of it in HBM) on a high-priority
stream that waits for the frame's render, and which the context's next
work waits for (torch.distributed.reduce makes the current stream wait for
the collective).  It does not include the xGMI transfer time of the other
ranks' buffers; the driver's 8-GPU run is the real measurement.

Both legs use the same context count, so the ratio full/share is the
emulated N-GPU speed-up with the collective's local cost in.  Wall ms per
frame over K frames, median of 3 runs.  Prints one JSON line per config.

usage: r04_scene_emu.py {config3|config4|config5} [N=8] [C=3] [K]
environment: CAM=reference (BASELINE's (0,0,5), the legs' camera since round 5)
or scene (the frame-filling camera); GRID=percent (PT_OPT_WF_GRID of every
context, default 100); TAIL=PT_OPT_WF_TAIL with C > 1 (default 0, -1 auto)."""
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

CONFIGS = {"config3": ("sphere", 1920, 1080, 8, 4, 12), "config4": ("sphere", 3840, 2160, 16, 8, 6),
           "config5": ("synthetic:10000000", 1920, 1080, 8, 4, 9)}


def main():
    key = sys.argv[1]
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    C = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    scene_name, W, H, spp, depth, K = CONFIGS[key]
    if len(sys.argv) > 4:
        K = int(sys.argv[4])
    dev = torch.device("cuda", 0)
    scene, cam, int_bits, desc = bench.load_scene(scene_name)
    if os.environ.get("CAM", "scene") == "reference":
        cam = scenes.DEFAULT_CAMERA
        desc = desc.split(", camera")[0] + ", camera (0,0,5) fov 60"
    grid = int(os.environ.get("GRID", "100"))
    v, i, n, _, _ = scene.arrays()
    del scene
    comm = torch.cuda.Stream(dev, priority=-1)
    ctxs = []
    streams = []
    for _ in range(C):
        r = ptamd.Renderer(0)
        r.upload_scene(v, i, n, int_bits=int_bits)
        r.upload_lights(scenes.REFERENCE_LIGHT)
        r.set_camera(cam)
        r.set_params(depth, 3)
        if C > 1:
            r.set_option(ptamd.PT_OPT_WF_TAIL, int(os.environ.get("TAIL", "0")))   # as dist_scene_leg with frames in flight
        r.set_option(ptamd.PT_OPT_WF_GRID, grid)
        hs = bench.HipStream(0)
        streams.append(hs)
        r.set_stream(hs.handle)
        frame = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
        r.bind_accum(frame.data_ptr(), W, H)
        sink = torch.empty_like(frame)
        ctxs.append((r, hs, frame, sink))
    del v, i, n

    def frame_once(j):
        r, hs, frame, sink = ctxs[j % C]
        r.clear()
        r.render(0, spp)
        comm.wait_stream(hs.torch)          # the reduce follows the render ...
        with torch.cuda.stream(comm):
            sink.copy_(frame)               # ... reads and writes the whole frame ...
        hs.torch.wait_stream(comm)          # ... and the context's next work waits for it

    def leg(nranks):
        for r, _, _, _ in ctxs:
            r.set_partition(nranks, 0)
        for j in range(C):
            frame_once(j)
        torch.cuda.synchronize()
        walls = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for j in range(K):
                frame_once(j)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e3 / K)
        return walls

    full = leg(1)
    want = ctxs[0][0].read_accum().view(np.uint32).copy()
    share = leg(N)
    ok = True
    for r, _, _, _ in ctxs[1:]:   # the full frames of the first leg are gone; check the shares agree
        ok = ok and np.array_equal(r.read_accum().view(np.uint32), ctxs[0][0].read_accum().view(np.uint32))
    f, s = float(np.median(full)), float(np.median(share))
    print(json.dumps({"config": key, "workload": f"{desc} {W}x{H} {spp}spp D{depth}", "emulated_ranks": N,
                      "contexts": C, "wf_grid_percent": grid, "wf_tail": int(os.environ.get("TAIL", "0")), "frames_per_run": K, "reduce_standin_bytes": W * H * 16,
                      "full_frame_ms": [round(x, 3) for x in full], "share_ms": [round(x, 3) for x in share],
                      "full_frame_ms_median": round(f, 3), "share_ms_median": round(s, 3),
                      "emulated_speedup": round(f / s, 3), "shares_bitwise_equal": ok,
                      "full_frame_nonzero": int(np.count_nonzero(want))}), flush=True)
    for r, hs, _, _ in ctxs:
        r.close()
    torch.cuda.synchronize()
    for hs in streams:
        hs.close()


if __name__ == "__main__":
    main()
