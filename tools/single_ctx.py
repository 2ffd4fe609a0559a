#!/usr/bin/env python3
"""The drop-in frame: box 1080p 8 spp on ONE context (one stream, one
accumulation buffer), frames back to back, each a whole frame from batch 0
(the reference renders one image at a time,
VulkanRayTracer.cpp:717-865).  Variants are output-invariant options
(`name:key=val,...`), each timed in runs of K frames after a warm-up load,
alternating variants between runs; every variant's last frame is checked
bitwise against the library-default frame.

usage: python tools/single_ctx.py [K] [variant ...]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "discovering-path-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401  (HIP runtime first)
import ptamd  # noqa: E402
import scenes  # noqa: E402


def make(opts):
    s = ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh()
    r = ptamd.Renderer(0)
    r.upload(s)
    r.upload_lights(scenes.REFERENCE_LIGHT)
    r.set_camera(scenes.DEFAULT_CAMERA)
    r.set_params(4, 3)
    r.resize_and_clear(1920, 1080)
    r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
    r.set_option(ptamd.PT_OPT_LAUNCH_TIMING, 1)
    for k, v in opts:
        r.set_option(k, v)
    return r


def parse(spec):
    name, _, rest = spec.partition(":")
    opts = []
    for kv in filter(None, rest.split(",")):
        k, _, v = kv.partition("=")
        opts.append((int(k), int(v)))
    return name, opts


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    specs = sys.argv[2:] or ["default:"]
    variants = [(n, make(o)) for n, o in map(parse, specs)]
    ref = None
    # warm load: 60 ms of frames so the clocks are up
    r0 = variants[0][1]
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.06:
        r0.render(0, 8)
        r0.synchronize()
    res = {n: [] for n, _ in variants}
    kern = {n: [] for n, _ in variants}
    for rep in range(6):
        for n, r in variants:
            r.render(0, 8)
            r.synchronize()
            r.reset_launch_times()
            t0 = time.perf_counter()
            for _ in range(k):
                r.render(0, 8)
            r.synchronize()
            res[n].append((time.perf_counter() - t0) * 1e3 / k)
            kt = r.launch_times_ms()
            if kt.size:
                kern[n].append(float(np.mean(kt)))
    want = variants[0][1].read_accum().view(np.uint32)
    for n, r in variants:
        same = bool(np.array_equal(r.read_accum().view(np.uint32), want))
        a = np.array(res[n])
        print(f"{n:24s} K={k:4d} ms/frame min {a.min():.4f} med {np.median(a):.4f} max {a.max():.4f} "
              f"kernel_ms {np.median(kern[n]) if kern[n] else float('nan'):.4f} same_as_first {same}", flush=True)


if __name__ == "__main__":
    main()
