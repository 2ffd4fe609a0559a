#!/usr/bin/env python3
"""Box frames back to back on one context/stream vs alternating between two
contexts (each its own stream and accumulation buffer, so frame k+1 starts
while frame k drains).  Wall time over K frames, and a bitwise check that
both contexts' frames equal the one-stream frame."""
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


def make():
    s = ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh()
    r = ptamd.Renderer(0)
    r.upload(s)
    r.upload_lights(scenes.REFERENCE_LIGHT)
    r.set_camera(scenes.DEFAULT_CAMERA)
    r.set_params(4, 3)
    r.resize_and_clear(1920, 1080)
    r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
    r.set_option(ptamd.PT_OPT_LAUNCH_TIMING, 0)
    return r


def run(rs, k):
    for i in range(10):
        rs[i % len(rs)].render(0, 8)
    for r in rs:
        r.synchronize()
    t0 = time.perf_counter()
    for i in range(k):
        rs[i % len(rs)].render(0, 8)
    for r in rs:
        r.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    a, b, c = make(), make(), make()
    a.render(0, 8)
    ref = a.read_accum()
    for rep in range(3):
        one = run([a], k)
        two = run([b, c], k)
        three = run([a, b, c], k)
        print(f"one stream {one:.4f} ms/frame, two contexts {two:.4f}, three {three:.4f}", flush=True)
    for r in (b, c):
        assert np.array_equal(r.read_accum().view(np.uint32), ref.view(np.uint32))
    print("frames bitwise equal")


if __name__ == "__main__":
    main()
