#!/usr/bin/env python3
"""The box frame on two contexts (the bench's N = 1 step: one lane per pixel,
frames alternating, own streams) with the live items in scan order (0) or
heaviest first (1), per context: runs of K frames after a warm GPU, wall ms
per frame (median of R runs), alternating variants.
  python tools/r05_box_order.py K R  V...   with V = o<ctx0><ctx1>, e.g. o00 o11 o01"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = sys.argv
import torch  # noqa: E402
import bench  # noqa: E402
import ptamd  # noqa: E402
import scenes  # noqa: E402


def make(order, stream):
    s = ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh()
    r = ptamd.Renderer(0)
    r.upload(s)
    r.upload_lights(scenes.REFERENCE_LIGHT)
    r.set_camera(scenes.DEFAULT_CAMERA)
    r.set_params(4, 3)
    r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
    r.set_option(ptamd.PT_OPT_LAUNCH_TIMING, 0)
    r.set_option(ptamd.PT_OPT_SAMPLE_LANES, 1)
    r.set_option(ptamd.PT_OPT_ITEM_ORDER, order)
    r.set_stream(stream.handle)
    r.resize_and_clear(1920, 1080)
    return r


def main():
    k, reps = int(sys.argv[1]), int(sys.argv[2])
    variants = sys.argv[3:]
    streams = [bench.HipStream(0), bench.HipStream(0)]
    sets = {v: [make(int(v[1]), streams[0]), make(int(v[2]), streams[1])] for v in variants}
    want = None
    for v, rs in sets.items():
        for r in rs:
            r.render(0, 8)
        torch.cuda.synchronize()
        img = rs[1].read_accum().view(np.uint32)
        want = img if want is None else want
        assert np.array_equal(img, want), v
    res = {v: [] for v in variants}
    for _ in range(reps):
        for v, rs in sets.items():
            for j in range(40):   # busy GPU before each run (clocks up)
                rs[j % 2].render(0, 8)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for j in range(k):
                rs[(j + 1) % 2].render(0, 8)   # as bench.py: after 5 warmup frames the run starts on context 1
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / k * 1e3)
    for v in variants:
        print(f"{v} K={k}: median {np.median(res[v]):.4f} ms/frame (min {np.min(res[v]):.4f}, max {np.max(res[v]):.4f})",
              flush=True)


if __name__ == "__main__":
    main()
