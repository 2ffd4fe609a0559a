#!/usr/bin/env python3
"""Large-scene frames back to back on one context vs alternating between two
contexts (own stream, accumulation buffer and wavefront buffers each), so
one frame's ray rounds run beside the other's drains.  Device-busy wall time
per frame over K frames; the contexts' frames checked bitwise equal."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "discovering-path-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
import ab_bench  # noqa: E402
import ptamd  # noqa: E402
import scenes  # noqa: E402


def main():
    name = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    nr = int(sys.argv[3]) if len(sys.argv) > 3 else 1   # rank 0's tile share of an nr-way split
    W, H, spp, depth = (3840, 2160, 16, 8) if name.endswith("4k") else (1920, 1080, 8, 4)
    scene, cam = ab_bench.load_scene(name.replace("_4k", ""))
    rs = []
    for _ in range(3):
        r = ptamd.Renderer(0)
        r.upload(scene)
        r.upload_lights(scenes.REFERENCE_LIGHT)
        r.set_camera(cam)
        r.set_params(depth, 3)
        r.set_partition(nr, 0)
        for kv in filter(None, os.environ.get("PT_SS_OPTS", "").split(",")):   # e.g. "17=0,2=1"
            key, _, val = kv.partition("=")
            r.set_option(int(key), int(val))
        r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
        s = torch.cuda.Stream()
        r.set_stream(s.cuda_stream)
        r.resize_and_clear(W, H)
        r.render(0, spp)
        rs.append((r, s))
    torch.cuda.synchronize()

    def run(ctx):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            ctx[i % len(ctx)][0].render(0, spp)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    for rep in range(2):
        print(f"{name} nr={nr}: one context {run(rs[:1]):.2f} ms/frame, two {run(rs[:2]):.2f}, "
              f"three {run(rs):.2f}", flush=True)
    a = rs[0][0].read_accum()
    for x in rs[1:]:
        assert np.array_equal(a.view(np.uint32), x[0].read_accum().view(np.uint32))
    print("frames bitwise equal")


if __name__ == "__main__":
    main()
