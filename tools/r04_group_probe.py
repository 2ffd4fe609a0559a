#!/usr/bin/env python3
"""Host cost of a multi-device context's render (pt_create_multi), with the
members' launches enqueued from the caller's thread or from per-member
enqueue threads (PT_GROUP_THREADS), on this box's one GPU (every member on
device 0, so the device time is the whole frame's; the host cost is what a
node of n GPUs would pay per frame).  box.obj 1080p, 8 spp per render.
Prints one JSON line.  usage: r04_group_probe.py [n=8]"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "discovering-path-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def child(n):
    import numpy as np
    import ptamd
    import scenes
    scene = ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh()
    v, i, nn, _, _ = scene.arrays()
    g = ptamd.Renderer(devices=[0] * n)
    g.upload_scene(v, i, nn)
    g.upload_lights(scenes.REFERENCE_LIGHT)
    g.set_camera(scenes.DEFAULT_CAMERA)
    g.set_params(4, 3)
    g.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
    g.resize_and_clear(1920, 1080)
    for _ in range(20):
        g.render(0, 8)
    g.synchronize()
    host, wall = [], []
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(50):
            g.render(0, 8)
        t1 = time.perf_counter()
        g.synchronize()
        t2 = time.perf_counter()
        host.append((t1 - t0) / 50 * 1e3)
        wall.append((t2 - t0) / 50 * 1e3)
    one = ptamd.Renderer(0)
    one.upload_scene(v, i, nn)
    one.upload_lights(scenes.REFERENCE_LIGHT)
    one.set_camera(scenes.DEFAULT_CAMERA)
    one.set_params(4, 3)
    one.resize_and_clear(1920, 1080)
    one.render(0, 8)
    same = bool(np.array_equal(g.read_accum().view(np.uint32), one.read_accum().view(np.uint32)))
    print(json.dumps({"members": n, "threads": os.environ.get("PT_GROUP_THREADS", "1"),
                      "host_ms_per_render": [round(x, 4) for x in host],
                      "wall_ms_per_render": [round(x, 4) for x in wall], "bitwise_equal_single_gpu": same}),
          flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "child":
        child(int(sys.argv[1]))
        sys.exit(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    for th in ("0", "1"):
        env = dict(os.environ, PT_GROUP_THREADS=th)
        r = subprocess.run([sys.executable, __file__, str(n), "child"], env=env, capture_output=True, text=True,
                           timeout=150)
        sys.stdout.write(r.stdout)
        if r.returncode:
            sys.stderr.write(r.stderr[-3000:])
            sys.exit(r.returncode)
