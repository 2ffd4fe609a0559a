#!/usr/bin/env python3
"""Interleaved A/B timing of kernel variants on one GPU (device time from the
library's per-launch HIP events).  Usage:
  python tools/ab_bench.py [--scene box|sphere|random:N] [--reps 10] VARIANT...
VARIANT = name:key=val,key=val with keys lds (PT_OPT_SCENE_IN_LDS), opt<k> (pt_set_option key k).
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "discovering-path-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ptamd  # noqa: E402
import scenes  # noqa: E402


def load_scene(name):
    if name == "box":
        return ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh(), scenes.DEFAULT_CAMERA
    if name == "box_away":   # every pixel culled: the kernel's fixed per-workgroup cost
        cam = np.array([-10, 0, 5, 0, 1, 0, 0, 0, 0, 1, 0, 0, 10, 0, 0, 0], np.float32)
        return ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh(), cam
    if name.startswith("sphere"):
        v, i = scenes.displaced_sphere(int(name.split(":")[1]) if ":" in name else 5)
        return ptamd.Scene.from_arrays(v, i).build_bvh(), scenes.camera((0.0, 0.5, 3.0))
    if name.startswith("random:"):
        v, i = scenes.random_triangles(int(name.split(":")[1]), seed=42)
        return ptamd.Scene.from_arrays(v, i).build_bvh(int_bits=True), scenes.camera((0.0, 0.0, 2.2))
    raise SystemExit(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="box")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    scene, cam = load_scene(a.scene)
    if os.environ.get("CAM") == "reference":   # BASELINE's camera (0,0,5), the legs' primary
        cam = scenes.DEFAULT_CAMERA
    rs = []
    for spec in a.variants:
        name, _, kv = spec.partition(":")
        r = ptamd.Renderer(0)
        depth, sss, nlights = 4, 3, 1
        for item in filter(None, kv.split(",")):
            k, v = item.split("=")
            if k == "depth":
                depth = int(v)
            elif k == "sss":
                sss = int(v)
            elif k == "nl":      # number of lights (0 or 1)
                nlights = int(v)
            elif k == "nr":      # emulate one rank of an N-GPU tile split: nr=N (rank 0)
                r.set_partition(int(v), 0)
            else:
                key = ptamd.PT_OPT_SCENE_IN_LDS if k == "lds" else int(k[3:])
                r.set_option(key, int(v))
        r.upload(scene)
        r.upload_lights(scenes.REFERENCE_LIGHT if nlights else scenes.REFERENCE_LIGHT[:0])
        r.set_camera(cam)
        r.set_params(depth, sss)
        r.resize_and_clear(a.w, a.h)
        rs.append((name, r))
    ref = None
    digest = None
    for name, r in rs:
        r.render(0, a.spp)   # warm + parity between variants
        img = r.read_accum()
        if digest is None:   # compared across library builds by tools/ab_libs_scenes.sh
            import hashlib
            digest = hashlib.sha1(img.tobytes()).hexdigest()[:12]
        if ref is None or a.no_parity:
            ref = img
        elif not np.array_equal(img.view(np.uint32), ref.view(np.uint32)):
            print(f"WARNING: variant {name} output differs from {rs[0][0]}")
        r.set_option(ptamd.PT_OPT_LAUNCH_TIMING, 1)
        r.reset_launch_times()
    for _ in range(a.reps):
        for name, r in rs:
            r.clear()
            r.render(0, a.spp)
            r.synchronize()
    out = {}
    for name, r in rs:
        t = r.launch_times_ms()
        out[name] = {"mean_ms": float(t.mean()), "min_ms": float(t.min()), "std_ms": float(t.std())}
    print(json.dumps({"scene": a.scene, "W": a.w, "H": a.h, "spp": a.spp, "frame_sha1": digest, "results": out}))


if __name__ == "__main__":
    main()
