#!/usr/bin/env python3
"""A/B of leg options on frames in flight (bench.py's leg loop without its
counting passes): arguments "name[@contexts]:key=val,key=val ..." alternating, each a set
of `contexts` contexts (own HIP stream each) rendering frames back to back;
prints ms per frame per run.  Every variant's last frame must be bitwise the
first variant's.
  LEG="sphere 1920 1080 8 4 3" CTX=3 FRAMES=12 REPS=3 python tools/r05_leg_ab.py base: g50:20=50
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = [sys.argv[0]] + sys.argv[1:]
import torch  # noqa: E402,F401
import bench  # noqa: E402
import ptamd  # noqa: E402
import scenes  # noqa: E402


def main():
    scene_name, W, H, spp, depth, nctx = os.environ.get("LEG", "sphere 1920 1080 8 4 3").split()
    W, H, spp, depth, nctx = int(W), int(H), int(spp), int(depth), int(nctx)
    frames = int(os.environ.get("FRAMES", "12"))
    reps = int(os.environ.get("REPS", "3"))
    cam_kind = os.environ.get("CAM", "reference")
    scene, cam, int_bits, desc = bench.load_scene(scene_name)
    if cam_kind == "reference":
        cam = scenes.DEFAULT_CAMERA
    v, i, n, _, _ = scene.arrays()
    variants = []
    for spec in sys.argv[1:]:
        name, _, kv = spec.partition(":")
        opts = [tuple(int(x) for x in e.split("=")) for e in filter(None, kv.split(","))]
        variants.append((name, opts))
    sets = {}
    for name, opts in variants:
        ctxs, streams = [], []
        nc = int(name.split("@")[1]) if "@" in name else nctx
        for k in range(nc):
            x = ptamd.Renderer(0)
            x.upload_scene(v, i, n, int_bits=int_bits)
            x.upload_lights(scenes.REFERENCE_LIGHT)
            x.set_camera(cam)
            x.set_params(depth, 3)
            x.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
            x.set_option(ptamd.PT_OPT_LAUNCH_TIMING, 0)
            if nc > 1:
                x.set_option(ptamd.PT_OPT_WF_TAIL, 0)
                hs = bench.HipStream(0)
                streams.append(hs)
                x.set_stream(hs.handle)
            for key, val in opts:
                x.set_option(key, val)
            x.resize_and_clear(W, H)
            ctxs.append(x)
        sets[name] = (ctxs, streams)
    ref = None
    for name, (ctxs, _) in sets.items():
        for x in ctxs:
            x.render(0, spp)
        torch.cuda.synchronize()
        img = ctxs[0].read_accum().view(np.uint32)
        if ref is None:
            ref = img
        elif not np.array_equal(img, ref):
            print(f"MISMATCH: variant {name} differs from the first", flush=True)
            sys.exit(1)
    print(f"{scene_name} {W}x{H}x{spp} D{depth} camera {cam_kind}, {nctx} contexts unless name@n, {frames} frames per run",
          flush=True)
    for r in range(reps):
        for name, (ctxs, _) in sets.items():
            ms = bench.time_frames_pipelined(ctxs, spp, frames, groups=1)
            print(f"rep {r} {name:12s} {float(ms[0]):.3f} ms/frame", flush=True)


if __name__ == "__main__":
    main()
