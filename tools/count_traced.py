#!/usr/bin/env python3
"""Work one frame really does (PT_OPT_COUNT_TRACED: walks, node visits,
triangle tests) under given kernel options, e.g.
  python tools/count_traced.py --scene sphere:6 16=64 16=80"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import ab_bench  # noqa: E402
import ptamd  # noqa: E402
import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="sphere:6")
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("variants", nargs="+", help="KEY=VAL[,KEY=VAL] per variant")
    a = ap.parse_args()
    scene, cam = ab_bench.load_scene(a.scene)
    r = ptamd.Renderer(0)
    r.upload(scene)
    r.upload_lights(scenes.REFERENCE_LIGHT)
    r.set_camera(cam)
    r.set_params(4, 3)
    r.resize_and_clear(a.w, a.h)
    for spec in a.variants:
        for kv in spec.split(","):
            k, v = kv.split("=")
            r.set_option(int(k), int(v))
        r.set_option(ptamd.PT_OPT_COUNT_TRACED, 1)
        r.reset_stats()
        r.clear()
        r.render(0, a.spp)
        t = r.traced()
        r.set_option(ptamd.PT_OPT_COUNT_TRACED, 0)
        print(json.dumps({"scene": a.scene, "variant": spec, "traced": {k: int(v) for k, v in t.items()}}), flush=True)


if __name__ == "__main__":
    main()
