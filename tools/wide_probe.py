#!/usr/bin/env python3
"""Lane-state census of the wide trace kernel (a PT_WIDE_PROBE build, loaded
with PTAMD_LIB=ab/<name>.so): per wave step, lanes walking / idle / waiting
on their leaf queue, and the share of steps that flush.
  PTAMD_LIB=ab/probe.so python3 tools/wide_probe.py --scene sphere:6"""
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
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--grid", type=int, default=100, help="PT_OPT_WF_GRID (percent of the traversal grid)")
    ap.add_argument("--refcam", action="store_true", help="BASELINE's camera (0,0,5), the legs' primary")
    a = ap.parse_args()
    scene, cam = ab_bench.load_scene(a.scene)
    r = ptamd.Renderer(0)
    r.upload(scene)
    r.upload_lights(scenes.REFERENCE_LIGHT)
    r.set_camera(scenes.DEFAULT_CAMERA if a.refcam else cam)
    r.set_option(ptamd.PT_OPT_WF_GRID, a.grid)
    r.set_params(4, 3)
    r.resize_and_clear(1920, 1080)
    r.reset_stats()
    r.render(0, a.spp)
    r.synchronize()
    t = r.traced()
    walking, idle_more, idle_drain, steps, waiting = (t["closest_walks"], t["shadow_walks"], t["nodes"],
                                                      t["tri_tests"], t["primaries"])
    lanes = 64.0 * max(steps, 1)
    print(json.dumps({"scene": a.scene, "grid": a.grid, "refcam": a.refcam, "wave_steps": steps, "walking": walking / lanes,
                      "idle_rays_left": idle_more / lanes, "idle_drain": idle_drain / lanes,
                      "waiting_on_queue": waiting / lanes}))


if __name__ == "__main__":
    main()
