#!/usr/bin/env python3
"""Flush-loop use of the wide trace kernel (a PT_WIDE_PROBE_FLUSH build,
loaded with PTAMD_LIB=ab/<name>.so): flushes, candidates per flush, the
largest queue per flush (the loop's trip count), and walking lanes per step.
  PTAMD_LIB=ab/fprobe.so python3 tools/flush_probe.py --scene sphere:6
The windows-per-flush figure needs the probe build of commit 97cc2b3 (its
counter [6] sums 64-candidate windows; the product source, kept at the
profiled text, sums each flush's largest queue there)."""
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
    r.set_option(ptamd.PT_OPT_WF_TAIL, 0)
    r.resize_and_clear(1920, 1080)
    r.reset_stats()
    r.render(0, a.spp)
    r.synchronize()
    t = r.traced()
    flushes, cands, maxq, steps, walking = (t["closest_walks"], t["shadow_walks"], t["nodes"], t["tri_tests"],
                                            t["primaries"])
    print(json.dumps({"scene": a.scene, "grid": a.grid, "refcam": a.refcam, "wave_steps": steps, "flushes": flushes,
                      "flushes_per_step": flushes / max(steps, 1),
                      "candidates_per_flush": cands / max(flushes, 1), "windows_per_flush": maxq / max(flushes, 1),
                      "window_lane_use": cands / max(64 * maxq, 1), "walking_lanes_per_step": walking / max(steps, 1)}))


if __name__ == "__main__":
    main()
