#!/usr/bin/env python3
"""Counters of the drain hand-off (a PT_WIDE_CARRY_PROBE build, PTAMD_LIB=ab/<name>.so):
records handed off, records claimed, CAS retries, flag polls, pick attempts."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import ab_bench  # noqa: E402
import ptamd  # noqa: E402
import scenes  # noqa: E402

scene, cam = ab_bench.load_scene(sys.argv[1] if len(sys.argv) > 1 else "sphere:6")
r = ptamd.Renderer(0)
r.upload(scene)
r.upload_lights(scenes.REFERENCE_LIGHT)
r.set_camera(cam)
r.set_params(4, 3)
r.resize_and_clear(1920, 1080)
r.reset_stats()
r.set_option(ptamd.PT_OPT_LAUNCH_TIMING, 1)
r.render(0, 8)
r.synchronize()
t = r.traced()
print(json.dumps({"handed_off": t["closest_walks"], "claimed": t["shadow_walks"], "cas_retries": t["nodes"],
                  "flag_polls": t["tri_tests"], "pick_attempts": t["primaries"],
                  "ms": float(r.launch_times_ms().mean())}))
