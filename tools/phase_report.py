#!/usr/bin/env python3
"""Per-phase wave-cycle shares of the render kernel from an instrumented
build (tools/phase_instrument.py).  Usage:
  PTAMD_LIB=ab/phase.so python3 tools/phase_report.py [ab_bench-style variant args]"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "discovering-path-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import ptamd  # noqa: E402
import ab_bench  # noqa: E402

NAMES = {1: "primary trace", 2: "shadow (direct)", 3: "sss trace", 4: "sss shadow", 5: "bounce trace"}


def main():
    scene_name = sys.argv[1] if len(sys.argv) > 1 else "box"
    opts = sys.argv[2:]
    scene, cam = ab_bench.load_scene(scene_name)
    r = ptamd.Renderer(0)
    for kv in opts:
        k, v = kv.split("=")
        r.set_option(int(k), int(v))
    r.upload(scene)
    r.upload_lights(ab_bench.scenes.REFERENCE_LIGHT)
    r.set_camera(cam)
    r.resize_and_clear(1920, 1080)
    L = ptamd.lib()
    f = L.pt_debug_phase
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros(16, np.uint64)
    r.render(0, 8)
    r.synchronize()
    f(buf.ctypes.data, 1)
    for _ in range(5):
        r.clear()
        r.render(0, 8)
    r.synchronize()
    f(buf.ctypes.data, 0)
    b = buf.astype(np.float64)
    tot = b[8]
    out = {"kernel_wave_cycles": tot}
    out["ray gen + cull"] = (b[0] - b[6]) / tot
    for k, n in NAMES.items():
        out[n] = b[k] / tot
    out["shading math"] = (b[6] - b[1:6].sum()) / tot
    out["fold"] = b[7] / tot
    out["outside sample loop"] = (tot - b[0] - b[7]) / tot
    out["  start..scene staged"] = b[9] / tot
    out["  start..sample loop"] = b[10] / tot
    out["  final store..end"] = b[11] / tot
    print(json.dumps({k: (round(v, 4) if k != "kernel_wave_cycles" else v) for k, v in out.items()}, indent=1))


if __name__ == "__main__":
    main()
