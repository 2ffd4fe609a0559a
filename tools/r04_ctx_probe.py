#!/usr/bin/env python3
"""Frames in flight for the large-scene legs: bench.py's own scene_leg (the
timed loop the bench line reports) with 1-5 contexts, for one BASELINE
config.  Prints one JSON line per context count.
usage: r04_ctx_probe.py {config3|config4|config5} [counts=2,3,4]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    key = sys.argv[1]
    counts = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "2,3,4").split(",")]
    leg = next(l for l in bench.SCENE_LEGS if l[0] == key)
    _, scene_name, W, H, spp, depth, steps, workload, _ = leg
    for c in counts:
        r = bench.scene_leg(scene_name, W, H, spp, depth, 3, steps, 0, workload, contexts=c)
        print(json.dumps({"config": key, "contexts": c, "ms_per_step": r.get("ms_per_step")}), flush=True)


if __name__ == "__main__":
    main()
