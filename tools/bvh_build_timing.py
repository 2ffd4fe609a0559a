#!/usr/bin/env python3
"""BVH build time (single thread vs all cores) and
binary scene-cache save/load time for the synthetic clouds.  CPU only.
  python3 tools/bvh_build_timing.py [T ...]"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "discovering-path-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import ptamd  # noqa: E402
import scenes  # noqa: E402


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [1_000_000]
    for t in sizes:
        v, i = scenes.random_triangles(t, seed=42)
        int_bits = 2 * t - 1 >= (1 << 24)
        row = {"triangles": t, "cores": os.cpu_count(), "int_bits": int_bits}
        arrays = None
        for threads in ([1, 0] if t <= 2_000_000 else [0]):
            s = ptamd.Scene.from_arrays(v, i)
            t0 = time.perf_counter()
            s.build_bvh(int_bits=int_bits, threads=threads)
            row[f"build_s_threads_{threads or 'all'}"] = round(time.perf_counter() - t0, 3)
            a = s.arrays()
            if arrays is not None:
                row["single_vs_parallel_identical"] = all(
                    np.array_equal(x.view(np.uint32), y.view(np.uint32)) for x, y in zip(arrays, a))
            arrays = a
        with tempfile.TemporaryDirectory() as d:
            p = os.path.join(d, "scene.ptscene")
            t0 = time.perf_counter()
            s.save(p)
            row["cache_save_s"] = round(time.perf_counter() - t0, 3)
            row["cache_bytes"] = os.path.getsize(p)
            t0 = time.perf_counter()
            c = ptamd.Scene.load_cache(p)
            row["cache_load_s"] = round(time.perf_counter() - t0, 3)
            c.close()
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
