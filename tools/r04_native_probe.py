#!/usr/bin/env python3
"""Host and device time of pt_dist_run per frame, by call length, for rank
0's share of an emulated N-way split (bench.py's PT_BENCH_EMULATE_RANKS=N
native path: a 1-rank communicator, the other slots as a device copy).

For calls of K = 20 and K = 200 frames, after a warm-up: host time to issue
the call (t_enq) and wall time to its completion, per frame, each call
bracketed by a synchronize.  Also the per-call fixed part: a 1-frame call.
Prints one JSON line.  usage: r04_native_probe.py [N=8]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "discovering-path-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import ptamd  # noqa: E402
import scenes  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda", 0)
    scene = ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh()
    v, i, n, _, _ = scene.arrays()
    r = ptamd.Renderer(0)
    r.upload_scene(v, i, n)
    r.upload_lights(scenes.REFERENCE_LIGHT)
    r.set_camera(scenes.DEFAULT_CAMERA)
    r.set_params(4, 3)
    r.set_partition(N, 0, [12] + [16] * (N - 1))
    r.resize_and_clear(1920, 1080)
    r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
    r.set_option(ptamd.PT_OPT_LAUNCH_TIMING, 4)
    r.render(0, 8)
    r.dist_init(ptamd.Renderer.dist_unique_id(), 1, 0)
    frames = torch.empty((3, 1080, 1920, 4), dtype=torch.float32, device=dev)

    def call(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r.dist_run(8, k, frames.data_ptr(), 3, n_streams=3)
        t1 = time.perf_counter()
        r.synchronize()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        return (t1 - t0) * 1e3, (t2 - t0) * 1e3

    # load the GPU for ~60 ms first (clocks up)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.06:
        call(50)
    out = {"N": N}
    for k in (1, 20, 200):
        res = [call(k) for _ in range(5)]
        out[f"k{k}_host_ms_per_frame"] = [round(a / k, 4) for a, _ in res]
        out[f"k{k}_wall_ms_per_frame"] = [round(b / k, 4) for _, b in res]
    time.sleep(0.3)
    a, b = call(20)
    out["k20_after_300ms_idle"] = {"host_ms_per_frame": round(a / 20, 4), "wall_ms_per_frame": round(b / 20, 4)}
    print(json.dumps(out), flush=True)
    r.dist_finalize()


if __name__ == "__main__":
    main()
