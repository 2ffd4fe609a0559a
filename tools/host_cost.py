#!/usr/bin/env python3
"""Host cost of the pieces of bench.py's N>1 step (render_packed through
ctypes, torch stream switches, a side-stream copy), measured on one GPU with
rank 0's share of an N-way split.  Prints microseconds per call."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "discovering-path-tracer_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import ptamd  # noqa: E402
import scenes  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda", 0)
scene = ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh()
v, i, n, _, _ = scene.arrays()
r = ptamd.Renderer(0)
r.upload_scene(v, i, n)
r.upload_lights(scenes.REFERENCE_LIGHT)
r.set_camera(scenes.DEFAULT_CAMERA)
r.set_params(4, 3)
r.set_partition(N, 0, [11] + [16] * (N - 1))
s0, s1 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
torch.cuda.set_stream(s0)
r.set_stream(s0.cuda_stream)
r.resize_and_clear(1920, 1080)
r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
r.render(0, 8)
per = r.items_live(0)[1]
slot = max(r.items_live(k)[0] for k in range(N)) * per * 4
send = torch.zeros(slot, device=dev)
recv = torch.zeros((N, slot), device=dev)
out = torch.empty((1080, 1920, 4), device=dev)
src = torch.zeros((N - 1) * slot, device=dev)


def t(label, fn, reps=200):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    dt = (time.perf_counter() - t0) / reps * 1e6
    torch.cuda.synchronize()
    print(f"{label:40s} {dt:8.2f} us")


t("r.render(0, 8)", lambda: r.render(0, 8))
t("r.render_packed(8, send)", lambda: r.render_packed(8, send.data_ptr()))
t("r.render_packed(8, send, recv, frame)", lambda: r.render_packed(8, send.data_ptr(), recv.data_ptr(), slot, out.data_ptr()))
r.set_option(ptamd.PT_OPT_LAUNCH_TIMING, 0)
t("  same, launch timing off", lambda: r.render_packed(8, send.data_ptr(), recv.data_ptr(), slot, out.data_ptr()))
t("torch.cuda.set_stream + r.set_stream", lambda: (torch.cuda.set_stream(s1), r.set_stream(s1.cuda_stream)))
t("s1.wait_stream(s0)", lambda: s1.wait_stream(s0))
t("recv[1:].view(-1).copy_(src)", lambda: recv[1:].view(-1).copy_(src))
t("torch.cuda.Event().record(s0)", lambda: torch.cuda.Event().record(s0))
t("ctypes no-op (pt_abi_version)", lambda: ptamd.lib().pt_abi_version())
