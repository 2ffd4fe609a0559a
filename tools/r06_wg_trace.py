#!/usr/bin/env python3
"""Per-workgroup timeline of one box 1080p8 frame (probe build ab/wgtrace.so,
-DPT_WG_TRACE: each live workgroup of render_kernel records its start and end
on the GPU wall clock, its CU and XCC, its lane count and first pixel).

usage: PTAMD_LIB=ab/wgtrace.so python tools/r06_wg_trace.py OUT.npz key=val,...
Prints a summary; the records go to OUT.npz for offline analysis."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "discovering-path-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401
import ptamd  # noqa: E402
import scenes  # noqa: E402

WALL_HZ = 100e6   # gfx9 s_memrealtime


def main():
    out = sys.argv[1]
    opts = [tuple(int(x) for x in kv.split("=")) for kv in filter(None, (sys.argv[2] if len(sys.argv) > 2 else "").split(","))]
    s = ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh()
    r = ptamd.Renderer(0)
    r.upload(s)
    r.upload_lights(scenes.REFERENCE_LIGHT)
    r.set_camera(scenes.DEFAULT_CAMERA)
    r.set_params(4, 3)
    r.resize_and_clear(1920, 1080)
    r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
    r.set_option(ptamd.PT_OPT_LAUNCH_TIMING, 1)
    for k, v in opts:
        r.set_option(k, v)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.1:
        r.render(0, 8)
        r.synchronize()
    r.reset_launch_times()
    r.render(0, 8)
    r.synchronize()
    kms = float(r.launch_times_ms()[-1])
    L = ptamd.lib()
    f = L.pt_probe_wg_trace
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros((1 << 16, 4), np.uint64)
    rc = f(buf.ctypes.data, buf.shape[0])
    assert rc == 0, rc
    mi = r.mixed_info()
    n = mi[1] if mi[0] else int(np.count_nonzero(buf[:, 1]))   # the last launch's live workgroups
    rec = buf[:n]
    t_0 = rec[:, 0].astype(np.int64)
    t_1 = rec[:, 1].astype(np.int64)
    base = t_0.min()
    st = (t_0 - base) / WALL_HZ * 1e6
    en = (t_1 - base) / WALL_HZ * 1e6
    dur = en - st
    meta = rec[:, 2]
    spl = ((meta >> np.uint64(8)) & np.uint64(0xf)).astype(int)
    xcc = (meta & np.uint64(0xff)).astype(int)
    hw = (meta >> np.uint64(32)).astype(np.int64)
    cu = (hw >> 8) & 0xf
    se = (hw >> 13) & 0x7
    xy = rec[:, 3]
    x0 = (xy >> np.uint64(32)).astype(int)
    y0 = (xy & np.uint64(0xffffffff)).astype(int)
    np.savez(out, st=st, en=en, spl=spl, xcc=xcc, cu=cu, se=se, x0=x0, y0=y0, kernel_ms=kms)
    print(f"opts {opts} mixed {mi}: {n} live workgroups, kernel {kms * 1e3:.1f} us, last live end {en.max():.1f} us")
    for v in sorted(set(spl)):
        m = spl == v
        d = dur[m]
        print(f"  spl {v}: {m.sum():5d} wgs, dur mean {d.mean():6.1f} p50 {np.median(d):6.1f} p90 "
              f"{np.percentile(d, 90):6.1f} max {d.max():6.1f} us; start p50 {np.median(st[m]):6.1f} max "
              f"{st[m].max():6.1f}; end max {en[m].max():6.1f}")
    # concurrency over time: resident live workgroups per 10-us bin
    edges = np.arange(0, en.max() + 10, 10)
    res = [int(np.count_nonzero((st < b + 10) & (en > b))) for b in edges]
    print("  resident per 10 us:", res)
    last = np.argsort(en)[-8:]
    for k in last:
        print(f"  late: wg {k} spl {spl[k]} ({x0[k]},{y0[k]}) start {st[k]:.1f} end {en[k]:.1f} dur {dur[k]:.1f}")
    # cost map: mean duration per 16x16 tile of the spl-1 (or all) workgroups by row band
    ys = np.unique(y0 // 16)
    band = {int(y): float(np.mean(dur[(y0 // 16) == y] * spl[(y0 // 16) == y])) for y in ys}
    print("  lane-normalised cost by tile row (dur x spl):", {k: round(v) for k, v in list(band.items())})


if __name__ == "__main__":
    main()
