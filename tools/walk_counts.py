#!/usr/bin/env python3
"""Work per ray of the culled wide walk (csrc/wide_walk.h, the trace kernel's
default: 64-B nodes, queued leaf tests, wave-flush merge) on the CPU, for
compile-time variants of the walk: node visits, triangle tests and walk
steps per ray, for ray families shaped like a frame's (camera rays, SSS rays
from just under the surface, bounce rays off it, shadow rays to the light),
every answer checked against the oracle's exhaustive walk.
usage: walk_counts.py [sphere|cloud] [n_rays] [NAME=-DFLAG,-DFLAG ...]"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib  # noqa: E402
import scenes  # noqa: E402
import test_wide  # noqa: E402

CSRC = os.path.join(ROOT, "discovering-path-tracer_amd", "csrc")


def build(name, flags):
    so = os.path.join(ROOT, "tools", "_build", f"libwalk_{name}.so")
    srcs = [os.path.join(ROOT, "tests", "wide_check.cpp"), os.path.join(CSRC, "scene", "wide_bvh.cpp")]
    oracle_lib.lib()
    os.makedirs(os.path.dirname(so), exist_ok=True)
    subprocess.check_call(
        ["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__",
         "-ffp-contract=off", "-fno-fast-math", "-I", CSRC, "-o", so] + flags + srcs +
        ["-L", os.path.join(ROOT, "oracle"), "-loracle", "-Wl,-rpath," + os.path.join(ROOT, "oracle")])
    test_wide._LIB = None
    old = test_wide.SO
    test_wide.SO = so
    L = test_wide.lib()
    test_wide.SO = old
    test_wide._LIB = None
    L.wide_steps.restype = ctypes.c_ulonglong
    return L


def unit(a):
    return (a / np.sqrt((a * a).sum(-1, keepdims=True))).astype(np.float32)


def frame_rays(v, idx, n, seed, cam):
    rng = np.random.default_rng(seed)
    V = v.reshape(-1, 3)
    P = V[idx.reshape(-1, 3)]
    nrm = unit(np.cross(P[:, 1] - P[:, 0], P[:, 2] - P[:, 0]))
    k = n // 4
    fam = {}
    tgt = rng.uniform(-1.2, 1.2, (k, 3)).astype(np.float32)
    fam["camera"] = (np.tile(cam, (k, 1)), unit(tgt - cam), 0, 0)
    t = rng.integers(0, len(P), k)
    b = rng.dirichlet([1, 1, 1], k).astype(np.float32)
    sp = (P[t] * b[:, :, None]).sum(1)
    fam["sss"] = ((sp - nrm[t] * 1e-3).astype(np.float32), unit(rng.normal(size=(k, 3))), 0, 0)
    d = unit(rng.normal(size=(k, 3)))
    d = np.where((d * nrm[t]).sum(1, keepdims=True) < 0, -d, d).astype(np.float32)
    fam["bounce"] = ((sp + nrm[t] * 1e-3).astype(np.float32), d, 0, 0)
    light = np.float32([0, 2, 0]) + rng.uniform(-1.25, 1.25, (k, 3)).astype(np.float32) * np.float32([1, 0, 1])
    o = (sp + nrm[t] * 1e-3).astype(np.float32)
    dist = np.sqrt(((light - o) ** 2).sum(1)).astype(np.float32)
    fam["shadow"] = (o, unit(light - o), 1, dist - np.float32(1e-3))
    out = {}
    for name, (o, d, kind, lim) in fam.items():
        r = np.zeros((len(o), 8), np.float32)
        r[:, 0:3] = o
        r[:, 3:6] = d
        r[:, 6] = kind
        r[:, 7] = lim
        out[name] = r
    return out


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "sphere"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    variants = [("base", [])] + [(a.split("=", 1)[0], a.split("=", 1)[1].split(",")) for a in sys.argv[3:]]
    if which == "sphere":
        v, i = scenes.displaced_sphere(6)
        cam = np.float32([0, 0.5, 3])
    else:
        v, i = scenes.random_triangles(1000000, seed=42)
        cam = np.float32([0, 0, 2.2])
    v, idx, nodes = test_wide._scene(v, i)
    rays = frame_rays(v, idx, n, 5, cam)
    for vname, flags in variants:
        L = build(vname, flags)
        for name, r in rays.items():
            L.wide_set_mode(test_wide.WIDE_SAH)
            L.wide_set_variant(64, 2)
            r = np.ascontiguousarray(r)
            out = np.zeros(4 * len(r), np.float32)
            st = np.zeros(8, np.uint64)
            err = ctypes.create_string_buffer(256)
            assert L.wide_check(v, v.size, idx, idx.size // 3, nodes, nodes.size // 8, 0, r, len(r), out, st, err,
                                256) == 0, err.value
            walked = len(r) - int(st[2])
            print(f"{vname:10s} {name:7s} bad {int(st[0] + st[1])} nodes/ray {st[3] / walked:.3f} "
                  f"tris/ray {st[4] / walked:.3f} steps/ray {L.wide_steps() / walked:.3f}", flush=True)


if __name__ == "__main__":
    main()
