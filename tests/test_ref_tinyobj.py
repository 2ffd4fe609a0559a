"""Pins OBJ ingest against the reference's own loader.

oracle/_ref/libref_tinyobj.so is the reference's vendored tinyobjloader
(external/tiny_obj_loader.h, compiled unmodified where it lies by
`make -C oracle ref`, wrapped as the reference's call site
VulkanRayTracer.cpp:64-92 uses it).  Both restatements -- the product's
pt_scene_parse_obj (csrc/scene/obj_loader.cpp) and the oracle's
oracle_obj_parse -- must reproduce its vertex floats bit for bit and its
triangle index order exactly: the order decides the BVH the builder makes
(BoundingVolumeHierarchy.cpp:25-82) and so every traversal tie-break.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as O
import ptamd
import scenes
from test_host import OBJ_CASES

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_tinyobj.so")
_REF = None


def ref_lib():
    global _REF
    if _REF is None:
        if not os.path.exists(REF_SO):
            if not os.path.exists("/root/reference/external/tiny_obj_loader.h"):
                pytest.skip("oracle/_ref not built and the reference tree is absent")
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"])
        L = ctypes.CDLL(REF_SO)
        sz = ctypes.c_size_t
        P = ctypes.c_void_p
        L.ref_obj_parse.argtypes = [ctypes.c_char_p, sz, P, ctypes.POINTER(sz), P, ctypes.POINTER(sz),
                                    P, ctypes.POINTER(sz), P, ctypes.POINTER(sz)]
        _REF = L
    return _REF


def ref_parse(text: bytes):
    L = ref_lib()
    n = [ctypes.c_size_t() for _ in range(4)]
    rc = L.ref_obj_parse(text, len(text), None, ctypes.byref(n[0]), None, ctypes.byref(n[1]), None,
                         ctypes.byref(n[2]), None, ctypes.byref(n[3]))
    assert rc == 0
    v = np.zeros(max(n[0].value, 1), np.float32)
    i = np.zeros(max(n[1].value, 1), np.uint32)
    t = np.zeros(max(n[2].value, 1), np.float32)
    m = np.zeros(max(n[3].value, 1), np.uint32)
    L.ref_obj_parse(text, len(text), v.ctypes.data, ctypes.byref(n[0]), i.ctypes.data, ctypes.byref(n[1]),
                    t.ctypes.data, ctypes.byref(n[2]), m.ctypes.data, ctypes.byref(n[3]))
    return v[: n[0].value], i[: n[1].value], t[: n[2].value], m[: n[3].value]


def _fmt(x, style, rng):
    if style == 0:
        return repr(float(x))
    if style == 1:
        return f"{x:.9e}"
    if style == 2:
        return f"{x:+.3E}"
    s = f"{x:.7f}"
    return s.replace("0.", ".", 1) if rng.random() < 0.5 else s


def _random_polygons(seed, n_faces=40):
    """Star-shaped and convex polygons of 3..14 corners in random planes, with
    jitter (non-planar) and varied number spellings."""
    rng = np.random.default_rng(seed)
    lines, nv = [], 0
    for _ in range(n_faces):
        k = int(rng.integers(3, 15))
        ang = np.sort(rng.uniform(0, 2 * np.pi, k))
        rad = rng.uniform(0.3, 2.0, k) if rng.random() < 0.6 else np.ones(k)
        pts = np.stack([np.cos(ang) * rad, np.sin(ang) * rad, rng.normal(0, 0.05, k)], 1)
        q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
        pts = pts @ q.T + rng.uniform(-5, 5, 3)
        if rng.random() < 0.3:
            pts = pts[::-1]
        style = int(rng.integers(0, 4))
        for p in pts:
            lines.append("v " + " ".join(_fmt(c, style, rng) for c in p))
        corners = [str(nv + j + 1) if rng.random() < 0.7 else str(j - k) for j in range(k)]
        if rng.random() < 0.3:
            corners = [c + "/" + str(1 + j % 3) for j, c in enumerate(corners)]
        lines.append("f " + " ".join(corners))
        nv += k
    lines = ["vt 0.5 0.5", "vt 0 1", "vt 1 0"] + lines
    return ("\n".join(lines) + "\n").encode()


def _combs(seed, n_faces=20):
    """Comb-shaped (deeply concave) polygons in the axis planes, exactly planar
    or jittered by 1e-3, some reversed, some with a repeated corner: the ear
    clipper's reflex, overlap and degenerate-cross branches."""
    rng = np.random.default_rng(seed)
    lines, nv = [], 0
    for _ in range(n_faces):
        k = int(rng.integers(2, 8))
        pts = []
        for j in range(k):
            pts += [(2 * j, 0), (2 * j + 1, rng.uniform(1, 4))]
        pts += [(2 * k, 0), (2 * k, -1), (0, -1)]
        if rng.random() < 0.3:
            pts = pts[::-1]
        ax = rng.permutation(3)
        for a, b in pts:
            p = [0.0, 0.0, 0.0]
            p[ax[0]], p[ax[1]] = a, b
            p[ax[2]] = float(rng.normal(0, 1e-3)) if rng.random() < 0.5 else 0.0
            lines.append("v %r %r %r" % tuple(float(c) for c in p))
        idx = list(range(nv + 1, nv + len(pts) + 1))
        if rng.random() < 0.3:
            idx.insert(2, idx[2])
        lines.append("f " + " ".join(map(str, idx)))
        nv += len(pts)
    return ("\n".join(lines) + "\n").encode()


CASES = dict(OBJ_CASES)
CASES["box.obj"] = open(scenes.BOX_OBJ, "rb").read()
for _s in range(6):
    CASES[f"random_polygons_{_s}"] = _random_polygons(_s)
    CASES[f"combs_{_s}"] = _combs(_s)


@pytest.mark.parametrize("case", sorted(CASES))
def test_restatements_match_reference_tinyobj(case):
    text = CASES[case]
    rv, ri, rt, rm = ref_parse(text)
    pv, pi, _, pt, pm = ptamd.Scene.parse_obj(text).arrays()
    ov, oi, ot = O.obj_parse(text)
    for name, v, i in (("product", pv, pi), ("oracle", ov, oi)):
        assert v.shape == rv.shape and np.array_equal(v.view(np.uint32), rv.view(np.uint32)), f"{name} vertices"
        assert np.array_equal(i, ri), f"{name} triangle index order"
    assert np.array_equal(pt.view(np.uint32), rt.view(np.uint32)) and np.array_equal(ot.view(np.uint32),
                                                                                    rt.view(np.uint32))
    assert np.array_equal(pm, rm)


def test_reference_loader_box_fixture():
    """The reference loader's box.obj: 8 vertices, 12 triangles, 14 uvs."""
    v, i, t, m = ref_parse(CASES["box.obj"])
    assert v.size == 24 and i.size == 36 and t.size == 28 and m.size == 12


def test_fuzzed_polygons_match_reference_tinyobj():
    """200 more generated files (both generators): product, oracle and the
    reference loader agree on every vertex bit and triangle index."""
    for seed in range(100, 200):
        for text in (_random_polygons(seed), _combs(seed)):
            rv, ri, _, rm = ref_parse(text)
            pv, pi, _, _, pm = ptamd.Scene.parse_obj(text).arrays()
            ov, oi, _ = O.obj_parse(text)
            assert np.array_equal(pv.view(np.uint32), rv.view(np.uint32)) and np.array_equal(pi, ri), seed
            assert np.array_equal(ov.view(np.uint32), rv.view(np.uint32)) and np.array_equal(oi, ri), seed
            assert np.array_equal(pm, rm), seed
