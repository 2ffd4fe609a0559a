"""Host side of the product without a GPU: the C-ABI library loads and exports
every symbol include/pathtracer.h declares, and the native scene layer (OBJ
ingest, BVH builder, light packing, camera) matches the oracle byte for byte."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle_lib as O
import ptamd
import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "pathtracer.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(pt_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_declared_symbol():
    decl = _declared_symbols()
    assert len(decl) >= 30
    L = ctypes.CDLL(ptamd.LIB_PATH)
    missing = [s for s in decl if not hasattr(L, s)]
    assert not missing, missing
    assert sorted(decl) == sorted(ptamd.EXPORTS)
    assert ptamd.lib().pt_abi_version() == 3   # 3: round 6 (pathtracer.h ABI history)


def test_no_gpu_fails_loudly():
    """The product never falls back to the CPU: without a device pt_create errors."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import ptamd\n"
            "try:\n    ptamd.Renderer(0)\nexcept ptamd.PTError as e:\n    print('ERR', e)\nelse:\n    print('OK')\n"
            % os.path.join(ROOT, "discovering-path-tracer_amd"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120).stdout
    assert out.startswith("ERR") or out.startswith("OK")   # OK only on a GPU box


def _product(v, i, int_bits=False, threads=0):
    s = ptamd.Scene.from_arrays(v, i).build_bvh(int_bits=int_bits, threads=threads)
    pv, pi, pn, _, _ = s.arrays()
    return pi, pn


@pytest.mark.parametrize("name", ["box", "random1", "random2", "random3", "random1000", "grid", "sphere"])
def test_bvh_byte_identical_to_oracle(name):
    if name == "box":
        v, i, _ = O.obj_parse(open(scenes.BOX_OBJ, "rb").read())
    elif name.startswith("random"):
        v, i = scenes.random_triangles(int(name[6:]), seed=5)
    elif name == "grid":
        v, i = scenes.grid_mesh(8)
    else:
        v, i = scenes.displaced_sphere(3)
    oi, on = O.bvh_build(v, i)
    pi, pn = _product(v, i)
    assert np.array_equal(pi, oi)
    assert np.array_equal(pn.reshape(-1).view(np.uint32), on.view(np.uint32))


def test_bvh_parallel_build_identical():
    """>= 200k triangles takes the multi-threaded subtree path."""
    v, i = scenes.random_triangles(300000, seed=9)
    oi, on = O.bvh_build(v, i)
    for threads in (1, 8):
        pi, pn = _product(v, i, threads=threads)
        assert np.array_equal(pi, oi)
        assert np.array_equal(pn.reshape(-1).view(np.uint32), on.view(np.uint32))


def test_bvh_int_bits_encoding():
    v, i = scenes.random_triangles(777, seed=2)
    fi, fn = _product(v, i)
    ii, inn = _product(v, i, int_bits=True)
    assert np.array_equal(fi, ii)
    assert np.array_equal(fn[:, [0, 1, 2, 4, 5, 6]], inn[:, [0, 1, 2, 4, 5, 6]])
    w = inn[:, [3, 7]].copy().view(np.int32)
    assert np.array_equal(w, fn[:, [3, 7]].astype(np.int32))


def test_bvh_errors():
    with pytest.raises(ptamd.PTError):
        ptamd.Scene.from_arrays(np.zeros(9, np.float32), np.zeros(0, np.uint32)).build_bvh()
    with pytest.raises(ptamd.PTError):
        ptamd.Scene.from_arrays(np.zeros(9, np.float32), np.array([0, 1, 5], np.uint32)).build_bvh()
    with pytest.raises(ptamd.PTError):
        ptamd.Scene.from_arrays(np.zeros(9, np.float32), np.array([0, 1], np.uint32))


OBJ_CASES = {
    "formats": b"v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvt 0 0\nvn 0 0 1\n"
               b"f 1/1/1 2/1/1 3/1/1\nf 1//1 3//1 4//1\nf -4 -2 -1\n",
    "quads_both_diagonals": b"v 0 0 0\nv 2 0 0\nv 2 1 0\nv 0 1 0\nv 0 0 1\nv 1 0 1\nv 3 1 1\nv 0 1 1\n"
                            b"f 1 2 3 4\nf 5 6 7 8\n",
    "numbers": b"v 1.5e1 -.25 +3\nv 0.000000012345678 1E-3 -0\nv 123456789.123456789 7 1e+2\n"
               b"v 0.1 0.2 0.3\nf 1 2 3\nf 2 3 4\n",
    "shapes_and_comments": b"# c\no A\nv 0 0 0\nv 1 0 0\nv 0 1 0\ng B\nusemtl x\nv 0 0 1\n  f 1 2 3\nf 2 3 4\n",
    "crlf": b"v 0 0 0\r\nv 1 0 0\r\nv 0 1 0\r\nf 1 2 3\r\n",
    # n-gons: tinyobj ear clipping (tiny_obj_loader.h:1740-1955)
    "ngon_convex_xy": b"v 0 0 0\nv 2 0 0\nv 3 1 0\nv 1 3 0\nv -1 1 0\nf 1 2 3 4 5\n",
    "ngon_concave_offset": b"v 1 1 0\nv 5 1 0\nv 5 5 0\nv 3 2 0\nv 1 5 0\nv 0.5 3 0\nf 1 2 3 4 5 6\nf 6 5 4 3 2 1\n",
    "ngon_planes": b"v 0 0 0\nv 0 2 0\nv 0 3 1\nv 0 1 3\nv 0 -1 1\nv 1 0 0\nv 3 0 1\nv 2 0 3\nv 0.5 0 2\nv 0 0 1\n"
                   b"f 1 2 3 4 5\nf 6 7 8 9 10 1\n",
    "ngon_collinear_start": b"v 0 0 0\nv 1 0 0\nv 2 0 0\nv 2 2 1\nv 0 2 1\nv -1 1 0.5\nv -0.5 0.2 0.1\nf 1 2 3 4 5 6 7\n",
    "ngon_star": b"v 0 3 0\nv 1 1 0\nv 3 1 0\nv 1.5 -0.5 0\nv 2 -3 0\nv 0 -1.5 0\nv -2 -3 0\nv -1.5 -0.5 0\n"
                 b"v -3 1 0\nv -1 1 0\nf 1 2 3 4 5 6 7 8 9 10\n",
}


@pytest.mark.parametrize("case", sorted(OBJ_CASES))
def test_obj_ingest_matches_oracle(case):
    text = OBJ_CASES[case]
    ov, oi, ot = O.obj_parse(text)
    v, i, _, uv, m = ptamd.Scene.parse_obj(text).arrays()
    assert np.array_equal(v.view(np.uint32), ov.view(np.uint32))
    assert np.array_equal(i, oi)
    assert np.array_equal(uv, ot)
    assert m.size == i.size // 3 and np.all(m == 0)


def test_obj_box_and_errors():
    v, i, _, uv, m = ptamd.Scene.load_obj(scenes.BOX_OBJ).arrays()
    assert v.size == 24 and i.size == 36 and uv.size == 28 and m.size == 12
    with pytest.raises(ptamd.PTError):
        ptamd.Scene.load_obj("/nonexistent.obj")
    with pytest.raises(ptamd.PTError):
        ptamd.Scene.parse_obj(b"v 0 0 0\nf 1 2 3\n")   # index out of range


def test_ngon_ear_clipping_known_answer():
    # convex pentagon with corner 0 at the origin: every ear is accepted at
    # guess 0, so tinyobj produces the fan (0,1,2) (0,2,3) (0,3,4)
    v, i, _, _, m = ptamd.Scene.parse_obj(OBJ_CASES["ngon_convex_xy"]).arrays()
    assert i.tolist() == [0, 1, 2, 0, 2, 3, 0, 3, 4] and m.size == 3
    # a 10-corner star keeps every corner and yields n-2 triangles
    v, i, _, _, m = ptamd.Scene.parse_obj(OBJ_CASES["ngon_star"]).arrays()
    assert i.size == 3 * 8 and sorted(set(i.tolist())) == list(range(10))


def test_light_and_camera_packing():
    l = ptamd.pack_light([0, 2, 0], [0, -3, 0], [10, 10, 10], [2.5, 2.5])
    assert l.tolist() == scenes.REFERENCE_LIGHT.tolist()     # normal normalized (Light.cpp:25)
    assert np.array_equal(ptamd.default_camera().view(np.uint32), scenes.DEFAULT_CAMERA.view(np.uint32))


def test_partition_masks_tile_the_frame():
    W, H = 100, 37
    for n in (1, 2, 3, 8):
        m = np.stack([ptamd.partition_owned(W, H, n, r) for r in range(n)])
        assert np.all(m.sum(0) == 1)


def test_scene_cache_round_trip(tmp_path):
    s = ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh()
    p = tmp_path / "box.ptscene"
    s.save(p)
    t = ptamd.Scene.load_cache(p)
    for a, b in zip(s.arrays(), t.arrays()):
        assert a.dtype == b.dtype and np.array_equal(a.view(np.uint32), b.view(np.uint32))
    # int-encoded trees keep their flag; a bigger random mesh round-trips too
    tv, ti = scenes.random_triangles(5000, seed=3)
    s2 = ptamd.Scene.from_arrays(tv, ti).build_bvh(int_bits=True)
    s2.save(tmp_path / "r.ptscene")
    t2 = ptamd.Scene.load_cache(tmp_path / "r.ptscene")
    assert all(np.array_equal(a.view(np.uint32), b.view(np.uint32)) for a, b in zip(s2.arrays(), t2.arrays()))
    # corruption, truncation, foreign files and missing files are errors
    raw = bytearray(p.read_bytes())
    raw[100] ^= 1
    (tmp_path / "bad.ptscene").write_bytes(bytes(raw))
    (tmp_path / "short.ptscene").write_bytes(p.read_bytes()[:-9])
    for bad in ("bad.ptscene", "short.ptscene"):
        with pytest.raises(ptamd.PTError):
            ptamd.Scene.load_cache(tmp_path / bad)
    with pytest.raises(ptamd.PTError):
        ptamd.Scene.load_cache(scenes.BOX_OBJ)
    with pytest.raises(ptamd.PTError):
        ptamd.Scene.load_cache(tmp_path / "missing.ptscene")
    with pytest.raises(ptamd.PTError):
        ptamd.Scene.load_obj(scenes.BOX_OBJ).save(tmp_path / "nobvh.ptscene")   # BVH not built


def test_write_image_png_and_pfm(tmp_path):
    import struct
    import zlib
    W, H = 70, 9
    rgba = np.zeros((H, W, 4), np.float32)
    rgba[..., 0] = np.linspace(-0.5, 1.5, W)[None, :]
    rgba[..., 1] = np.linspace(0, 1, H)[:, None]
    rgba[..., 2] = 0.0031308
    ptamd.write_image(tmp_path / "a.png", rgba, W, H, "png")
    data = (tmp_path / "a.png").read_bytes()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, chunks = 8, {}
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        typ, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + body)
        chunks[typ] = body
        pos += 12 + n
    assert struct.unpack(">IIBBBBB", chunks[b"IHDR"]) == (W, H, 8, 2, 0, 0, 0)
    raw = np.frombuffer(zlib.decompress(chunks[b"IDAT"]), np.uint8).reshape(H, 1 + 3 * W)
    assert np.all(raw[:, 0] == 0)
    img = raw[:, 1:].reshape(H, W, 3)[::-1]          # top row = last buffer row
    lin = np.clip(rgba[..., :3].astype(np.float64), 0, 1)
    srgb = np.where(lin <= 0.0031308, 12.92 * lin, 1.055 * lin ** (1 / 2.4) - 0.055)
    assert np.max(np.abs(img.astype(int) - np.floor(srgb * 255 + 0.5).astype(int))) <= 1
    ptamd.write_image(tmp_path / "a.pfm", rgba, W, H, "pfm")
    pfm = (tmp_path / "a.pfm").read_bytes()
    head = f"PF\n{W} {H}\n-1.0\n".encode()
    assert pfm.startswith(head)
    body = np.frombuffer(pfm[len(head):], np.float32).reshape(H, W, 3)
    assert np.array_equal(body, rgba[..., :3])
    with pytest.raises(ptamd.PTError):
        ptamd.write_image(tmp_path / "no_such_dir" / "x.png", rgba, W, H)


def test_partition_spreads_centred_geometry_evenly():
    """The rotated tile order (pt_device.h tile_block) deals each of 8 ranks
    an even share of box.obj's live rectangle at 1080p; plain row-major order
    put 5.7 % more on rank 0 (column stripes, 120 % 8 == 0)."""
    W, H = 1920, 1080
    rects = ptamd.primary_cull_rects(scenes.DEFAULT_CAMERA, W, H, [-1, -1, -1], [1, 1, 1], scenes.REFERENCE_LIGHT)
    x0, x1, y0, y1 = rects[0]
    xs = 2 * np.arange(W, dtype=np.float32) / np.float32(W) - 1
    ys = 2 * np.arange(H, dtype=np.float32) / np.float32(H) - 1
    live = ((xs >= x0) & (xs <= x1))[None, :] & ((ys >= y0) & (ys <= y1))[:, None]
    for n in (2, 4, 8):
        share = np.array([np.count_nonzero(live & ptamd.partition_owned(W, H, n, r)) for r in range(n)], float)
        assert share.max() / share.mean() < 1.01, (n, share)


def test_partition_slots_masks_tile_the_frame():
    """pt_set_partition_slots shares: every pixel owned exactly once, and the
    shares follow the slot counts (box 1080p, the root with 6 of 62 slots)."""
    W, H = 1920, 1080
    slots = [6] + [8] * 7
    m = np.stack([ptamd.partition_owned(W, H, 8, r, slots) for r in range(8)])
    assert np.all(m.sum(0) == 1)
    share = m.reshape(8, -1).mean(1)
    assert abs(share[0] / share[1:].mean() - 6 / 8) < 0.02
    for n in (2, 3):   # one slot each is the plain partition
        for r in range(n):
            assert np.array_equal(ptamd.partition_owned(W, H, n, r, [1] * n), ptamd.partition_owned(W, H, n, r))


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_multi_device_members_cover_the_frame_once(n):
    """pt_create_multi gives member r the tiles of rank r of an n-way
    pt_set_partition: over the members every pixel is rendered exactly once
    (the frame on the first device is then the single-GPU frame), for ragged
    frame sizes too."""
    for W, H in ((1920, 1080), (70, 45), (17, 300)):
        cover = np.zeros((H, W), np.int32)
        for r in range(n):
            cover += ptamd.partition_owned(W, H, n, r).astype(np.int32)
        assert np.all(cover == 1), (n, W, H)


def test_create_multi_argument_errors_without_a_gpu():
    """Bad member lists fail with an error, never a crash (this container has
    no GPU: a valid list fails at device enumeration)."""
    import ctypes
    L = ptamd.lib()
    out = ctypes.c_void_p()
    none = np.zeros(0, np.int32)
    assert L.pt_create_multi(None, 2, ctypes.byref(out)) < 0
    assert L.pt_create_multi(none.ctypes.data, 0, ctypes.byref(out)) < 0
    devs = np.array([0, 0], np.int32)
    rc = L.pt_create_multi(devs.ctypes.data, 2, ctypes.byref(out))
    assert rc < 0 and not out.value
    assert L.pt_last_error()


def test_gather_ceilings_are_the_best_measured_patterns():
    """the node-fetch rooflines price against the best
    rate any measured access pattern reached (tools/gather_roof.hip mlp,
    profiles/r05), and config 5's composed ceiling min(R_L2 / h, R_miss /
    (1 - h)) is at least each resource's own rate."""
    import json
    import sys
    sys.path.insert(0, ROOT)
    import bench
    rows = [json.loads(x) for x in open(os.path.join(ROOT, bench.GATHER_FILE)) if x.startswith("{")]
    l2 = max(d["Grec_per_s"] for d in rows if d["case"] == "l2_4MB")
    hbm = max(d["Grec_per_s"] for d in rows if d["case"] == "hbm1GB")
    for wl in ("sphere_1080p8", "sphere_4k16_d8_refcam"):
        g = bench.gather_roofline(wl)
        assert g["bound"] == "l2_gather" and g["Grec_per_s"] == l2
    g = bench.gather_roofline("synthetic10M_1080p8_refcam")   # no profile: the loosest true ceiling
    assert g["bound"] == "hbm_gather" and g["Grec_per_s"] == l2
    for h in (0.1, 0.5, 0.9):
        g = bench.gather_roofline("synthetic10M_1080p8", ("p", {"trace_kernel_l2": {"hit_fraction": h}}))
        assert g["Grec_per_s"] >= hbm - 1e-6 and g["Grec_per_s"] >= min(l2, hbm / (1 - h)) - 1e-2
        assert abs(g["Grec_per_s"] - min(l2 / h, hbm / (1 - h))) < 0.01
