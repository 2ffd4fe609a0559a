"""The culled wide-BVH walk (csrc/wide_walk.h) against the oracle's exhaustive
traceRay (raytrace_comp.comp:159-204), on the CPU.

tests/wide_check.cpp compiles the walk's own step function for the host and
runs it ray by ray beside oracle_trace.  Every closest hit must have the
oracle's t bits and triangle (normal bits), every shadow query its
"!hit || t >= limit" answer (:359, :398).  The rays are chosen to stress the
cull bound: grazing rays nearly in a triangle's plane (|det| near the 1e-6
acceptance), origins on surfaces (the reference's +-1e-3 offsets), origins
inside boxes, axis-parallel directions (handed to the exact walk), and
shadow limits just around the hit distance.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oracle_lib
import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "discovering-path-tracer_amd", "csrc")
SO = os.path.join(ROOT, "tests", "_build", "libwide_check.so")
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        srcs = [os.path.join(ROOT, "tests", "wide_check.cpp"), os.path.join(CSRC, "scene", "wide_bvh.cpp")]
        deps = srcs + [os.path.join(CSRC, f) for f in ("wide_walk.h", "pt_isect.h", "pt_math.h")]
        oracle_lib.lib()   # builds liboracle.so if needed
        if not os.path.exists(SO) or any(os.path.getmtime(d) > os.path.getmtime(SO) for d in deps):
            os.makedirs(os.path.dirname(SO), exist_ok=True)
            subprocess.check_call(
                ["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__",
                 "-ffp-contract=off", "-fno-fast-math", "-I", CSRC, "-o", SO] + srcs +
                ["-L", os.path.join(ROOT, "oracle"), "-loracle", "-Wl,-rpath," + os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(SO)
        F32P = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
        U32P = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
        U64P = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
        I32P = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
        F64P = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
        sz = ctypes.c_size_t
        L.wide_info.argtypes = [F32P, sz, U32P, sz, F32P, sz, ctypes.c_int, I32P, ctypes.c_char_p, sz]
        L.wide_check.argtypes = [F32P, sz, U32P, sz, F32P, sz, ctypes.c_int, F32P, sz, F32P, U64P,
                                 ctypes.c_char_p, sz]
        L.wide_coeffs.argtypes = [F32P, F32P, F64P, F32P]
        L.wide_set_mode.argtypes = [ctypes.c_int]
        L.wide_set_variant.argtypes = [ctypes.c_int, ctypes.c_int]
        L.wide_dump.argtypes = [F32P, sz, U32P, sz, F32P, sz, ctypes.c_int, F32P, sz, I32P, ctypes.c_char_p, sz]
        L.wide_dump.restype = ctypes.c_longlong
        L.wide_counts.argtypes = [F32P, sz, U32P, sz, F32P, sz, ctypes.c_int, F32P, sz, I32P, I32P, ctypes.c_char_p,
                                  sz]
        _LIB = L
    return _LIB


def _scene(v, i):
    idx, nodes = oracle_lib.bvh_build(v, i)
    return np.ascontiguousarray(v, np.float32), idx, nodes


# the two ways the wide nodes group the reference's leaves (scene/wide_bvh.h)
WIDE_FROM_REFERENCE, WIDE_SAH = 0, 1
# (grouping, node bytes, queued leaf tests): the kernel's default is (SAH, 64,
# 2: queued, flushed wave-wide); 64-B nodes hold boxes rounded outward onto an 8-bit grid and test a
# leaf's exact box before its hit counts (wide_walk.h); queued: leaf hits are
# tested in flushes, as one lane of the trace kernel does (PT_WIDE_QUEUE)
BUILDS = pytest.mark.parametrize(
    "build", [(WIDE_SAH, 64, 1), (WIDE_SAH, 64, 0), (WIDE_SAH, 128, 1), (WIDE_SAH, 128, 0),
              (WIDE_FROM_REFERENCE, 64, 1), (WIDE_FROM_REFERENCE, 128, 0), (WIDE_SAH, 64, 2), (WIDE_SAH, 128, 2),
              (WIDE_FROM_REFERENCE, 64, 2)],
    ids=["sah-64-queue", "sah-64", "sah-128-queue", "sah-128", "reference_tree-64-queue", "reference_tree-128",
         "sah-64-waveflush", "sah-128-waveflush", "reference_tree-64-waveflush"])


def check(v, idx, nodes, rays, build=(WIDE_SAH, 64, 1)):
    L = lib()
    L.wide_set_mode(build[0])
    L.wide_set_variant(build[1], build[2])
    rays = np.ascontiguousarray(rays, np.float32)
    n = rays.size // 8
    out = np.zeros(4 * n, np.float32)
    st = np.zeros(8, np.uint64)
    err = ctypes.create_string_buffer(256)
    rc = L.wide_check(v, v.size, idx, idx.size // 3, nodes, nodes.size // 8, 0, rays, n, out, st, err, 256)
    assert rc == 0, err.value.decode()
    return out.reshape(n, 4), st


def _unit(a):
    a = np.asarray(a, np.float32)
    return (a / np.sqrt((a * a).sum(-1, keepdims=True))).astype(np.float32)


def make_rays(v, idx, n, seed, lo=-1.2, hi=1.2):
    """A mix of ray families (see the module docstring); n x 8 float32."""
    rng = np.random.default_rng(seed)
    V = v.reshape(-1, 3)
    T = idx.reshape(-1, 3)
    P = V[T]                                 # triangles x 3 x 3
    e1, e2 = P[:, 1] - P[:, 0], P[:, 2] - P[:, 0]
    nrm = _unit(np.cross(e1, e2))
    out = []
    k = n // 6
    # 1. random origins in / around the scene, random directions
    o = rng.uniform(lo * 1.5, hi * 1.5, (k, 3)).astype(np.float32)
    out.append((o, _unit(rng.normal(size=(k, 3)))))
    # 2. from a camera-like point outside towards random scene points
    o = np.tile(np.float32([0.3, 0.2, 3.0]), (k, 1))
    tgt = rng.uniform(lo, hi, (k, 3)).astype(np.float32)
    out.append((o, _unit(tgt - o)))
    # 3. from surface points (offset +-1e-3 along the normal, :355, :370) in random directions
    t = rng.integers(0, len(T), k)
    b = rng.dirichlet([1, 1, 1], k).astype(np.float32)
    sp = (P[t] * b[:, :, None]).sum(1)
    sgn = np.where(rng.random(k) < 0.5, 1e-3, -1e-3).astype(np.float32)[:, None]
    out.append(((sp + nrm[t] * sgn).astype(np.float32), _unit(rng.normal(size=(k, 3)))))
    # 4. grazing: nearly in a triangle's plane, aimed at it from far away
    t = rng.integers(0, len(T), k)
    b = rng.dirichlet([1, 1, 1], k).astype(np.float32)
    tp = (P[t] * b[:, :, None]).sum(1)
    inplane = _unit(np.cross(nrm[t], rng.normal(size=(k, 3))))
    tilt = (10.0 ** rng.uniform(-7, -2, k)).astype(np.float32)[:, None] * np.where(rng.random((k, 1)) < .5, 1, -1)
    d = _unit(inplane + nrm[t] * tilt)
    dist = rng.uniform(0.01, 2.0, (k, 1)).astype(np.float32)
    out.append(((tp - d * dist).astype(np.float32), d))
    # 5. axis-parallel and nearly axis-parallel directions (exact hand-back / huge invDir)
    o = rng.uniform(lo, hi, (k, 3)).astype(np.float32)
    d = np.zeros((k, 3), np.float32)
    ax = rng.integers(0, 3, k)
    d[np.arange(k), ax] = np.where(rng.random(k) < 0.5, 1.0, -1.0)
    tiny = rng.random(k) < 0.5
    d[tiny] += rng.normal(size=(int(tiny.sum()), 3)).astype(np.float32) * np.float32(1e-30)
    out.append((o, d))
    # 6. from inside leaf boxes: triangle centroids, random directions
    t = rng.integers(0, len(T), n - 5 * k)
    out.append((P[t].mean(1).astype(np.float32), _unit(rng.normal(size=(n - 5 * k, 3)))))
    o = np.concatenate([a for a, _ in out]).astype(np.float32)
    d = np.concatenate([b for _, b in out]).astype(np.float32)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = o
    rays[:, 3:6] = d
    return rays


def run_scene(v, i, n_rays, seed, build=(WIDE_SAH, 64, 1)):
    v, idx, nodes = _scene(v, i)
    rays = make_rays(v, idx, n_rays, seed)
    out, st = check(v, idx, nodes, rays, build)     # closest
    assert st[0] == 0, f"closest-hit mismatches: {int(st[0])} (first ray {int(st[7])}: {rays[int(st[7])]})"
    # shadow queries with limits around the closest hit (and far / negative / NaN ones)
    rng = np.random.default_rng(seed + 1)
    sh = rays.copy()
    sh[:, 6] = 1.0
    t = out[:, 2]
    hit = out[:, 3] > 0
    jitter = rng.choice(np.float32([0.0, 1e-7, -1e-7, 1e-4, -1e-4, 0.1, -0.5]), len(t))
    lim = np.where(hit, t * (np.float32(1) + jitter.astype(np.float32)), rng.uniform(0.1, 5, len(t)))
    special = rng.random(len(t))
    lim = np.where(special < 0.02, np.float32(np.nan), lim)
    lim = np.where((special >= 0.02) & (special < 0.04), np.float32(-1.0), lim)
    lim = np.where((special >= 0.04) & (special < 0.06), np.float32(1e30), lim)
    sh[:, 7] = lim.astype(np.float32)
    _, st2 = check(v, idx, nodes, sh, build)
    assert st2[1] == 0, f"shadow mismatches: {int(st2[1])} (first ray {int(st2[7])}: {sh[int(st2[7])]})"
    return st, st2


def test_coefficients_bound_shape():
    """Small triangles get tight bounds (c1 just below 1, eps tiny); huge ones
    give up culling."""
    co = np.zeros(4, np.float64)
    node = np.zeros(4, np.float32)
    assert lib().wide_coeffs(np.float32([0.02, 0, 0]), np.float32([0, 0.02, 0.001]), co, node) == 0
    k1, k2, eps0, eps1 = co
    assert 0 < k1 < 1e-3 and 0 < k2 < 1e-3 and eps0 < 1e-5 and eps1 < 1e-3
    c1, E0, E1, _ = node
    assert 0.999 < c1 < 1.0 and E0 >= eps0 and E1 >= eps1 and E1 >= k2 / c1
    # the device evaluates c1' (t_near - E' Smax ...) with the (1 - 2^-20)
    # t_near factor folded into the constants (node_cull_consts): c1' is at
    # most c1 k and each E' at least E / k, so the threshold is never above
    # c1 (t_near k - E Smax ...) of the unfolded bound
    k, u = 1.0 - 2.0 ** -20, 2.0 ** -24
    c1_unfolded = (1.0 - k1) / (1.0 + 3 * u / (1 - 3 * u)) * k
    assert float(c1) <= c1_unfolded * k
    assert float(E0) >= eps0 * (1.0 + 2.0 ** -18) / k
    assert float(E1) >= max(eps1, k2 / c1_unfolded) * (1.0 + 2.0 ** -18) / k
    assert lib().wide_coeffs(np.float32([2, 0, 0]), np.float32([0, 2, 0]), co, node) == 1


@BUILDS
def test_wide_walk_random_cloud(build):
    v, i = scenes.random_triangles(20000, seed=7)
    st, st2 = run_scene(v, i, 60000, seed=11, build=build)
    # far fewer node fetches than the exhaustive walk, and (4-wide) never more
    # triangle tests; the 8-wide walk's leaf tests may run up to a queue's
    # worth behind its best hit (a node brings up to eight), so a few more
    assert st[3] < st[5] / 3, (int(st[3]), int(st[5]))
    assert st[4] <= st[6] * (1.02 if build[1] == 80 else 1.0), (int(st[4]), int(st[6]))
    assert st[2] > 0   # axis-parallel rays went to the exact walk


@BUILDS
def test_wide_walk_displaced_sphere(build):
    v, i = scenes.displaced_sphere(subdiv=4)
    run_scene(v, i, 60000, seed=12, build=build)


@BUILDS
def test_wide_walk_grid_ties(build):
    """Axis-aligned coplanar quads: equal t across triangles, tie-break by visit rank."""
    v, i = scenes.grid_mesh(8)
    run_scene(v, i, 40000, seed=13, build=build)


@BUILDS
def test_wide_walk_box_big_triangles(build):
    v, i, _ = oracle_lib.obj_parse(open(scenes.BOX_OBJ, "rb").read())
    run_scene(v, i, 40000, seed=14, build=build)


@BUILDS
def test_wide_walk_dense_tiny_cloud(build):
    """A dense cloud of small triangles: many near-equal hit distances, and
    culling cuts the triangle tests."""
    v, i = scenes.random_triangles(30000, seed=9, spread=0.2, size=0.004)
    st, _ = run_scene(v, i, 40000, seed=15, build=build)
    # (queued tests cull against a best hit that lags by up to a queue's worth;
    # an 8-wide node queues up to eight leaves at once)
    assert st[4] < (0.8 if not build[2] else 0.97 if build[1] == 80 else 0.95) * st[6], (int(st[4]), int(st[6]))


def test_wide_info_and_refusals():
    v, i = scenes.random_triangles(1000, seed=3)
    v, idx, nodes = _scene(v, i)
    info = np.zeros(2, np.int32)
    err = ctypes.create_string_buffer(256)
    L = lib()
    assert L.wide_info(v, v.size, idx, idx.size // 3, nodes, nodes.size // 8, 0, info, err, 256) == 0
    assert 0 < info[0] < 1000 and 1 < info[1] < 64
    bad = nodes.copy().reshape(-1, 8)
    bad[1, 0] = bad[0, 0] - 1.0   # a child box sticking out of the root
    assert L.wide_info(v, v.size, idx, idx.size // 3, bad.reshape(-1), nodes.size // 8, 0, info, err, 256) == 1
    assert b"contain" in err.value


def _dump(v, idx, nodes, build):
    L = lib()
    L.wide_set_mode(build)
    nt = idx.size // 3
    cap = 32 * (nt + 8)
    out = np.zeros(cap, np.float32)
    rt = np.zeros(nt, np.int32)
    err = ctypes.create_string_buffer(256)
    n = L.wide_dump(v, v.size, idx, nt, nodes, nodes.size // 8, 0, out, cap, rt, err, 256)
    assert n > 0, err.value.decode()
    return out[:n].reshape(-1, 32).copy(), rt


@pytest.mark.parametrize("build", [WIDE_SAH, WIDE_FROM_REFERENCE], ids=["sah", "reference_tree"])
def test_wide_tree_invariants(build):
    """The premises of the walk's exactness (wide_walk.h), on the built tree:
    every leaf child carries the reference's leaf box bitwise and every leaf
    rank appears once; every inner child's box contains every leaf box below
    it; the SAH build is deterministic (threaded, same tree twice)."""
    sv, si = scenes.displaced_sphere(subdiv=4)
    v, idx, nodes = _scene(sv, si)
    W, rank_tri = _dump(v, idx, nodes, build)
    if build == WIDE_SAH:
        W2, rank_tri2 = _dump(v, idx, nodes, build)
        assert np.array_equal(W.view(np.uint32), W2.view(np.uint32)) and np.array_equal(rank_tri, rank_tri2)
    N = nodes.reshape(-1, 8)
    # reference leaves in right-first DFS order -> their boxes by rank
    order, st = [], [0]
    while st:
        k = st.pop()
        left, right = N[k, 3], N[k, 7]
        if left == -1:
            order.append(k)
        else:
            st += [int(left), int(right)]
    leaf_lo = N[order, 0:3]
    leaf_hi = N[order, 4:7]
    assert np.array_equal(N[order, 7].astype(np.int64), rank_tri.astype(np.int64))
    refs = W[:, 24:28].copy().view(np.int32)
    lo = np.stack([W[:, 0:4], W[:, 8:12], W[:, 16:20]], -1)    # node, child, axis
    hi = np.stack([W[:, 4:8], W[:, 12:16], W[:, 20:24]], -1)
    seen = np.zeros(len(order), np.int32)

    def leaves_below(w):
        out = []
        for j in range(4):
            r = int(refs[w, j])
            if r == -2 ** 31:
                continue
            out += [~r] if r < 0 else leaves_below(r)
        return out

    for w in range(len(W)):
        for j in range(4):
            r = int(refs[w, j])
            if r == -2 ** 31:
                continue
            if r < 0:
                seen[~r] += 1
                assert np.array_equal(lo[w, j].view(np.uint32), leaf_lo[~r].view(np.uint32))
                assert np.array_equal(hi[w, j].view(np.uint32), leaf_hi[~r].view(np.uint32))
            elif w < 64 or w % 97 == 0:   # containment of every leaf below (a sample of inner nodes)
                below = leaves_below(r)
                assert (leaf_lo[below] >= lo[w, j]).all() and (leaf_hi[below] <= hi[w, j]).all()
    assert (seen == 1).all()
