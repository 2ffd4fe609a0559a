"""Deterministic test/bench scenes and the reference's fixed inputs."""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BOX_OBJ = os.path.join(ROOT, "tests", "golden", "box.obj")

# Camera.cpp:4-10 / Camera.h:34-36 default orbit camera as the std140 UBO.
DEFAULT_CAMERA = np.array([0, 0, 5, 0, 0, 0, -1, 0, 0, 1, 0, 0, 60, 0, 0, 0], np.float32)
# VulkanRayTracer.cpp:149-162 light, packed as Light.cpp:16-33 (normal already unit).
REFERENCE_LIGHT = np.array([0, 2, 0, 0, 0, -1, 0, 0, 10, 10, 10, 0, 2.5, 2.5, 0, 0], np.float32)


def camera(pos, up=(0, 1, 0), fov=60.0):
    """UBO for a camera at `pos` looking at the origin (Camera::getDirection)."""
    p = np.array(pos, np.float64)
    d = (0.0 - p) / np.linalg.norm(p)
    ubo = np.zeros(16, np.float32)
    ubo[0:3] = p
    ubo[4:7] = d
    ubo[8:11] = up
    ubo[12] = fov
    return ubo


def random_triangles(n, seed=42, spread=1.0, size=0.01):
    """SURVEY.md §8d config 5 generator: centroids ~U[-1,1]^3, vertex offsets
    ~U[-size,size]^3, unshared vertices."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(-spread, spread, (n, 1, 3)).astype(np.float32)
    off = rng.uniform(-size, size, (n, 3, 3)).astype(np.float32)
    v = (c + off).astype(np.float32).reshape(-1)
    idx = np.arange(3 * n, dtype=np.uint32)
    return v, idx


def grid_mesh(n=8, seed=0):
    """Axis-aligned quads on a grid: many equal centroid keys, exercising the
    unstable sort's tie order."""
    rng = np.random.default_rng(seed)
    verts, idx = [], []
    for i in range(n):
        for j in range(n):
            z = float(rng.integers(0, 3)) * 0.25 - 0.25
            base = len(verts)
            x0, y0 = -1 + 2 * i / n, -1 + 2 * j / n
            x1, y1 = x0 + 2 / n, y0 + 2 / n
            verts += [(x0, y0, z), (x1, y0, z), (x1, y1, z), (x0, y1, z)]
            idx += [base, base + 1, base + 2, base, base + 2, base + 3]
    return np.array(verts, np.float32).reshape(-1), np.array(idx, np.uint32)


def displaced_sphere(subdiv=5, seed=3):
    """Stand-in for the missing Sylveon.obj: an
    icosphere with radial noise — deep BVH, divergent secondary rays."""
    t = (1.0 + 5 ** 0.5) / 2
    V = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    F = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2),
         (10, 7, 6), (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11),
         (6, 2, 10), (8, 6, 7), (9, 8, 1)]
    V = [np.array(v, np.float64) / np.linalg.norm(v) for v in V]
    for _ in range(subdiv):
        cache, nf = {}, []

        def mid(a, b):
            k = (min(a, b), max(a, b))
            if k not in cache:
                m = V[a] + V[b]
                V.append(m / np.linalg.norm(m))
                cache[k] = len(V) - 1
            return cache[k]

        for a, b, c in F:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        F = nf
    V = np.array(V)
    rng = np.random.default_rng(seed)
    r = 1.0 + 0.08 * rng.standard_normal(len(V))
    V = (V * r[:, None]).astype(np.float32)
    return V.reshape(-1), np.array(F, np.uint32).reshape(-1)
