"""Primary-ray culling (pt_primary_cull_rects): a pixel outside
every rectangle must have no primary ray that reaches the root box or a light.

CPU tests: the Box-Muller radius bound the rectangles rest on, extreme-ray
probes of culled pixels (aperture and jitter at their bounds), and oracle
renders whose culled pixels must come out exactly (0,0,0,1).
"""
import itertools

import numpy as np
import pytest

import oracle_lib
import ptamd
import scenes

RG = 13.25   # Box-Muller radius bound used by the host code


@pytest.fixture(scope="module")
def box():
    v, i, _ = oracle_lib.obj_parse(open(scenes.BOX_OBJ, "rb").read())
    ri, nodes = oracle_lib.bvh_build(v, i)
    return v, ri, nodes


def test_gauss_radius_bound():
    # u1 = max(1e-38, u) (raytrace_comp.comp:220): the largest radius is at 1e-38
    lg = oracle_lib.math(0, np.array([1e-38, 2.0 ** -32, 0.5], np.float32))
    r = np.sqrt(np.float32(-2.0) * lg)
    assert r[0] < RG and r[0] > 13.2
    assert np.all(r[1:] < r[0])
    # |sin|, |cos| never exceed 1 on the shader's argument range [0, 2pi]
    th = np.linspace(0, 2 * np.pi, 200001, dtype=np.float32)
    assert np.all(np.abs(oracle_lib.math(2, th)) <= 1.0)
    assert np.all(np.abs(oracle_lib.math(3, th)) <= 1.0)


def _frame(cam):
    cpos, cdir, cup, fov = cam[0:3].astype(np.float64), cam[4:7].astype(np.float64), cam[8:11].astype(np.float64), float(cam[12])
    right = np.cross(cdir, -cup)
    right /= np.linalg.norm(right)
    up = np.cross(right, cdir)
    up /= np.linalg.norm(up)
    return cpos, cdir, right, up, np.tan(np.radians(fov * 0.5))


def _rays(cam, W, H, px, py, ox, oy, jx, jy):
    """Primary rays of raytrace_comp.comp:430-460 for given aperture/jitter draws (float64)."""
    cpos, cdir, right, up, T = _frame(cam)
    A = W / H
    ndcx = (2.0 * px / W - 1.0) + jx * 0.5 / W
    ndcy = (2.0 * py / H - 1.0) + jy * 0.5 / H
    o = cpos + right * ox + up * oy
    b = cdir - right * (ndcx * T * A) - up * (ndcy * T)
    b /= np.linalg.norm(b)
    d = cpos + 3.0 * b - o
    return o, d / np.linalg.norm(d)


def _slab_hit(o, d, lo, hi):
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t0 = (lo - o) * inv
        t1 = (hi - o) * inv
    tmin = np.nanmax(np.fmin(t0, t1))
    tmax = np.nanmin(np.fmax(t0, t1))
    return tmin <= tmax and tmax >= 0


def _light_hit(o, d, L):
    pos, n = L[0:3].astype(np.float64), L[4:7].astype(np.float64)
    nn = n / np.linalg.norm(n)
    basis = np.array([0.0, 1.0, 0.0]) if abs(nn[1]) < 0.999 else np.array([1.0, 0.0, 0.0])
    r = np.cross(nn, basis)
    r /= np.linalg.norm(r)
    u = np.cross(r, nn)
    den = np.dot(n, d)
    if abs(den) < 1e-4:
        return False
    t = np.dot(n, pos - o) / den
    if t <= 0:
        return False
    th = o + d * t - pos
    return abs(np.dot(th, r)) <= L[12] * 0.5 and abs(np.dot(th, u)) <= L[13] * 0.5


def _culled_mask(rects, W, H):
    px = np.arange(W, dtype=np.float32)
    py = np.arange(H, dtype=np.float32)
    nx = (np.float32(2.0) * px / np.float32(W)) - np.float32(1.0)
    ny = (np.float32(2.0) * py / np.float32(H)) - np.float32(1.0)
    live = np.zeros((H, W), bool)
    for x0, x1, y0, y1 in rects:
        live |= ((ny >= y0) & (ny <= y1))[:, None] & ((nx >= x0) & (nx <= x1))[None, :]
    return ~live


TWO_LIGHTS = np.concatenate([scenes.REFERENCE_LIGHT,
                             np.array([1.5, 0.5, 2.0, 0, -1, 0, 0, 0, 3, 2, 1, 0, 0.5, 1.0, 0, 0], np.float32)])

CASES = [
    ("default", scenes.DEFAULT_CAMERA, 96, 54, scenes.REFERENCE_LIGHT),
    ("orbit", scenes.camera((3.0, 2.0, 4.0)), 80, 60, scenes.REFERENCE_LIGHT),
    ("far_wide", scenes.camera((0.0, 0.5, 12.0), fov=100.0), 64, 64, TWO_LIGHTS),
    ("narrow", scenes.camera((1.0, -1.0, 7.0), fov=20.0), 70, 40, TWO_LIGHTS),
    ("tiny", scenes.DEFAULT_CAMERA, 17, 13, scenes.REFERENCE_LIGHT),
    ("tilted_up", np.array([0, 0, 14, 0, 0, 0, -2, 0, 0.3, 1, 0.2, 0, 45, 0, 0, 0], np.float32), 64, 48,
     scenes.REFERENCE_LIGHT),
]


@pytest.mark.parametrize("name,cam,W,H,lights", CASES, ids=[c[0] for c in CASES])
def test_culled_pixels_have_no_reaching_primary_ray(name, cam, W, H, lights):
    lo, hi = np.full(3, -1.0, np.float32), np.full(3, 1.0, np.float32)   # box.obj root
    rects = ptamd.primary_cull_rects(cam, W, H, lo, hi, lights)
    assert rects is not None
    culled = _culled_mask(rects, W, H)
    assert culled.any() and not culled.all()
    rho, J = 0.02 * RG, RG
    probes = list(itertools.product((-rho, 0.0, rho), (-rho, 0.0, rho), (-J, 0.0, J), (-J, 0.0, J)))
    rnd = np.random.default_rng(7)
    L = np.asarray(lights, np.float32).reshape(-1, 16)
    ys, xs = np.nonzero(culled)
    pick = rnd.choice(len(xs), size=min(len(xs), 150), replace=False)
    for k in pick:
        px, py = int(xs[k]), int(ys[k])
        extra = [(rnd.uniform(-rho, rho), rnd.uniform(-rho, rho), rnd.uniform(-J, J), rnd.uniform(-J, J)) for _ in range(20)]
        for ox, oy, jx, jy in probes + extra:
            o, d = _rays(cam, W, H, px, py, ox, oy, jx, jy)
            assert not _slab_hit(o, d, lo.astype(np.float64), hi.astype(np.float64)), (name, px, py, ox, oy, jx, jy)
            for li in L:
                assert not _light_hit(o, d, li), (name, px, py, ox, oy, jx, jy)


def test_cull_rects_are_tight_enough_to_matter():
    # box.obj at 1080p: the box and the light cover well under half the frame
    lo, hi = np.full(3, -1.0, np.float32), np.full(3, 1.0, np.float32)
    rects = ptamd.primary_cull_rects(scenes.DEFAULT_CAMERA, 1920, 1080, lo, hi, scenes.REFERENCE_LIGHT)
    frac = _culled_mask(rects, 1920, 1080).mean()
    assert frac > 0.5, frac


def test_cull_disabled_when_object_reaches_camera_plane():
    lo, hi = np.full(3, -1.0, np.float32), np.full(3, 1.0, np.float32)
    inside = scenes.camera((0.0, 0.0, 0.5))
    assert ptamd.primary_cull_rects(inside, 64, 64, lo, hi, scenes.REFERENCE_LIGHT) is None
    behind = np.array([0, 0, 5, 0, 0, 0, 1, 0, 0, 1, 0, 0, 60, 0, 0, 0], np.float32)   # looking away
    assert ptamd.primary_cull_rects(behind, 64, 64, lo, hi, scenes.REFERENCE_LIGHT) is None
    degenerate = np.array([0, 0, 5, 0, 0, 1, 0, 0, 0, 1, 0, 0, 60, 0, 0, 0], np.float32)   # dir parallel to up
    assert ptamd.primary_cull_rects(degenerate, 64, 64, lo, hi, scenes.REFERENCE_LIGHT) is None
    many = np.tile(scenes.REFERENCE_LIGHT, 8)
    assert ptamd.primary_cull_rects(scenes.DEFAULT_CAMERA, 64, 64, lo, hi, many) is None


@pytest.mark.parametrize("name,cam,W,H,lights", CASES[:4], ids=[c[0] for c in CASES[:4]])
def test_oracle_renders_culled_pixels_as_background(box, name, cam, W, H, lights):
    v, idx, nodes = box
    lo = nodes.reshape(-1, 8)[0, 0:3]
    hi = nodes.reshape(-1, 8)[0, 4:7]
    rects = ptamd.primary_cull_rects(cam, W, H, lo, hi, lights)
    culled = _culled_mask(rects, W, H)
    img, _ = oracle_lib.render(v, idx, nodes, cam, lights, W, H, 0, 4, max_depth=1, sss_bounces=0)
    img = img.reshape(H, W, 4)
    assert np.array_equal(img[culled].view(np.uint32),
                          np.tile(np.array([0, 0, 0, 1], np.float32), (int(culled.sum()), 1)).view(np.uint32))
