"""The oracle pinned: against the reference's own recorded BVH dump
(tests/golden/box_bvh.json), hand-derived known answers for
single rays, and its own determinism/consistency properties."""
import json
import os

import numpy as np
import pytest

import oracle_lib as O
import scenes

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def box():
    v, i, t = O.obj_parse(open(scenes.BOX_OBJ, "rb").read())
    ri, nodes = O.bvh_build(v, i)
    return v, i, t, ri, nodes.reshape(-1, 8)


def test_box_obj_parse(box):
    v, i, t, _, _ = box
    g = json.load(open(os.path.join(GOLDEN, "box_bvh.json")))
    assert v.size // 3 == g["n_vertices"] and i.size // 3 == g["n_triangles"] and t.size // 2 == g["n_uvs"]
    # quads split on the shorter diagonal; all diagonals equal -> [0,1,3],[1,2,3] (tiny_obj_loader.h:1587-1604)
    assert i[:6].tolist() == [0, 4, 2, 4, 6, 2]


def test_box_bvh_matches_reference_dump(box):
    _, _, _, ri, nodes = box
    g = json.load(open(os.path.join(GOLDEN, "box_bvh.json")))
    assert nodes.shape[0] == g["n_nodes"]
    assert ri.reshape(-1, 3).tolist() == g["reordered_triangles"]
    assert nodes[0, :3].tolist() == g["root"]["min"] and nodes[0, 4:7].tolist() == g["root"]["max"]
    assert [nodes[0, 3], nodes[0, 7]] == g["root"]["w"]
    # pre-order: every internal node's left child is the next node
    for k in np.flatnonzero(nodes[:, 3] != -1):
        assert nodes[k, 3] == k + 1


def test_bvh_leaf_and_tree_invariants():
    v, i = scenes.random_triangles(5000, seed=11)
    ri, nodes = O.bvh_build(v, i)
    nodes = nodes.reshape(-1, 8)
    assert nodes.shape[0] == 2 * 5000 - 1
    leaves = nodes[nodes[:, 3] == -1]
    assert sorted(leaves[:, 7].astype(int).tolist()) == list(range(5000))
    assert sorted(map(tuple, ri.reshape(-1, 3).tolist())) == sorted(map(tuple, i.reshape(-1, 3).tolist()))


def test_known_answer_rays(box):
    v, _, _, ri, nodes = box
    # straight at the front face z=+1 from the default camera position
    hit, t, p, n, ctr = O.trace(v, ri, nodes, [0, 0, 5], [0, 0, -1])
    assert hit and t == pytest.approx(4.0, abs=1e-6) and p == pytest.approx([0, 0, 1], abs=1e-6)
    assert abs(n[2]) == pytest.approx(1.0) and abs(n[0]) < 1e-6
    # all 11 internal nodes are hit (exhaustive: 23 visits); with dir.x = dir.y = 0
    # only the leaves of the z=+1 and z=-1 faces pass their slab test
    assert ctr[0] == 1 and ctr[1] == 23 and ctr[2] == 4
    # a miss tests only the root
    hit, t, _, _, ctr = O.trace(v, ri, nodes, [0, 0, 5], [0, 1, 0])
    assert not hit and t == pytest.approx(1e30) and ctr[1] == 1 and ctr[2] == 0
    # from inside the cube (an SSS ray) every node is visited and the far face is hit
    hit, t, p, _, _ = O.trace(v, ri, nodes, [0, 0, 0.5], [1, 0, 0])
    assert hit and t == pytest.approx(1.0) and p[0] == pytest.approx(1.0)


def test_render_threads_and_row_subsets_agree(box):
    v, _, _, ri, nodes = box
    cam, light = scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT
    a1, s1 = O.render(v, ri, nodes, cam, light, 64, 48, n_batches=2, nthreads=1)
    a8, s8 = O.render(v, ri, nodes, cam, light, 64, 48, n_batches=2, nthreads=8)
    assert np.array_equal(a1.view(np.uint32), a8.view(np.uint32)) and np.array_equal(s1, s8)
    acc = np.zeros_like(a1)
    tot = np.zeros(3, np.uint64)
    for ph in range(3):
        _, s = O.render(v, ri, nodes, cam, light, 64, 48, n_batches=2, row_stride=3, row_phase=ph, accum=acc)
        tot += s
    assert np.array_equal(acc.view(np.uint32), a1.view(np.uint32)) and np.array_equal(tot, s1)


def test_progressive_batches_equal_one_call(box):
    v, _, _, ri, nodes = box
    cam, light = scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT
    seq = np.zeros(40 * 30 * 4, np.float32)
    for b in range(4):
        O.render(v, ri, nodes, cam, light, 40, 30, first_batch=b, n_batches=1, accum=seq)
    one, _ = O.render(v, ri, nodes, cam, light, 40, 30, first_batch=0, n_batches=4)
    assert np.array_equal(seq.view(np.uint32), one.view(np.uint32))


def test_light_visible_pixels_show_intensity(box):
    """Top rows look at the light from below (image row 0 = scene bottom for the
    default camera): the pre-pass returns intensity 10."""
    v, _, _, ri, nodes = box
    acc, _ = O.render(v, ri, nodes, scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, 64, 64, n_batches=1)
    img = acc.reshape(64, 64, 4)
    assert np.all(img[..., 3] == 1.0)
    assert np.any(img[..., :3] == 10.0)
    assert img[0:4].max() < 10.0 and np.any(img[60:64, :, 0] == 10.0)


def test_oracle_frame_is_frozen(box):
    """The oracle's box frame is pinned by a committed checksum
    (tests/golden/make_golden.py) so a change to the checker cannot pass
    silently."""
    v, _, _, ri, nodes = box
    g = json.load(open(os.path.join(GOLDEN, "oracle_frames.json")))
    for case in g["cases"]:
        acc, st = O.render(v, ri, nodes, scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, case["W"], case["H"],
                           n_batches=case["spp"], max_depth=case["depth"], sss_bounces=case["sss"])
        import hashlib
        assert hashlib.sha256(acc.tobytes()).hexdigest() == case["sha256"], case
        assert st.tolist() == case["stats"], case
