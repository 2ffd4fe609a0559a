"""GPU parity: the HIP kernel (through the C ABI) against the CPU oracle.

The bar is bitwise equality of the accumulation buffer (north_star asks for
1e-4 per channel; the design target is bit-exact) and exact
equality of the reference-traversal counters.
"""
import numpy as np
import pytest

import oracle_lib as O
import ptamd
import scenes

pytestmark = pytest.mark.gpu

TOL = 1e-4   # north_star per-channel tolerance; every assertion below is stricter (bitwise)


def _setup(v, i, n, cam=scenes.DEFAULT_CAMERA, lights=scenes.REFERENCE_LIGHT, depth=4, sss=3, int_bits=False,
           lds=1):
    r = ptamd.Renderer(0)
    r.set_option(ptamd.PT_OPT_SCENE_IN_LDS, lds)
    r.upload_scene(v, i, n, int_bits=int_bits)
    r.upload_lights(lights)
    r.set_camera(cam)
    r.set_params(depth, sss)
    return r


def _box():
    s = ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh()
    v, i, n, _, _ = s.arrays()
    return v, i, n


def _oracle(v, i, n, W, H, first=0, nb=1, depth=4, sss=3, cam=scenes.DEFAULT_CAMERA,
            lights=scenes.REFERENCE_LIGHT, **kw):
    return O.render(v, i, n.reshape(-1), cam, lights, W, H, first_batch=first, n_batches=nb,
                    max_depth=depth, sss_bounces=sss, **kw)


def _assert_same(gpu, ref, what=""):
    assert gpu.shape == ref.shape
    if not np.array_equal(gpu.view(np.uint32), ref.view(np.uint32)):
        bad = np.flatnonzero(gpu.view(np.uint32) != ref.view(np.uint32))
        diff = np.nanmax(np.abs(gpu[bad] - ref[bad])) if bad.size else 0.0
        raise AssertionError(f"{what}: {bad.size} of {gpu.size} floats differ (max |diff| {diff}); "
                             f"first at pixel {bad[0] // 4} gpu={gpu[bad[0]]} ref={ref[bad[0]]}")


@pytest.mark.parametrize("lds", [0, 2])
@pytest.mark.parametrize("W,H,depth,nb", [(256, 256, 1, 1), (256, 256, 4, 1), (64, 48, 4, 8), (17, 13, 4, 3)])
def test_box_matches_oracle(W, H, depth, nb, lds):
    v, i, n = _box()
    r = _setup(v, i, n, depth=depth, lds=lds)
    r.resize_and_clear(W, H)
    r.render(0, nb)
    gpu = r.read_accum()
    ref, _ = _oracle(v, i, n, W, H, nb=nb, depth=depth)
    _assert_same(gpu, ref, f"box {W}x{H} d{depth} spp{nb}")
    assert np.all(np.abs(gpu - ref) <= TOL)


@pytest.mark.parametrize("spl", [1, 2, 4, 8])
@pytest.mark.parametrize("nb", [1, 3, 8, 13])
def test_sample_lanes(spl, nb):
    """Every sample-lane mapping gives the oracle's frame, including sample
    counts that are not multiples of the lane count and ragged tiles."""
    v, i, n = _box()
    r = _setup(v, i, n)
    r.set_option(ptamd.PT_OPT_SAMPLE_LANES, spl)
    r.resize_and_clear(40, 27)
    r.render(2, nb)
    ref, _ = _oracle(v, i, n, 40, 27, first=2, nb=nb)
    _assert_same(r.read_accum(), ref, f"spl={spl} nb={nb}")


def _scene_cases():
    gv, gi = scenes.grid_mesh(6)
    sv, si = scenes.displaced_sphere(2)
    tv, ti = scenes.random_triangles(1000, seed=1000)
    two = np.concatenate([scenes.REFERENCE_LIGHT,
                          ptamd.pack_light([0.5, 0.5, 1.5], [0, 0, -1], [2, 4, 8], [0.5, 1.0])])
    return [("grid2lights", gv, gi, scenes.camera((0.0, 0.0, 3.0)), two, 3, 2),
            ("sphere", sv, si, scenes.camera((0.0, 0.5, 3.0)), scenes.REFERENCE_LIGHT, 4, 3),
            ("random", tv, ti, scenes.camera((0.3, 0.2, 2.2)), scenes.REFERENCE_LIGHT, 4, 3),
            ("nolight_d2", tv, ti, scenes.camera((0.3, 0.2, 2.2)), np.zeros(0, np.float32), 2, 1),
            ("depth0", sv, si, scenes.camera((0.0, 3.0, 0.5), up=(0, 0, 1)), scenes.REFERENCE_LIGHT, 0, 3),
            ("sss0", sv, si, scenes.camera((0.0, 0.5, 3.0)), scenes.REFERENCE_LIGHT, 4, 0)]


def test_removed_kernels_are_refused():
    """The lane state-machine kernel, child-pair records and 8-wide nodes were
    measured slower on every scene and removed: their
    options fail loudly instead of silently running another kernel."""
    v, i, n = _box()
    r = _setup(v, i, n)
    for key, val in ((ptamd.PT_OPT_KERNEL, 2), (ptamd.PT_OPT_SM_BATCH, 8), (ptamd.PT_OPT_PAIRS, 1),
                     (ptamd.PT_OPT_WIDE_NODE, 80)):
        with pytest.raises(ptamd.PTError, match="removed"):
            r.set_option(key, val)


def test_dispatch_sequence_equals_fused_render():
    v, i, n = _box()
    r = _setup(v, i, n)
    r.resize_and_clear(96, 80)
    for b in range(5):
        r.dispatch(b)
    seq = r.read_accum()
    r.clear()
    r.render(0, 5)
    fused = r.read_accum()
    _assert_same(fused, seq, "dispatch x5 vs render(0,5)")
    r.clear()
    r.render(0, 2)
    r.render(2, 3)
    _assert_same(r.read_accum(), seq, "render(0,2)+render(2,3)")


@pytest.mark.parametrize("lds", [0, 2])
def test_stats_mode_counts_and_output(lds):
    v, i, n = _box()
    W, H, nb = 128, 96, 3
    r = _setup(v, i, n, lds=lds)
    r.resize_and_clear(W, H)
    r.render(0, nb)
    plain = r.read_accum()
    r.clear()
    r.set_stats_mode(True)
    r.reset_stats()
    r.render(0, nb)
    counted = r.read_accum()
    st = r.stats()
    ref, ost = _oracle(v, i, n, W, H, nb=nb)
    _assert_same(counted, plain, "stats-mode image vs fast image")
    _assert_same(counted, ref, "stats-mode image vs oracle")
    assert (st["rays"], st["nodes"], st["leaf_tests"]) == tuple(int(x) for x in ost)
    assert st["samples"] == W * H * nb


@pytest.mark.parametrize("lds", [0, 1])
def test_box_1080p_8spp_full_frame(lds):
    """The bench configuration (BASELINE.json configs[1]) compared in full."""
    v, i, n = _box()
    r = _setup(v, i, n, lds=lds)
    r.resize_and_clear(1920, 1080)
    r.render(0, 8)
    gpu = r.read_accum()
    ref, _ = _oracle(v, i, n, 1920, 1080, nb=8)
    _assert_same(gpu, ref, "box 1080p 8spp")


def test_box_1080p_8spp_bench_options_two_contexts():
    """The headline's timed configuration exactly as bench.py runs it at N = 1
    (BASELINE configs[1]): two contexts on streams of
    their own, frames alternating between them with no wait in between (two in
    flight), PT_OPT_SAMPLE_LANES 1, PT_OPT_ITEM_ORDER 0, PT_OPT_FRESH_BATCH0 1
    over stale accumulators; every context's last frame against the oracle's
    whole frame (raytrace_comp.comp:420-470)."""
    import torch
    v, i, n = _box()
    ctxs, streams = [], []
    for _ in range(2):
        r = _setup(v, i, n)
        r.set_option(ptamd.PT_OPT_SAMPLE_LANES, 1)
        r.set_option(ptamd.PT_OPT_ITEM_ORDER, 0)
        r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
        s = torch.cuda.Stream(torch.device("cuda", 0))
        streams.append(s)
        r.set_stream(s.cuda_stream)
        r.resize_and_clear(1920, 1080)
        ctxs.append(r)
    for k in range(7):
        ctxs[k % 2].render(0, 8)
    for r in ctxs:
        r.synchronize()
    ref, _ = _oracle(v, i, n, 1920, 1080, nb=8)
    for k, r in enumerate(ctxs):
        _assert_same(r.read_accum(), ref, f"bench options, context {k}")
    for r in ctxs:
        r.close()


def test_mixed_lanes_static_and_measured_schedules():
    """PT_OPT_MIXED_LANES (the one-context drop-in frame): live tiles at one
    lane per pixel and tile parts at more lanes -- uniform lanes first, then
    the schedule built from the measured block costs
    (the cost feedback of two launches) -- each frame bitwise the oracle's
    (raytrace_comp.comp:420-470); a camera change drops the measured costs.
    pt_mixed_info: 0 uniform lanes (while measuring), 2 the measured
    schedule."""
    v, i, n = _box()
    r = _setup(v, i, n)
    r.resize_and_clear(1920, 1080)
    ref, _ = _oracle(v, i, n, 1920, 1080, nb=8)
    seen = set()
    for k in range(12):
        r.render(0, 8)
        r.synchronize()
        seen.add(r.mixed_info()[0])
        if k in (0, 11):
            _assert_same(r.read_accum(), ref, f"mixed lanes, frame {k}, schedule {r.mixed_info()}")
    sched, items, measured = r.mixed_info()
    assert sched == 2 and measured >= 2 and items > 0, r.mixed_info()
    assert 0 in seen   # uniform lanes while the costs are measured
    # another camera: back to the uniform schedule, same parity
    cam2 = scenes.camera((0.4, 0.3, 4.0))
    r.set_camera(cam2)
    r.render(0, 8)
    assert r.mixed_info()[0] == 0
    ref2, _ = _oracle(v, i, n, 1920, 1080, nb=8, cam=cam2)
    _assert_same(r.read_accum(), ref2, "mixed lanes after a camera change")


@pytest.mark.parametrize("budget,spl,nb,first", [(50, 4, 8, 0), (1000, 4, 3, 2), (100, 8, 13, 0), (7, 2, 5, 1)])
def test_mixed_lanes_static_budgets(budget, spl, nb, first):
    """Static mixed schedules with every whole-tile budget, lane count and
    sample count (fewer samples than lanes, progressive continuation over a
    stale accumulator), ragged edge tiles."""
    v, i, n = _box()
    r = _setup(v, i, n)
    r.set_option(ptamd.PT_OPT_MIXED_LANES, budget)
    r.set_option(ptamd.PT_OPT_SAMPLE_LANES, spl)
    W, H = 333, 250
    r.resize_and_clear(W, H)
    if first:
        r.render(0, first)
    r.render(first, nb)
    assert r.mixed_info()[0] == 1
    ref, _ = _oracle(v, i, n, W, H, first=0, nb=first + nb)
    _assert_same(r.read_accum(), ref, f"mixed budget {budget} spl {spl} nb {nb} first {first}")


def test_culled_items_written_once_per_layout():
    """A launch skips the fill of culled items that already hold (0,0,0,1) in
    its buffer under the same item layout (render_impl's culled_state): every
    frame of a sequence that exercises the state -- repeats, a continuation,
    a camera change and back (the previous camera's live pixels become
    culled), a clear, a caller buffer full of NaN with and without
    PT_OPT_FRESH_BATCH0 -- is bitwise the oracle's."""
    import torch
    v, i, n = _box()
    W, H = 333, 250
    cam2 = scenes.camera((0.6, -0.4, 3.2))
    r = _setup(v, i, n)
    r.resize_and_clear(W, H)
    want1_2, _ = _oracle(v, i, n, W, H, nb=2)
    want1_5, _ = _oracle(v, i, n, W, H, nb=5)
    want2_2, _ = _oracle(v, i, n, W, H, nb=2, cam=cam2)
    r.render(0, 2)
    _assert_same(r.read_accum(), want1_2, "first frame")
    r.render(0, 2)
    _assert_same(r.read_accum(), want1_2, "repeat (fill skipped)")
    r.render(2, 3)
    _assert_same(r.read_accum(), want1_5, "continuation")
    r.set_camera(cam2)
    r.render(0, 2)
    _assert_same(r.read_accum(), want2_2, "another camera")
    r.set_camera(scenes.DEFAULT_CAMERA)
    r.render(0, 2)
    _assert_same(r.read_accum(), want1_2, "back to the first camera")
    r.clear()
    r.render(0, 2)
    _assert_same(r.read_accum(), want1_2, "after a clear")
    nanbuf = torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda:0")
    r.bind_accum(nanbuf.data_ptr(), W, H)
    r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
    for k in range(2):
        r.render(0, 2)
        _assert_same(r.read_accum(), want1_2, f"fresh frame {k} over NaN")
    r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 0)
    r.render(0, 2)
    _assert_same(r.read_accum(), want1_2, "reference semantics after fresh frames")
    nanbuf.fill_(float("nan"))   # written behind the library's back: bind again
    r.bind_accum(nanbuf.data_ptr(), W, H)
    r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
    r.render(0, 2)
    _assert_same(r.read_accum(), want1_2, "fresh frame over a re-bound NaN buffer")
    r.close()


def test_partition_sum_is_bit_exact():
    v, i, n = _box()
    W, H, nb = 200, 120, 2
    full = _setup(v, i, n)
    full.resize_and_clear(W, H)
    full.render(0, nb)
    want = full.read_accum()
    for nranks in (2, 3, 8):
        acc = np.full(W * H * 4, -0.0, np.float32)   # -0 is the IEEE additive identity
        for rank in range(nranks):
            r = _setup(v, i, n)
            r.set_partition(nranks, rank)
            r.resize_and_clear(W, H)
            r.render(0, nb)
            part = r.read_accum()
            acc = (acc + part).astype(np.float32)
        _assert_same(acc, want, f"sum over {nranks} ranks")


def test_fresh_batch0_ignores_stale_accumulator():
    v, i, n = _box()
    r = _setup(v, i, n)
    r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
    r.resize_and_clear(64, 40)
    r.render(0, 3)          # leaves a finished frame in the buffer
    r.render(0, 4)          # restarts at batch 0 without clearing
    ref, _ = _oracle(v, i, n, 64, 40, nb=4)
    _assert_same(r.read_accum(), ref, "fresh restart")
    r.render(4, 2)          # continuing batches still read the accumulator
    ref, _ = _oracle(v, i, n, 64, 40, nb=6)
    _assert_same(r.read_accum(), ref, "fresh + continue")


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_tile_gather_assembles_frame(nranks):
    """pt_tiles_pack on every rank + pt_tiles_unpack on the root = the
    single-GPU frame (the gather path bench.py uses for N > 2)."""
    import torch
    v, i, n = _box()
    W, H = 150, 70
    frame = torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda")
    root = None
    for rank in range(nranks):
        r = _setup(v, i, n)
        r.set_partition(nranks, rank)
        r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
        r.resize_and_clear(W, H)
        r.render(0, 8)
        buf = torch.empty((r.tiles_owned(), 256, 4), dtype=torch.float32, device="cuda")
        r.tiles_pack(buf.data_ptr())
        r.synchronize()
        if root is None:
            root = r
        root.tiles_unpack(buf.data_ptr(), rank, frame.data_ptr())
        root.synchronize()
    ref, _ = _oracle(v, i, n, W, H, nb=8)
    _assert_same(frame.cpu().numpy().reshape(-1), ref, f"gather over {nranks}")


@pytest.mark.parametrize("ntri,int_bits", [(1, False), (2, False), (1000, False), (20000, True), (40000, False)])
def test_random_triangles(ntri, int_bits):
    tv, ti = scenes.random_triangles(ntri, seed=ntri)
    s = ptamd.Scene.from_arrays(tv, ti).build_bvh(int_bits=int_bits)
    v, i, n, _, _ = s.arrays()
    cam = scenes.camera((0.3, 0.2, 2.2))
    r = _setup(v, i, n, cam=cam, int_bits=int_bits)
    r.resize_and_clear(96, 64)
    r.render(0, 2)
    gpu = r.read_accum()
    ref, _ = _oracle(v, i, n, 96, 64, nb=2, cam=cam, int_bits=int_bits)
    _assert_same(gpu, ref, f"random {ntri}")


@pytest.mark.parametrize("lds", [0, 1])
def test_grid_ties_and_two_lights(lds):
    """lds=0 walks from device memory with paired shadow/closest walks: the
    first light's shadow rays single, the second's paired."""
    gv, gi = scenes.grid_mesh(6)
    s = ptamd.Scene.from_arrays(gv, gi).build_bvh()
    v, i, n, _, _ = s.arrays()
    lights = np.concatenate([scenes.REFERENCE_LIGHT,
                             ptamd.pack_light([0.5, 0.5, 1.5], [0, 0, -1], [2, 4, 8], [0.5, 1.0])])
    cam = scenes.camera((0.0, 0.0, 3.0))
    r = _setup(v, i, n, cam=cam, lights=lights, depth=3, sss=2, lds=lds)
    r.resize_and_clear(64, 64)
    r.render(3, 2)
    gpu = r.read_accum()
    ref, _ = _oracle(v, i, n, 64, 64, first=3, nb=2, depth=3, sss=2, cam=cam, lights=lights)
    _assert_same(gpu, ref, "grid")


@pytest.mark.parametrize("lds", [0, 1])
def test_edge_params(lds):
    v, i, n = _box()
    for depth, sss, lights in [(0, 3, scenes.REFERENCE_LIGHT), (4, 0, scenes.REFERENCE_LIGHT),
                               (2, 1, np.zeros(0, np.float32)), (3, 1, scenes.REFERENCE_LIGHT)]:
        r = _setup(v, i, n, depth=depth, sss=sss, lights=lights, lds=lds)
        r.resize_and_clear(48, 40)
        r.render(0, 2)
        ref, _ = _oracle(v, i, n, 48, 40, nb=2, depth=depth, sss=sss, lights=lights)
        _assert_same(r.read_accum(), ref, f"depth={depth} sss={sss} lights={lights.size // 16}")


@pytest.mark.parametrize("lds", [0, 1])
def test_displaced_sphere_substitute(lds):
    sv, si = scenes.displaced_sphere(3)
    s = ptamd.Scene.from_arrays(sv, si).build_bvh()
    v, i, n, _, _ = s.arrays()
    cam = scenes.camera((0.0, 0.5, 3.0))
    r = _setup(v, i, n, cam=cam, lds=lds)
    r.resize_and_clear(80, 60)
    r.render(0, 2)
    ref, _ = _oracle(v, i, n, 80, 60, nb=2, cam=cam)
    _assert_same(r.read_accum(), ref, "sphere")


def test_errors_are_reported():
    r = ptamd.Renderer(0)
    with pytest.raises(ptamd.PTError):
        r.render(0, 1)              # no scene
    v, i, n = _box()
    with pytest.raises(ptamd.PTError):
        r.upload_scene(v, i[:-3], n)  # node count mismatch
    bad = n.copy()
    bad[0, 7] = 99.0                # right child out of range
    with pytest.raises(ptamd.PTError):
        r.upload_scene(v, i, bad)


CULL_CAMS = [
    scenes.DEFAULT_CAMERA,
    scenes.camera((3.0, 2.0, 4.0)),
    scenes.camera((0.0, 0.5, 12.0), fov=100.0),
    scenes.camera((1.0, -1.0, 7.0), fov=20.0),
    np.array([0, 0, 14, 0, 0, 0, -2, 0, 0.3, 1, 0.2, 0, 45, 0, 0, 0], np.float32),
    scenes.camera((0.0, 0.0, 0.5)),   # inside the box: culling not derivable
]


@pytest.mark.parametrize("cam", range(len(CULL_CAMS)))
@pytest.mark.parametrize("W,H", [(96, 54), (17, 13)])
def test_primary_culling_is_exact(cam, W, H):
    """PT_OPT_PRIMARY_CULL on (default) and off give the oracle's frame."""
    v, i, n = _box()
    lights = np.concatenate([scenes.REFERENCE_LIGHT,
                             np.array([1.5, 0.5, 2.0, 0, -1, 0, 0, 0, 3, 2, 1, 0, 0.5, 1.0, 0, 0], np.float32)])
    ref, _ = _oracle(v, i, n, W, H, nb=4, cam=CULL_CAMS[cam], lights=lights)
    for cull in (1, 0):
        r = _setup(v, i, n, cam=CULL_CAMS[cam], lights=lights)
        r.set_option(ptamd.PT_OPT_PRIMARY_CULL, cull)
        r.resize_and_clear(W, H)
        r.render(0, 4)
        _assert_same(r.read_accum(), ref, f"cull={cull} cam {cam} {W}x{H}")


def test_primary_culling_with_stale_accumulator():
    """Culled pixels fold a non-trivial prior state exactly: camera switched
    without a clear (first batch > 0 and first batch 0 over a finite image)."""
    v, i, n = _box()
    W, H = 64, 48
    camA, camB, camC = CULL_CAMS[1], CULL_CAMS[0], CULL_CAMS[2]
    ref, _ = _oracle(v, i, n, W, H, first=0, nb=2, cam=camA)
    ref, _ = _oracle(v, i, n, W, H, first=2, nb=3, cam=camB, accum=ref)
    ref2, _ = _oracle(v, i, n, W, H, first=0, nb=2, cam=camC, accum=ref.copy())
    for spl in (1, 2, 4):
        r = _setup(v, i, n, cam=camA)
        r.set_option(ptamd.PT_OPT_SAMPLE_LANES, spl)
        r.resize_and_clear(W, H)
        r.render(0, 2)
        r.set_camera(camB)
        r.render(2, 3)
        _assert_same(r.read_accum(), ref, f"spl {spl} first>0 over stale")
        r.set_camera(camC)
        r.render(0, 2)
        _assert_same(r.read_accum(), ref2, f"spl {spl} first=0 over stale")


def test_progressive_loop_camera_reset_and_async_readback():
    """mainLoop semantics (VulkanRayTracer.cpp:717-865): a camera change
    restarts at batch 0 over the old image (prev*0), batches are capped, and
    readbacks return the image as of their begin while rendering goes on."""
    v, i, n = _box()
    W, H = 64, 48
    camA, camB = scenes.camera((3.0, 2.0, 4.0)), scenes.DEFAULT_CAMERA
    r = _setup(v, i, n, cam=camA)
    r.resize_and_clear(W, H)
    assert r.progressive_camera(camA) is True
    assert r.progressive_advance(2) == (0, 2)
    t1 = r.readback_begin()                       # image after camA batches 0-1
    assert r.progressive_advance(1) == (2, 1)
    assert r.progressive_camera(camA) is False    # unchanged camera: no reset
    assert r.progressive_camera(camB) is True     # reset to batch 0 over the camA image
    assert r.progressive_advance(5, limit=4) == (0, 4)   # capped
    assert r.progressive_advance(5, limit=4) == (4, 0)
    t2 = r.readback_begin()
    img2 = r.readback_end(t2)
    img1 = r.readback_end(t1)
    refA, _ = _oracle(v, i, n, W, H, first=0, nb=2, cam=camA)
    _assert_same(img1, refA, "readback after camA 0-1")
    acc = refA.copy()
    acc, _ = _oracle(v, i, n, W, H, first=2, nb=1, cam=camA, accum=acc)
    acc, _ = _oracle(v, i, n, W, H, first=0, nb=4, cam=camB, accum=acc)
    _assert_same(img2, acc, "camB 0-3 over camA image")
    _assert_same(r.read_accum(), acc, "accumulator")
    with pytest.raises(ptamd.PTError):
        r.readback_end(t2)                        # already collected


@pytest.mark.parametrize("nranks,cam,mode", [(2, 0, "pack"), (3, 1, "pack"), (8, 0, "pack"), (2, 5, "pack"),
                                           (3, 1, "direct"), (8, 0, "direct"), (2, 5, "direct"),
                                           (3, 0, "direct-scan-order"), (2, 1, "direct-wavefront")])
def test_sparse_item_exchange_assembles_frame(nranks, cam, mode):
    """pt_items_pack (live items only) on every rank + one pt_items_unpack_all
    on the root = the single-GPU frame; culled items are rebuilt as
    (0,0,0,1).  Camera 5 sits inside the box (no culling: every item live).
    "direct": pt_render_packed writes the live items into the slot in the
    render launch itself (the accumulator, pre-filled with NaN, stays
    untouched); "scan-order": PT_OPT_ITEM_ORDER 0; "wavefront": the wavefront
    kernel, which renders then packs."""
    import torch
    v, i, n = _box()
    W, H = 150, 70
    camera = CULL_CAMS[cam]
    rs, counts = [], []
    for rank in range(nranks):
        r = _setup(v, i, n, cam=camera)
        r.set_partition(nranks, rank)
        r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
        if mode.endswith("scan-order"):
            r.set_option(ptamd.PT_OPT_ITEM_ORDER, 0)
        if mode.endswith("wavefront"):
            r.set_option(ptamd.PT_OPT_KERNEL, 3)
        r.resize_and_clear(W, H)
        r.render(0, 8)
        rs.append(r)
    per = rs[0].items_live(0)[1]
    counts = [rs[0].items_live(k)[0] for k in range(nranks)]
    assert all(rs[k].items_live(k) == (counts[k], per) for k in range(nranks))
    slot = max(counts) * per * 4
    src = torch.full((nranks, max(slot, 4)), float("nan"), dtype=torch.float32, device="cuda")
    rs_keep = []
    for k, r in enumerate(rs):
        if mode.startswith("direct"):
            if not mode.endswith("wavefront"):
                nan = torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda")
                r.bind_accum(nan.data_ptr(), W, H)
                rs_keep.append(nan)
            r.render_packed(8, src[k].data_ptr())
            r.synchronize()
            if not mode.endswith("wavefront"):
                assert torch.isnan(nan).all(), "pt_render_packed wrote the accumulation buffer"
        else:
            r.items_pack(src[k].data_ptr())
            r.synchronize()
    frame = torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda")
    rs[0].items_unpack_all(src.data_ptr(), src.shape[1], frame.data_ptr())
    rs[0].synchronize()
    ref, _ = _oracle(v, i, n, W, H, nb=8, cam=camera)
    _assert_same(frame.cpu().numpy().reshape(-1), ref, f"sparse exchange over {nranks}")
    if cam == 5:
        assert sum(counts) * per >= W * H
    else:
        assert sum(counts) * per < W * H          # culled items are not shipped


@pytest.mark.parametrize("nranks,cam,kernel", [(2, 0, 0), (3, 1, 0), (8, 0, 0), (2, 5, 0), (3, 0, 3)])
def test_render_packed_assembles_previous_frame(nranks, cam, kernel):
    """The pipelined tile-split step: every rank's pt_render_packed writes its
    live items to its slot, and the root's next pt_render_packed assembles
    those slots into the frame in the same launch (kernel 3: the wavefront
    fallback, separate launches).  Both gathered frames equal the oracle; a
    change of item layout in between (frame size) is refused."""
    import torch
    v, i, n = _box()
    W, H = 150, 70
    camera = CULL_CAMS[cam]
    rs = []
    for rank in range(nranks):
        r = _setup(v, i, n, cam=camera)
        r.set_partition(nranks, rank)
        if kernel:
            r.set_option(ptamd.PT_OPT_KERNEL, kernel)
        r.resize_and_clear(W, H)
        r.render(0, 8)
        rs.append(r)
    per = rs[0].items_live(0)[1]
    slot = max(4, max(rs[0].items_live(k)[0] for k in range(nranks)) * per * 4)
    src = [torch.full((nranks, slot), float("nan"), dtype=torch.float32, device="cuda") for _ in range(2)]
    for k, r in enumerate(rs):
        r.render_packed(8, src[0][k].data_ptr())
        r.synchronize()
    frame = torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda")
    for k in range(nranks - 1, -1, -1):   # the root (0) last: it assembles frame 1
        if k == 0:
            rs[0].render_packed(8, src[1][0].data_ptr(), src[0].data_ptr(), slot, frame.data_ptr())
        else:
            rs[k].render_packed(8, src[1][k].data_ptr())
        rs[k].synchronize()
    ref, _ = _oracle(v, i, n, W, H, nb=8, cam=camera)
    _assert_same(frame.cpu().numpy().reshape(-1), ref, f"frame 1 assembled in frame 2's launch, {nranks} ranks")
    frame2 = torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda")
    rs[0].items_unpack_all(src[1].data_ptr(), slot, frame2.data_ptr())
    rs[0].synchronize()
    _assert_same(frame2.cpu().numpy().reshape(-1), ref, "frame 2")
    rs[0].resize_and_clear(W + 16, H)   # another item layout
    with pytest.raises(ptamd.PTError):
        rs[0].render_packed(8, src[0][0].data_ptr(), src[1].data_ptr(), slot, frame.data_ptr())


# ---- wavefront pipeline (PT_OPT_KERNEL 3) ----------------------------------

@pytest.mark.parametrize("lds,spl", [(0, 1), (2, 4), (0, 8)])
def test_wavefront_kernel_box(lds, spl):
    v, i, n = _box()
    r = _setup(v, i, n, lds=lds)
    r.set_option(ptamd.PT_OPT_KERNEL, ptamd.KERNEL_WAVEFRONT)
    r.set_option(ptamd.PT_OPT_SAMPLE_LANES, spl)
    r.resize_and_clear(70, 45)
    r.render(1, 5)
    ref, _ = _oracle(v, i, n, 70, 45, first=1, nb=5)
    _assert_same(r.read_accum(), ref, f"wavefront box lds={lds} spl={spl}")


@pytest.mark.parametrize("case", range(6))
def test_wavefront_kernel_scenes(case):
    name, sv, si, cam, lights, depth, sss = _scene_cases()[case]
    s = ptamd.Scene.from_arrays(sv, si).build_bvh()
    v, i, n, _, _ = s.arrays()
    r = _setup(v, i, n, cam=cam, lights=lights, depth=depth, sss=sss, lds=0)
    r.set_option(ptamd.PT_OPT_KERNEL, ptamd.KERNEL_WAVEFRONT)
    r.resize_and_clear(56, 40)
    r.render(0, 3)
    ref, _ = _oracle(v, i, n, 56, 40, nb=3, depth=depth, sss=sss, cam=cam, lights=lights)
    _assert_same(r.read_accum(), ref, f"wavefront {name}")


@pytest.mark.parametrize("paths", [1, 3000, 7000])
def test_wavefront_batch_chunks(paths):
    """Launches larger than PT_OPT_WF_PATHS run in chunks of whole batches
    (1 = one batch per chunk): same frame, over a stale accumulator too."""
    v, i, n = _box()
    W, H = 50, 41
    camA, camB = CULL_CAMS[1], CULL_CAMS[0]
    ref, _ = _oracle(v, i, n, W, H, first=0, nb=3, cam=camA)
    ref, _ = _oracle(v, i, n, W, H, first=3, nb=7, cam=camB, accum=ref)
    r = _setup(v, i, n, cam=camA)
    r.set_option(ptamd.PT_OPT_KERNEL, ptamd.KERNEL_WAVEFRONT)
    r.set_option(ptamd.PT_OPT_WF_PATHS, paths)
    r.resize_and_clear(W, H)
    r.render(0, 3)
    r.set_camera(camB)
    r.render(3, 7)
    _assert_same(r.read_accum(), ref, f"wavefront chunks of {paths} paths")


@pytest.mark.parametrize("cam", range(len(CULL_CAMS)))
def test_wavefront_culling_and_partition(cam):
    """Culling (compact items + fill) and a tile partition under the wavefront
    kernel: every rank's owned pixels equal the oracle's."""
    v, i, n = _box()
    W, H = 96, 54
    ref, _ = _oracle(v, i, n, W, H, nb=4, cam=CULL_CAMS[cam])
    ref = ref.reshape(H, W, 4)
    for nranks, rank in [(1, 0), (3, 2)]:
        r = _setup(v, i, n, cam=CULL_CAMS[cam])
        r.set_option(ptamd.PT_OPT_KERNEL, ptamd.KERNEL_WAVEFRONT)
        r.set_partition(nranks, rank)
        r.resize_and_clear(W, H)
        r.render(0, 4)
        got = r.read_accum().reshape(H, W, 4)
        own = ptamd.partition_owned(W, H, nranks, rank)
        _assert_same(got[own].reshape(-1), ref[own].reshape(-1), f"wavefront cam {cam} rank {rank}/{nranks}")


def test_wavefront_rejects_stats_mode():
    v, i, n = _box()
    r = _setup(v, i, n)
    r.set_option(ptamd.PT_OPT_KERNEL, ptamd.KERNEL_WAVEFRONT)
    r.set_stats_mode(True)
    r.resize_and_clear(16, 16)
    with pytest.raises(ptamd.PTError):
        r.render(0, 1)


# ---- shadow rays skipped when their answer cannot change the image ---------
@pytest.mark.parametrize("lds", [0, 1])
@pytest.mark.parametrize("kernel", [1, 3])
def test_shadow_skip_light_intensities(lds, kernel):
    """shadow_needed: a light term with diff = 0 is +-0 only for a finite
    intensity.  A negative intensity (terms -0: skipped) and an infinite one
    (inf * 0 = NaN: must be traced) next to the reference light, on every
    kernel.  NaNs are compared as NaN (their sign/payload is the platform's);
    every other float bitwise."""
    v, i, n = _box()
    lights = np.concatenate([scenes.REFERENCE_LIGHT,
                             ptamd.pack_light([2.5, 0.5, 0.0], [-1, 0, 0], [-3.0, 0.5, 2.0], [1.0, 1.0]),
                             ptamd.pack_light([-2.5, 0.0, 0.5], [1, 0, 0], [np.inf, 1.0, 0.25], [0.5, 0.5])])
    cam = scenes.camera((0.5, 1.5, 3.5))
    r = _setup(v, i, n, cam=cam, lights=lights, lds=lds)
    r.set_option(ptamd.PT_OPT_KERNEL, kernel)
    r.resize_and_clear(40, 32)
    r.render(0, 3)
    gpu = r.read_accum()
    ref, _ = _oracle(v, i, n, 40, 32, nb=3, cam=cam, lights=lights)
    nan_g, nan_r = np.isnan(gpu), np.isnan(ref)
    assert np.array_equal(nan_g, nan_r), f"NaN pattern differs in {np.count_nonzero(nan_g != nan_r)} floats"
    assert nan_r.any() and (~nan_r).any()
    _assert_same(np.where(nan_g, 0, gpu).astype(np.float32), np.where(nan_r, 0, ref).astype(np.float32),
                 f"kernel {kernel} lds {lds}")


# ---- launch timing (bench.py's kernel_ms / launch_interval_ms) -------------
def test_launch_timing_sampling_and_span():
    """PT_OPT_LAUNCH_TIMING k: an event pair around every k-th launch;
    pt_launch_span_ms covers first timed start to last timed end and reports
    how many launches that span holds.  Output does not depend on timing."""
    v, i, n = _box()
    r = _setup(v, i, n)
    r.resize_and_clear(64, 48)
    r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
    r.render(0, 2)
    want = r.read_accum()
    with pytest.raises(ptamd.PTError):
        r.set_option(ptamd.PT_OPT_LAUNCH_TIMING, -1)
    for every, launches, timed, covered in [(1, 5, 5, 5), (3, 7, 3, 7), (4, 5, 2, 5)]:
        r.set_option(ptamd.PT_OPT_LAUNCH_TIMING, every)
        r.reset_launch_times()
        for _ in range(launches):
            r.render(0, 2)
        t = r.launch_times_ms()
        assert t.size == timed and np.all(t > 0), (every, t)
        span, n_cov = r.launch_span_ms()
        assert n_cov == covered and span >= t.max() > 0, (every, span, n_cov)
        _assert_same(r.read_accum(), want, f"timing every {every}")
    r.set_option(ptamd.PT_OPT_LAUNCH_TIMING, 0)
    r.reset_launch_times()
    r.render(0, 2)
    assert r.launch_times_ms().size == 0
    with pytest.raises(ptamd.PTError):
        r.launch_span_ms()


@pytest.mark.parametrize("kernel", [0, 3])
def test_render_packed_on_alternating_streams(kernel):
    """bench.py's N>1 step: one context renders frames k = 0..5 with
    pt_render_packed on two alternating streams without host synchronisation,
    frame k also assembling frame k-2's slot.  The wavefront kernel renders
    through context buffers (accumulation, path lists), so its launches on
    different streams must be ordered by the library (order_shared); every
    assembled frame equals the oracle bitwise."""
    import torch
    v, i, n = _box()
    W, H = 96, 64
    r = _setup(v, i, n, cam=CULL_CAMS[1])
    if kernel:
        r.set_option(ptamd.PT_OPT_KERNEL, kernel)
    r.set_partition(1, 0)
    r.resize_and_clear(W, H)
    r.render(0, 4)
    per = r.items_live(0)[1]
    slot = max(4, r.items_live(0)[0] * per * 4)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    # frame k writes slot buffer k % 4 and assembles buffer (k - 2) % 4, both
    # last touched on its own stream: only the library's buffers are shared
    bufs = [torch.full((1, slot), float("nan"), dtype=torch.float32, device="cuda") for _ in range(4)]
    frames = [torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda") for _ in range(4)]
    torch.cuda.synchronize()
    for k in range(6):
        r.set_stream(streams[k % 2].cuda_stream)
        if k >= 2:
            r.render_packed(4, bufs[k % 4].data_ptr(), bufs[(k - 2) % 4].data_ptr(), slot, frames[k - 2].data_ptr())
        else:
            r.render_packed(4, bufs[k % 4].data_ptr())
    torch.cuda.synchronize()
    ref, _ = _oracle(v, i, n, W, H, nb=4, cam=CULL_CAMS[1])
    for k in range(4):
        _assert_same(frames[k].cpu().numpy().reshape(-1), ref, f"kernel {kernel} frame {k}")


# ---- slotted partition (pt_set_partition_slots) -----------------------------
@pytest.mark.parametrize("slots", [[2, 1, 3], [6, 8, 8, 8], [1, 5]])
def test_partition_slots_sum_and_sparse_exchange(slots):
    """Unequal shares: the -0/+0 cleared partials of all ranks sum to the
    single-GPU frame; the dense tile gather and the sparse live-item exchange
    with pt_render_packed (the root assembling every rank's slot) give it
    bitwise too; the ranks' item counts follow the slots."""
    import torch
    v, i, n = _box()
    W, H, nb = 150, 70, 4
    N = len(slots)
    want, _ = _oracle(v, i, n, W, H, nb=nb, cam=CULL_CAMS[1])
    acc = np.full(W * H * 4, -0.0, np.float32)
    rs = []
    for rank in range(N):
        r = _setup(v, i, n, cam=CULL_CAMS[1])
        r.set_partition(N, rank, slots)
        r.resize_and_clear(W, H)
        r.render(0, nb)
        acc = (acc + r.read_accum()).astype(np.float32)
        owned = ptamd.partition_owned(W, H, N, rank, slots).reshape(-1)
        assert r.tiles_owned() * 256 >= np.count_nonzero(owned)
        rs.append(r)
    _assert_same(acc, want, f"sum over slots {slots}")
    # dense tiles: pack every rank's owned tiles, unpack them all on rank 0
    frame = torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda")
    for k, r in enumerate(rs):
        buf = torch.empty((max(r.tiles_owned(), 1) * 256 * 4,), dtype=torch.float32, device="cuda")
        r.tiles_pack(buf.data_ptr())
        r.synchronize()
        rs[0].tiles_unpack(buf.data_ptr(), k, frame.data_ptr())
        rs[0].synchronize()
    _assert_same(frame.cpu().numpy().reshape(-1), want, f"tile gather, slots {slots}")
    # sparse: render_packed on every rank, assembly on the root
    per = rs[0].items_live(0)[1]
    counts = [rs[0].items_live(k)[0] for k in range(N)]
    slot = max(4, max(counts) * per * 4)
    src = torch.full((N, slot), float("nan"), dtype=torch.float32, device="cuda")
    for k, r in enumerate(rs):
        r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
        r.render_packed(nb, src[k].data_ptr())
        r.synchronize()
    frame2 = torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda")
    rs[0].items_unpack_all(src.data_ptr(), slot, frame2.data_ptr())
    rs[0].synchronize()
    _assert_same(frame2.cpu().numpy().reshape(-1), want, f"sparse exchange, slots {slots}")
    for bad in ([0] + slots[1:], [65] + slots[1:]):   # 1..64 slots per rank
        with pytest.raises(ptamd.PTError):
            rs[0].set_partition(N, 0, bad)
    with pytest.raises(ptamd.PTError):
        rs[0].set_partition(N, 0, slots[:-1])


def test_reslotting_one_renderer_keeps_item_lists_right():
    """Re-slotting a live context ([3,3,1] -> [3,2,2]: same period, count and
    first slot position for rank 0, different tiles) must rebuild the cached
    compact-launch item lists: the -0/+0 partials of the re-slotted renderers
    still sum to the oracle's frame, and each rank's sparse live-item pack
    assembles it (items_key lacked the other slot positions)."""
    import torch
    v, i, n = _box()
    W, H, nb = 150, 70, 3
    want, _ = _oracle(v, i, n, W, H, nb=nb, cam=CULL_CAMS[1])
    rs = [_setup(v, i, n, cam=CULL_CAMS[1]) for _ in range(3)]
    for slots in ([3, 3, 1], [3, 2, 2], [1, 1, 1]):
        acc = np.full(W * H * 4, -0.0, np.float32)
        for rank, r in enumerate(rs):
            r.set_partition(3, rank, slots)
            r.resize_and_clear(W, H)
            r.render(0, nb)
            acc = (acc + r.read_accum()).astype(np.float32)
        _assert_same(acc, want, f"sum after re-slotting to {slots}")
        per = rs[0].items_live(0)[1]
        slot = max(max(rs[0].items_live(k)[0] for k in range(3)) * per * 4, 4)
        recv = torch.zeros((3, slot), dtype=torch.float32, device="cuda")
        for rank, r in enumerate(rs):
            r.items_pack(recv[rank].data_ptr())
            r.synchronize()
        frame = torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda")
        rs[0].items_unpack_all(recv.data_ptr(), slot, frame.data_ptr())
        rs[0].synchronize()
        _assert_same(frame.cpu().numpy().reshape(-1), want, f"sparse exchange after re-slotting to {slots}")


@pytest.mark.parametrize("scene", ["box", "sphere"])
def test_count_traced_mode(scene):
    """PT_OPT_COUNT_TRACED: the output is bit-identical, and the three fast
    kernels (path-recursive with the scene in LDS, path-recursive walking
    device memory with paired walks, wavefront pipeline) start the same walks
    and generate the same primaries; the two path-recursive ones also visit
    the same nodes and run the same triangle tests.  The counts sit below the reference's
    exhaustive ones (stats mode) and the primaries equal the live samples."""
    if scene == "box":
        v, i, n = _box()
        cam = scenes.DEFAULT_CAMERA
    else:
        sv, si = scenes.displaced_sphere(3)
        v, i, n, _, _ = ptamd.Scene.from_arrays(sv, si).build_bvh().arrays()
        cam = scenes.camera((0.0, 0.5, 3.0))
    W, H, nb = 160, 96, 4
    ref, ost = _oracle(v, i, n, W, H, nb=nb, cam=cam)
    counts = {}
    for name, lds, kernel, wide in (("lds", 2, 1, 0), ("dev", 0, 1, 0), ("wf", 0, 3, 0), ("wide", 0, 3, 1)):
        if scene == "sphere" and lds == 2:
            continue   # 5K triangles do not fit the LDS variant
        r = _setup(v, i, n, cam=cam, lds=lds)
        r.set_option(ptamd.PT_OPT_KERNEL, kernel)
        r.set_option(ptamd.PT_OPT_WIDE, wide)
        r.set_option(ptamd.PT_OPT_COUNT_TRACED, 1)
        r.resize_and_clear(W, H)
        r.reset_stats()
        r.render(0, nb)
        _assert_same(r.read_accum(), ref, f"{scene} {name} counting")
        assert r.last_kernel() == kernel
        counts[name] = r.traced()
    first = next(iter(counts.values()))
    for name, c in counts.items():
        # every kernel starts the same walks and generates the same primaries
        for k in ("closest_walks", "shadow_walks", "primaries"):
            assert c[k] == first[k], (name, k, c, first)
    if "lds" in counts:   # the two path-recursive kernels do the same node visits and tests
        assert counts["lds"] == counts["dev"]
    # the wavefront kernel queues shadow leaves (PT_WF_SHADOW_QUEUE): a shadow
    # walk may run a few nodes past its occluder before the queue is tested
    assert counts["wf"]["nodes"] >= counts["dev"]["nodes"]
    assert counts["wf"]["tri_tests"] >= counts["dev"]["tri_tests"]
    # the culled wide walk: 4-wide nodes, nearest first, culled past the best hit
    assert counts["wide"]["nodes"] < counts["dev"]["nodes"]
    if scene == "sphere":
        assert counts["wide"]["tri_tests"] < counts["dev"]["tri_tests"]
    walks = first["closest_walks"] + first["shadow_walks"]
    assert 0 < walks < int(ost[0])
    assert 0 < first["nodes"] < int(ost[1])
    assert first["tri_tests"] <= int(ost[2])
    assert 0 < first["primaries"] <= W * H * nb
    # culling off: every sample generates its primary ray
    r = _setup(v, i, n, cam=cam, lds=0)
    r.set_option(ptamd.PT_OPT_PRIMARY_CULL, 0)
    r.set_option(ptamd.PT_OPT_COUNT_TRACED, 1)
    r.resize_and_clear(W, H)
    r.reset_stats()
    r.render(0, nb)
    assert r.traced()["primaries"] == W * H * nb
    _assert_same(r.read_accum(), ref, f"{scene} counting, culling off")


# ---- culled wide walk (PT_OPT_WIDE, wide_walk.h) ---------------------------

def _wide_case(case):
    if case == "sphere":
        sv, si = scenes.displaced_sphere(4)
        return sv, si, scenes.camera((0.0, 0.5, 3.0)), scenes.REFERENCE_LIGHT, False
    if case == "cloud_int_bits":
        sv, si = scenes.random_triangles(20000, seed=7)
        return sv, si, scenes.camera((0.3, 0.2, 2.2)), scenes.REFERENCE_LIGHT, True
    if case == "dense_cloud":
        sv, si = scenes.random_triangles(50000, seed=9, spread=0.3, size=0.004)
        return sv, si, scenes.camera((0.1, 0.2, 1.2)), scenes.REFERENCE_LIGHT, False
    if case == "grid2lights":
        sv, si = scenes.grid_mesh(6)
        two = np.concatenate([scenes.REFERENCE_LIGHT,
                              ptamd.pack_light([0.5, 0.5, 1.5], [0, 0, -1], [2, 4, 8], [0.5, 1.0])])
        return sv, si, scenes.camera((0.0, 0.0, 3.0)), two, False
    s = ptamd.Scene.load_obj(scenes.BOX_OBJ)   # "box": big triangles, nothing culled
    v, i, _, _, _ = s.build_bvh().arrays()
    return v, i, scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, False


@pytest.mark.parametrize("node", [64, 128])
@pytest.mark.parametrize("build", [1, 0], ids=["sah", "reference_tree"])
@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("case", ["sphere", "cloud_int_bits", "dense_cloud", "grid2lights", "box"])
def test_wide_walk_matches_oracle(case, mode, build, node):
    """The culled wide walk (wavefront pipeline, device-memory scene) gives the
    oracle's frame bit for bit, over either grouping of the reference's leaves
    (PT_OPT_WIDE_BUILD: binned SAH, or the reference's own tree) and either
    node layout (PT_OPT_WIDE_NODE: 64-B nodes with grid-rounded boxes and
    exact leaf tests, or float boxes); mode 2 hands every odd ray of each
    round to the exact threaded walk in the shading kernel (the path rays
    with a zero direction component take)."""
    sv, si, cam, lights, int_bits = _wide_case(case)
    v, i, n, _, _ = ptamd.Scene.from_arrays(sv, si).build_bvh(int_bits=int_bits).arrays()
    r = _setup(v, i, n, cam=cam, lights=lights, int_bits=int_bits, lds=0)
    r.set_option(ptamd.PT_OPT_WIDE_BUILD, build)
    r.upload_scene(v, i, n, int_bits=int_bits)   # the build option is read at upload
    r.set_option(ptamd.PT_OPT_KERNEL, 3)
    r.set_option(ptamd.PT_OPT_WIDE, mode)
    r.set_option(ptamd.PT_OPT_WIDE_NODE, node)
    info = r.wide_info()
    assert info[0] > 0 and info[1] > 0, info
    r.resize_and_clear(80, 52)
    r.render(1, 4)
    ref, _ = _oracle(v, i, n, 80, 52, first=1, nb=4, cam=cam, lights=lights, int_bits=int_bits)
    _assert_same(r.read_accum(), ref, f"wide walk {case} mode {mode}")


def test_wide_walk_refused_tree_keeps_exact_walk():
    """A tree whose parent box does not contain a child's (not a
    BoundingVolumeHierarchy.cpp tree) gets no wide walk: pt_wide_info says why,
    and the frame (exact threaded walk) still equals the oracle's on the same
    arrays."""
    sv, si = scenes.displaced_sphere(3)
    v, i, n, _, _ = ptamd.Scene.from_arrays(sv, si).build_bvh().arrays()
    n = n.copy()
    n[0, 0] = n[1, 0] + 0.05   # the root's min.x inside its right child's box
    r = _setup(v, i, n, cam=scenes.camera((0.0, 0.5, 3.0)), lds=0)
    info = r.wide_info()
    assert info[0] == 0 and "contain" in info[2]
    r.set_option(ptamd.PT_OPT_KERNEL, 3)
    r.resize_and_clear(48, 40)
    r.render(0, 2)
    ref, _ = _oracle(v, i, n, 48, 40, nb=2, cam=scenes.camera((0.0, 0.5, 3.0)))
    _assert_same(r.read_accum(), ref, "refused wide tree")


@pytest.mark.parametrize("tail", [1 << 30, 3000, 1])
@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("node", [64, 128])
@pytest.mark.parametrize("case", ["sphere", "cloud_int_bits", "dense_cloud", "grid2lights", "box"])
def test_wavefront_tail_kernel_matches_oracle(case, node, mode, tail):
    """PT_OPT_WF_TAIL: once a round's list is shorter than `tail` rays,
    wf_tail_kernel runs every remaining path to its end in one launch (walk,
    path_step, the next walk in the same lane).  2^30: the whole frame in the
    tail kernel from the first list; 3000: the late rounds; 1: never (the
    rounds alone).  Over a stale accumulator, with mode 2 handing every odd
    ray of the rounds to the exact walk: the oracle's frame bit for bit, and
    the counting mode's walks equal to the rounds' own."""
    sv, si, cam, lights, int_bits = _wide_case(case)
    v, i, n, _, _ = ptamd.Scene.from_arrays(sv, si).build_bvh(int_bits=int_bits).arrays()
    W, H = 80, 52
    ref, _ = _oracle(v, i, n, W, H, nb=2, cam=cam, lights=lights, int_bits=int_bits)
    ref, _ = _oracle(v, i, n, W, H, first=2, nb=3, cam=cam, lights=lights, int_bits=int_bits, accum=ref)
    r = _setup(v, i, n, cam=cam, lights=lights, int_bits=int_bits, lds=0)
    r.set_option(ptamd.PT_OPT_KERNEL, 3)
    r.set_option(ptamd.PT_OPT_WIDE, mode)
    r.set_option(ptamd.PT_OPT_WIDE_NODE, node)
    r.set_option(ptamd.PT_OPT_WF_TAIL, tail)
    r.resize_and_clear(W, H)
    r.render(0, 2)
    r.render(2, 3)
    _assert_same(r.read_accum(), ref, f"tail kernel {case} node {node} mode {mode} tail {tail}")


@pytest.mark.parametrize("case", ["sphere", "cloud_int_bits"])
def test_wavefront_tail_kernel_counts_and_two_streams(case):
    """The tail kernel's counting variant starts the same closest-hit walks as
    the rounds (shadow walks differ only by the fused walks' bookkeeping:
    both count each walk once), and with two streams (each half's own lists
    and counters) the frame is still the oracle's."""
    sv, si, cam, lights, int_bits = _wide_case(case)
    v, i, n, _, _ = ptamd.Scene.from_arrays(sv, si).build_bvh(int_bits=int_bits).arrays()
    W, H, nb = 120, 72, 2
    ref, _ = _oracle(v, i, n, W, H, nb=nb, cam=cam, lights=lights, int_bits=int_bits)
    got = {}
    for tail in (0, 1 << 30, 5000):
        r = _setup(v, i, n, cam=cam, lights=lights, int_bits=int_bits, lds=0)
        r.set_option(ptamd.PT_OPT_KERNEL, 3)
        r.set_option(ptamd.PT_OPT_WF_TAIL, tail)
        r.set_option(ptamd.PT_OPT_COUNT_TRACED, 1)
        r.reset_stats()
        r.resize_and_clear(W, H)
        r.render(0, nb)
        _assert_same(r.read_accum(), ref, f"counting tail {tail} {case}")
        got[tail] = r.traced()
        r.set_option(ptamd.PT_OPT_COUNT_TRACED, 0)
        r.set_option(ptamd.PT_OPT_WF_STREAMS, 2)
        r.resize_and_clear(W, H)
        r.render(0, nb)
        _assert_same(r.read_accum(), ref, f"two streams tail {tail} {case}")
    for tail in (1 << 30, 5000):
        assert got[tail]["closest_walks"] == got[0]["closest_walks"], (tail, got)
        assert got[tail]["primaries"] == got[0]["primaries"], (tail, got)


@pytest.mark.parametrize("case", ["sphere", "cloud_int_bits"])
def test_wavefront_two_streams(case):
    """PT_OPT_WF_STREAMS 2: the chunk's pixels as two halves on two streams
    (own lists, counters and stack overflow areas), over a stale accumulator
    and a culled camera: the oracle's frame."""
    sv, si, cam, lights, int_bits = _wide_case(case)
    v, i, n, _, _ = ptamd.Scene.from_arrays(sv, si).build_bvh(int_bits=int_bits).arrays()
    W, H = 200, 120
    ref, _ = _oracle(v, i, n, W, H, nb=2, cam=cam, lights=lights, int_bits=int_bits)
    ref, _ = _oracle(v, i, n, W, H, first=2, nb=3, cam=cam, lights=lights, int_bits=int_bits, accum=ref)
    r = _setup(v, i, n, cam=cam, lights=lights, int_bits=int_bits, lds=0)
    r.set_option(ptamd.PT_OPT_KERNEL, 3)
    r.set_option(ptamd.PT_OPT_WF_STREAMS, 2)
    r.resize_and_clear(W, H)
    r.render(0, 2)
    r.render(2, 3)
    _assert_same(r.read_accum(), ref, f"two streams {case}")


@pytest.mark.parametrize("case", ["sphere", "cloud_int_bits"])
def test_wide_walk_partitioned_ranks_sum_to_oracle(case):
    """Tile shares of a device-memory scene on the culled wide walk (the
    wavefront pipeline as each rank of a multi-GPU frame runs it: equal
    shares over 3 ranks and unequal slotted shares over 2): the ranks'
    +0/-0 partial frames sum to the oracle's full frame bit for bit."""
    sv, si, cam, lights, int_bits = _wide_case(case)
    v, i, n, _, _ = ptamd.Scene.from_arrays(sv, si).build_bvh(int_bits=int_bits).arrays()
    W, H, nb = 96, 64, 3
    ref, _ = _oracle(v, i, n, W, H, nb=nb, cam=cam, lights=lights, int_bits=int_bits)
    for nranks, slots in ((3, None), (2, [3, 1])):
        acc = np.full(W * H * 4, -0.0, np.float32)   # -0 is the IEEE additive identity
        for rank in range(nranks):
            r = _setup(v, i, n, cam=cam, lights=lights, int_bits=int_bits, lds=0)
            r.set_option(ptamd.PT_OPT_KERNEL, 3)
            if slots is None:
                r.set_partition(nranks, rank)
            else:
                r.set_partition(nranks, rank, slots)
            assert r.wide_info()[0] > 0
            r.resize_and_clear(W, H)
            r.render(0, nb)
            acc = (acc + r.read_accum()).astype(np.float32)
        _assert_same(acc, ref.reshape(-1), f"wide walk {case}, {nranks} ranks, slots {slots}")


def test_wide_walk_reupload_deeper_scene():
    """A context that rendered a shallow wide tree, then gets a scene whose
    wide tree needs a deeper stack (the per-lane overflow area is sized by the
    scene's stack bound), renders the deeper scene's oracle frame;
    and a third upload back to the shallow scene as well."""
    shallow = scenes.random_triangles(64, seed=4, spread=0.4, size=0.05)
    deep = scenes.random_triangles(200000, seed=5, spread=0.6, size=0.003)
    cam = scenes.camera((0.0, 0.1, 1.6))
    r = None
    depths = []
    for sv, si in (shallow, deep, shallow):
        v, i, n, _, _ = ptamd.Scene.from_arrays(sv, si).build_bvh().arrays()
        if r is None:
            r = _setup(v, i, n, cam=cam, lds=0)
            r.set_option(ptamd.PT_OPT_KERNEL, 3)
        else:
            r.upload_scene(v, i, n)
        info = r.wide_info()
        assert info[0] > 0, info
        depths.append(info[1])
        r.resize_and_clear(72, 56)
        r.render(0, 2)
        ref, _ = _oracle(v, i, n, 72, 56, nb=2, cam=cam)
        _assert_same(r.read_accum(), ref, f"re-upload, stack bound {info[1]}")
    assert depths[1] > depths[0], depths


@pytest.mark.parametrize("fuse", [0, 1])
@pytest.mark.parametrize("case", ["sphere", "grid2lights", "cloud_int_bits"])
def test_wide_walk_fused_shadow_rays(case, fuse):
    """PT_OPT_WF_FUSE: the trace kernel walks a closest hit's first-light
    shadow ray in the same lane (the shading kernel takes both answers) or
    not; over a stale accumulator, depth 3, either way the oracle's frame."""
    sv, si, cam, lights, int_bits = _wide_case(case)
    v, i, n, _, _ = ptamd.Scene.from_arrays(sv, si).build_bvh(int_bits=int_bits).arrays()
    W, H = 96, 72
    ref, _ = _oracle(v, i, n, W, H, nb=1, depth=3, cam=cam, lights=lights, int_bits=int_bits)
    ref, _ = _oracle(v, i, n, W, H, first=1, nb=3, depth=3, cam=cam, lights=lights, int_bits=int_bits, accum=ref)
    r = _setup(v, i, n, cam=cam, lights=lights, int_bits=int_bits, lds=0, depth=3)
    r.set_option(ptamd.PT_OPT_KERNEL, 3)
    r.set_option(ptamd.PT_OPT_WF_FUSE, fuse)
    r.resize_and_clear(W, H)
    r.render(0, 1)
    r.render(1, 3)
    _assert_same(r.read_accum(), ref, f"fuse {fuse} {case}")


@pytest.mark.parametrize("first,nb", [(0, 16), (3, 6), (7, 9), (1000, 3)])
def test_one_lane_fold_over_stale_accumulator(first, nb):
    """The one-lane-per-pixel fold (PT_OPT_SAMPLE_LANES 1: each lane folds its
    own samples, no hand-off; batch + 1 a power of two divides by multiplying,
    a running alpha of 1 stays 1) against the oracle's running mean (:467-469)
    over an accumulator holding arbitrary values, alpha included, from batch
    `first` on."""
    v, i, n = _box()
    W, H = 80, 56
    rng = np.random.default_rng(first + nb)
    stale = rng.uniform(-3.0, 3.0, W * H * 4).astype(np.float32)
    stale[3::4][::3] = 1.0    # some pixels with alpha exactly 1
    r = _setup(v, i, n)
    r.set_option(ptamd.PT_OPT_SAMPLE_LANES, 1)
    r.set_option(ptamd.PT_OPT_PRIMARY_CULL, 0)
    import torch
    buf = torch.from_numpy(stale.copy()).to("cuda:0")
    r.bind_accum(buf.data_ptr(), W, H)
    r.render(first, nb)
    ref, _ = O.render(v, i, n.reshape(-1), scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, W, H, first_batch=first,
                      n_batches=nb, accum=stale.copy())
    _assert_same(r.read_accum(), ref, f"one-lane fold from batch {first}, {nb} batches")


def test_wavefront_grid_fraction_is_output_invariant():
    """PT_OPT_WF_GRID (a smaller persistent traversal grid) and
    PT_OPT_WF_REFILL (the idle-lane count at which a wave claims new rays)
    change which lane walks which ray, never a bit of the frame."""
    sv, si = scenes.displaced_sphere(3)
    s = ptamd.Scene.from_arrays(sv, si).build_bvh()
    v, i, n, _, _ = s.arrays()
    cam = scenes.camera((0.0, 0.5, 3.0))
    frames = []
    cases = ((100, 0), (37, 0), (5, 0), (100, 1), (25, 4), (100, 64))   # (grid %, refill lanes; 0 auto)
    for g, rf in cases:
        r = _setup(v, i, n, cam=cam, lds=0)
        r.set_option(ptamd.PT_OPT_KERNEL, ptamd.KERNEL_WAVEFRONT)
        r.set_option(ptamd.PT_OPT_WF_GRID, g)
        r.set_option(ptamd.PT_OPT_WF_REFILL, rf)
        r.resize_and_clear(160, 96)
        r.render(0, 3)
        assert r.last_kernel() == ptamd.KERNEL_WAVEFRONT
        frames.append(r.read_accum())
    for (g, rf), f in zip(cases[1:], frames[1:]):
        _assert_same(f, frames[0], f"grid {g} %, refill at {rf} idle lanes")
    with pytest.raises(ptamd.PTError):
        r.set_option(ptamd.PT_OPT_WF_GRID, 0)
    with pytest.raises(ptamd.PTError):
        r.set_option(ptamd.PT_OPT_WF_REFILL, 65)
