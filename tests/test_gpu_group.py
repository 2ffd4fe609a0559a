"""One context over several devices (pt_create_multi, SURVEY §8b
`create(device_ordinals[], n)`).

The box this suite runs on has one GPU, so the members share device 0: every
member still owns its own context, stream and tile share, and the group's
exchange runs exactly as across devices (peer stores into the frame on the
first device, or packed tiles copied with hipMemcpyPeerAsync).  Every frame
must be bitwise the single-GPU frame and the oracle's."""
import numpy as np
import pytest

import oracle_lib as O
import ptamd
import scenes

pytestmark = pytest.mark.gpu


def _box():
    s = ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh()
    v, i, n, _, _ = s.arrays()
    return v, i, n


def _setup(r, v, i, n, cam=scenes.DEFAULT_CAMERA, depth=4, int_bits=False):
    r.upload_scene(v, i, n, int_bits=int_bits)
    r.upload_lights(scenes.REFERENCE_LIGHT)
    r.set_camera(cam)
    r.set_params(depth, 3)
    return r


def _same(a, b, what):
    if not np.array_equal(a.view(np.uint32), b.view(np.uint32)):
        bad = np.flatnonzero(a.view(np.uint32) != b.view(np.uint32))
        raise AssertionError(f"{what}: {bad.size} floats differ, first at pixel {bad[0] // 4}: {a[bad[0]]} vs {b[bad[0]]}")


def test_group_of_one_is_a_plain_context():
    v, i, n = _box()
    g = _setup(ptamd.Renderer(devices=[0]), v, i, n)
    assert g.group_info() == ([0], False)
    g.resize_and_clear(96, 64)
    g.render(0, 3)
    ref, _ = O.render(v, i, n.reshape(-1), scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, 96, 64, n_batches=3)
    _same(g.read_accum(), ref, "group of one vs oracle")


@pytest.mark.parametrize("exchange", [0, 1])
@pytest.mark.parametrize("members", [2, 3, 8])
def test_group_frame_equals_single_gpu(members, exchange):
    """Members on device 0 (the only one here); the frame after fused renders,
    progressive dispatches on top, and a fresh frame over a stale image."""
    v, i, n = _box()
    W, H = 160, 100
    g = _setup(ptamd.Renderer(devices=[0] * members), v, i, n)
    g.set_option(ptamd.PT_OPT_GROUP_EXCHANGE, exchange)
    devs, peer = g.group_info()
    assert devs == [0] * members and peer == (exchange == 0)
    one = _setup(ptamd.Renderer(0), v, i, n)
    for r in (g, one):
        r.resize_and_clear(W, H)
        r.render(0, 2)
        r.dispatch(2)
        r.dispatch(3)
    _same(g.read_accum(), one.read_accum(), f"{members} members, exchange {exchange}: batches 0-3")
    ref, _ = O.render(v, i, n.reshape(-1), scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, W, H, n_batches=4)
    _same(g.read_accum(), ref, "group vs oracle")
    # a fresh frame from batch 0 over the old image, as the progressive loop
    # does after a camera change
    cam2 = scenes.camera((0.4, 0.3, 4.0))
    for r in (g, one):
        r.set_camera(cam2)
        r.render(0, 2)
    _same(g.read_accum(), one.read_accum(), "camera change, fresh batch 0")


def test_group_progressive_loop_and_readback():
    v, i, n = _box()
    g = _setup(ptamd.Renderer(devices=[0, 0, 0]), v, i, n)
    g.resize_and_clear(64, 48)
    assert g.progressive_camera(scenes.DEFAULT_CAMERA)
    assert g.progressive_advance(3) == (0, 3)
    t = g.readback_begin()
    assert g.progressive_advance(2) == (3, 2)
    snap = g.readback_end(t)
    ref3, _ = O.render(v, i, n.reshape(-1), scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, 64, 48, n_batches=3)
    _same(snap, ref3, "readback snapshot after 3 batches")
    ref5, _ = O.render(v, i, n.reshape(-1), scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, 64, 48, n_batches=5)
    _same(g.read_accum(), ref5, "5 batches")
    assert not g.progressive_camera(scenes.DEFAULT_CAMERA)
    assert g.progressive_advance(100, limit=7) == (5, 2)


def test_group_stats_sum_to_the_single_gpu_counts():
    v, i, n = _box()
    g = _setup(ptamd.Renderer(devices=[0, 0]), v, i, n)
    one = _setup(ptamd.Renderer(0), v, i, n)
    for r in (g, one):
        r.resize_and_clear(64, 40)
        r.set_stats_mode(True)
        r.reset_stats()
        r.render(0, 2)
    assert g.stats() == one.stats()
    _same(g.read_accum(), one.read_accum(), "stats mode")


def test_group_wavefront_scene_matches_single_gpu():
    """A device-memory scene on the wavefront pipeline with the culled wide
    walk, split over 3 members."""
    sv, si = scenes.displaced_sphere(3)
    s = ptamd.Scene.from_arrays(sv, si).build_bvh()
    v, i, n, _, _ = s.arrays()
    cam = scenes.camera((0.0, 0.5, 3.0))
    g = _setup(ptamd.Renderer(devices=[0, 0, 0]), v, i, n, cam=cam)
    one = _setup(ptamd.Renderer(0), v, i, n, cam=cam)
    for r in (g, one):
        r.set_option(ptamd.PT_OPT_KERNEL, ptamd.KERNEL_WAVEFRONT)
        r.resize_and_clear(128, 96)
        r.render(0, 2)
    assert g.last_kernel() == ptamd.KERNEL_WAVEFRONT
    _same(g.read_accum(), one.read_accum(), "wavefront, 3 members")


def test_group_rejects_share_calls():
    v, i, n = _box()
    g = _setup(ptamd.Renderer(devices=[0, 0]), v, i, n)
    g.resize_and_clear(32, 32)
    with pytest.raises(ptamd.PTError, match="multi-device"):
        g.set_partition(2, 0)
    with pytest.raises(ptamd.PTError, match="multi-device"):
        g.tiles_owned()
    with pytest.raises(ptamd.PTError):
        ptamd.Renderer(devices=[0, 99])


def test_group_check_matches_on_one_device():
    """PT_OPT_GROUP_CHECK 2 runs the peer-store probe on the first render even
    with every member on device 0: the peer-store and staged probe frames
    agree bit for bit, peer stores stay in force, and the frame is the
    single-GPU frame."""
    v, i, n = _box()
    g = _setup(ptamd.Renderer(devices=[0, 0, 0]), v, i, n)
    assert g.group_check()[0] == -1   # one device: not armed by default
    g.set_option(ptamd.PT_OPT_GROUP_CHECK, 2)
    g.resize_and_clear(96, 64)
    assert g.group_check()[0] == -2   # armed: runs on the next render
    g.render(0, 3)
    state, ms_peer, ms_staged = g.group_check()
    assert state == 0 and ms_peer > 0 and ms_staged > 0
    assert g.group_info()[1] is True
    ref, _ = O.render(v, i, n.reshape(-1), scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, 96, 64, n_batches=3)
    _same(g.read_accum(), ref, "after the check")


def test_group_check_mismatch_falls_back_to_staged_copies():
    """PT_OPT_GROUP_CHECK 3 forces the probe comparison to fail (one flipped
    bit, a test-only option): the context must fall back to the staged
    exchange for good and still produce the single-GPU frame -- including
    the history accumulated before the switch."""
    v, i, n = _box()
    W, H = 128, 80
    g = _setup(ptamd.Renderer(devices=[0, 0]), v, i, n)
    g.resize_and_clear(W, H)
    g.render(0, 2)                        # peer stores, no check yet
    assert g.group_info()[1] is True
    g.set_option(ptamd.PT_OPT_GROUP_CHECK, 3)
    g.dispatch(2)                         # the check runs first, fails, staged from here on
    state, _, _ = g.group_check()
    assert state == 1
    assert g.group_info()[1] is False
    g.dispatch(3)
    ref, _ = O.render(v, i, n.reshape(-1), scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, W, H, n_batches=4)
    _same(g.read_accum(), ref, "batches 0-1 by peer stores, 2-3 by staged copies")


def test_group_exchange_switch_keeps_the_accumulation():
    """switching to the staged exchange between progressive
    advances must continue the frame's accumulation (each member's buffer
    starts from the frame), and switching back too."""
    v, i, n = _box()
    W, H = 96, 64
    g = _setup(ptamd.Renderer(devices=[0, 0, 0]), v, i, n)
    g.resize_and_clear(W, H)
    assert g.progressive_camera(scenes.DEFAULT_CAMERA)
    assert g.progressive_advance(2) == (0, 2)
    g.set_option(ptamd.PT_OPT_GROUP_EXCHANGE, 1)
    assert g.progressive_advance(2) == (2, 2)
    g.set_option(ptamd.PT_OPT_GROUP_EXCHANGE, 0)
    assert g.progressive_advance(1) == (4, 1)
    ref, _ = O.render(v, i, n.reshape(-1), scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, W, H, n_batches=5)
    _same(g.read_accum(), ref, "exchange 0 -> 1 -> 0 across advances")


def _devices():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif("_devices() < 2")
@pytest.mark.parametrize("exchange", [0, 1])
def test_group_on_distinct_devices(exchange):
    """members on distinct GPUs -- peer stores into the
    first device's frame over xGMI (after the context's own probe check) or
    staged copies -- bitwise the single-GPU frame, through the progressive
    loop and a readback.  Skipped on a one-GPU box (every box this build
    had); the driver's multi-GPU node runs it."""
    nd = min(_devices(), 4)
    v, i, n = _box()
    W, H = 160, 100
    g = _setup(ptamd.Renderer(devices=list(range(nd))), v, i, n)
    g.set_option(ptamd.PT_OPT_GROUP_EXCHANGE, exchange)
    g.resize_and_clear(W, H)
    assert g.progressive_camera(scenes.DEFAULT_CAMERA)
    assert g.progressive_advance(3) == (0, 3)
    t = g.readback_begin()
    assert g.progressive_advance(2) == (3, 2)
    snap = g.readback_end(t)
    if exchange == 0:
        assert g.group_check()[0] in (0, 1)   # the probe ran; 1 would mean staged copies took over
    ref3, _ = O.render(v, i, n.reshape(-1), scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, W, H, n_batches=3)
    _same(snap, ref3, f"{nd} devices, exchange {exchange}: snapshot after 3 batches")
    ref5, _ = O.render(v, i, n.reshape(-1), scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, W, H, n_batches=5)
    _same(g.read_accum(), ref5, f"{nd} devices, exchange {exchange}: 5 batches")


def test_group_check_probe_frames_are_not_counted():
    """The peer-store probe frames (PT_OPT_GROUP_CHECK) run with the members'
    counters off: stats mode and traced counts after the checked render are
    the single-GPU frame's."""
    v, i, n = _box()
    g = _setup(ptamd.Renderer(devices=[0, 0]), v, i, n)
    one = _setup(ptamd.Renderer(0), v, i, n)
    g.set_option(ptamd.PT_OPT_GROUP_CHECK, 2)
    for r in (g, one):
        r.resize_and_clear(64, 40)
        r.set_stats_mode(True)
        r.reset_stats()
        r.render(0, 2)
    assert g.group_check()[0] == 0
    assert g.stats() == one.stats()
    g.set_stats_mode(False)
    one.set_stats_mode(False)
    g.resize_and_clear(64, 40)   # re-arms the check
    for r in (g, one):
        r.set_option(ptamd.PT_OPT_COUNT_TRACED, 1)
        r.reset_stats()
        r.render(0, 2)
    assert g.group_check()[0] == 0
    assert g.traced() == one.traced()


def test_group_check_rearmed_after_a_failed_render():
    """A render that fails before the probe can run (no scene yet) leaves the
    peer-store check armed for the next render."""
    v, i, n = _box()
    g = ptamd.Renderer(devices=[0, 0])
    g.set_option(ptamd.PT_OPT_GROUP_CHECK, 2)
    g.resize_and_clear(48, 32)
    with pytest.raises(ptamd.PTError):
        g.render(0, 1)
    assert g.group_check()[0] == -2
    _setup(g, v, i, n)
    g.render(0, 2)
    assert g.group_check()[0] == 0
    ref, _ = O.render(v, i, n.reshape(-1), scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, 48, 32, n_batches=2)
    _same(g.read_accum(), ref, "after a failed first render")
