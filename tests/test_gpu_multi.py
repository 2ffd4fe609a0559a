"""The product's N > 1 path on the GPU, in fresh processes.

bench.py --gpus 2 under torch.distributed.run: two ranks, each driving
libptamd on device 0 (a 1-GPU box; RCCL needs one GPU per rank, so the
collectives run on gloo staged through the host), render their tile shares,
exchange them -- the sparse live-item gather with pt_render_packed's fused
assembly, or the -0/+0 SUM reduce -- and rank 0 checks the assembled frames
bitwise against a single-GPU render (--verify).  The children are started as
subprocesses, never exec'd over this (GPU-initialised) test process."""
import json
import os
import socket
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd, env, timeout=180):
    """subprocess.run with the children's stacks on a hang: bench.py dumps
    every thread's stack to stderr after PT_BENCH_TRACEBACK_AFTER_S, and a
    timeout reports the tail of what the children wrote."""
    # a collective one rank never reaches fails after 90 s with the others'
    # stacks (bench.py's process-group timeout), inside the test's own limit
    env = dict(env, PT_BENCH_TRACEBACK_AFTER_S=str(timeout - 30), PT_BENCH_PG_TIMEOUT_S="90")
    env.setdefault("PT_BENCH_DETAIL", os.path.join(tempfile.mkdtemp(prefix="ptbench"), "detail.json"))
    try:
        return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    except subprocess.TimeoutExpired as e:
        def tail(x):
            return (x.decode(errors="replace") if isinstance(x, bytes) else (x or ""))[-6000:]
        raise AssertionError(f"timed out after {timeout} s\nstdout:\n{tail(e.stdout)}\nstderr:\n{tail(e.stderr)}")


def _record(res):
    """bench.py's full record of a run: the last stdout line is the compact
    line the driver parses (at most bench.LINE_MAX_BYTES), naming the detail
    file that holds the full record."""
    last = res.stdout.strip().splitlines()[-1]
    assert len(last) <= 6144, len(last)
    line = json.loads(last)
    return json.load(open(line["detail_file"]))


# torchrun --standalone binds its rendezvous store to a port of its own
# choosing (a port picked here and handed over could be taken in between:
# EADDRINUSE); the single-rank native test sets MASTER_PORT itself.
def _free_port():
    """A free port below the ephemeral range (32768+), so no client socket
    of an earlier run can be holding it."""
    import random
    for _ in range(200):
        p = random.randrange(20000, 30000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    raise RuntimeError("no free port in 20000-29999")


@pytest.mark.parametrize("collective,extra", [("gather", []), ("reduce", []), ("gather", ["--assemble", "0"]),
                                             ("ipc", [])])
def test_two_rank_bench_verifies_bitwise(collective, extra):
    env = dict(os.environ, PT_BENCH_DEVICE="0", PT_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--standalone", "--local-addr", "127.0.0.1",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "2", "--verify",
           "--no-scene-legs", "--collective", collective] + extra
    res = _run(cmd, env)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-4000:]
    out = _record(res)
    assert out["n_gpus"] == 2
    assert out["verified_bitwise_vs_single_gpu"] is True
    assert out["config"]["rays_traced"] > 0
    if collective == "ipc":
        # the ranks rendered straight into the root's frame buffers (HIP IPC
        # within the one GPU), no fallback to the gather
        assert "exchange_fallback" not in out["config"], out["config"]
        assert out["config"]["parallelism"] == "tiles2-ipc-peer-stores"


@pytest.mark.parametrize("streams", [2, 3])
def test_native_step_loop_single_rank_rccl(streams):
    """pt_dist_run (RCCL driven from C++) at N = 1 on the box: a real RCCL
    communicator of one rank, the grouped self send/recv, the two- or
    three-stream pipeline (frames k-2 / k-3 assembled in frame k's launch),
    the fused and the trailing assemblies -- checked bitwise by bench.py's
    self-check and by --verify over every assembled frame."""
    env = dict(os.environ, PT_BENCH_FORCE_DIST="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "7", "--warmup", "3", "--verify",
           "--no-scene-legs", "--no-cpu-baseline", "--streams", str(streams)]
    res = _run(cmd, env)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-4000:]
    out = _record(res)
    assert out["config"]["step_loop"].startswith("native"), res.stderr[-2000:]
    assert out["verified_bitwise_vs_single_gpu"] is True


SHIM = os.path.join(ROOT, "tests", "_build", "libptdistshim.so")


@pytest.mark.parametrize("streams", [1, 2, 3])
def test_native_step_loop_two_ranks_grouped_send_recv(streams):
    """pt_dist_run's N > 1 schedule with two processes on the one GPU: the
    grouped ncclSend/ncclRecv of every frame go through the stand-in
    (tests/dist_shim.cpp via PT_RCCL_LIB: the same bytes moved between the
    processes over hipIpc handles), the root receives rank 1's live items
    into its receive sets and assembles frames k-max(2, streams) inside its
    render launches.  bench.py's 6-frame self-check and --verify compare every
    assembled frame bitwise with a single-GPU render.  (Throughput over xGMI
    is not measured by this: the stand-in is host-synchronous.)"""
    assert os.path.exists(SHIM), "build it first: make -C tests"
    env = dict(os.environ, PT_BENCH_DEVICE="0", PT_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1",
               PT_RCCL_LIB=SHIM)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--standalone", "--local-addr", "127.0.0.1",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "3", "--verify",
           "--no-scene-legs", "--streams", str(streams)]
    res = _run(cmd, env)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-4000:]
    out = _record(res)
    assert out["n_gpus"] == 2
    assert out["config"]["step_loop"] == "native (pt_dist_run, PT_RCCL_LIB stand-in)", res.stderr[-2000:]
    assert out["verified_bitwise_vs_single_gpu"] is True


def test_two_rank_scene_legs_reduce_bitwise():
    """bench.py's N > 1 scene legs (configs 4 and 5 across the GPUs, here at
    reduced size): each rank renders its tiles of the large-scene frame on
    the wavefront pipeline, one SUM reduce of the -0/+0-cleared
    accumulators, and rank 0 checks the reduced frame bitwise against its own
    whole-frame render.  The 2^24-node int encoding is exercised by the
    full-size run (the driver's multi-GPU bench)."""
    env = dict(os.environ, PT_BENCH_DEVICE="0", PT_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1",
               PT_BENCH_DIST_LEGS="config4 sphere 640 360 4 8 2;config5 synthetic:300000 480 270 2 4 2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--standalone", "--local-addr", "127.0.0.1",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1"]
    res = _run(cmd, env)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-4000:]
    out = _record(res)
    legs = out["configs"]
    assert set(legs) == {"config4", "config5"}, legs
    for key, leg in legs.items():
        assert "error" not in leg, leg
        assert leg["n_gpus"] == 2
        assert leg["verified_bitwise_vs_single_gpu"] is True, key
        assert leg["config"]["rays_per_frame"] > 0 and leg["config"]["rays_traced"] > 0


@pytest.mark.parametrize("streams", [2, 3])
def test_native_loop_back_to_back_calls(streams):
    """Two pt_dist_run calls with no synchronize in between: the
    second call's first frames reuse the send slots, receive sets and frame
    buffers the first call's last gathers and trailing assemblies may still
    be using; pt_dist_run's entry barrier orders them.  A one-rank real RCCL
    communicator in this process; every frame buffer must hold the
    single-GPU frame afterwards.  (The two-process schedule runs through the
    host-synchronous stand-in, which cannot show overlap hazards: they are
    covered by this ordering and by the driver's multi-GPU runs.)"""
    import numpy as np
    import torch
    import ptamd
    import scenes
    scene = ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh()
    v, i, n, _, _ = scene.arrays()

    def setup():
        r = ptamd.Renderer(0)
        r.upload_scene(v, i, n)
        r.upload_lights(scenes.REFERENCE_LIGHT)
        r.set_camera(scenes.DEFAULT_CAMERA)
        r.set_params(4, 3)
        r.resize_and_clear(320, 200)
        return r
    one = setup()
    one.render(0, 4)
    want = one.read_accum().view(np.uint32)
    r = setup()
    r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
    r.render(0, 4)   # fixes the item layout
    r.dist_init(ptamd.Renderer.dist_unique_id(), 1, 0)
    frames = torch.full((3, 200, 320, 4), float("nan"), dtype=torch.float32, device="cuda:0")
    r.dist_run(4, 5, frames.data_ptr(), 3, n_streams=streams)
    r.dist_run(4, 4, frames.data_ptr(), 3, n_streams=streams)
    r.dist_wait(30000)
    r.synchronize()
    for f in range(3):
        got = frames[f].cpu().numpy().reshape(-1).view(np.uint32)
        assert np.array_equal(got, want), f"frame buffer {f}"
    r.dist_finalize()


def test_native_loop_assembles_culled_items_once_per_buffer_and_layout():
    """The root writes a frame buffer's culled items -- the constant
    (0,0,0,1) -- in its first whole assembly of a layout and afterwards
    rebuilds only the live items there.  Buffers new to
    the loop, and every buffer after a camera change (another culled set),
    get a whole assembly again: each must hold the single-GPU frame."""
    import numpy as np
    import torch
    import ptamd
    import scenes
    scene = ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh()
    v, i, n, _, _ = scene.arrays()
    cam2 = scenes.camera((0.5, -0.3, 3.5))

    def setup(cam):
        r = ptamd.Renderer(0)
        r.upload_scene(v, i, n)
        r.upload_lights(scenes.REFERENCE_LIGHT)
        r.set_camera(cam)
        r.set_params(4, 3)
        r.resize_and_clear(320, 200)
        return r

    def want(cam):
        one = setup(cam)
        one.render(0, 4)
        return one.read_accum().view(np.uint32).copy()

    w1, w2 = want(scenes.DEFAULT_CAMERA), want(cam2)
    assert not np.array_equal(w1, w2)
    r = setup(scenes.DEFAULT_CAMERA)
    r.set_option(ptamd.PT_OPT_FRESH_BATCH0, 1)
    r.render(0, 4)   # fixes the item layout
    r.dist_init(ptamd.Renderer.dist_unique_id(), 1, 0)

    def check(frames, w, what):
        r.dist_wait(30000)
        r.synchronize()
        for f in range(frames.shape[0]):
            got = frames[f].cpu().numpy().reshape(-1).view(np.uint32)
            assert np.array_equal(got, w), f"{what}, frame buffer {f}"

    a = torch.full((3, 200, 320, 4), float("nan"), dtype=torch.float32, device="cuda:0")
    r.dist_run(4, 5, a.data_ptr(), 3, n_streams=3)
    r.dist_run(4, 4, a.data_ptr(), 3, n_streams=3)   # live items only: the culled constants stay
    check(a, w1, "same buffers, same layout")
    b = torch.full((3, 200, 320, 4), float("nan"), dtype=torch.float32, device="cuda:0")
    r.dist_run(4, 4, b.data_ptr(), 3, n_streams=3)   # new buffers: whole assemblies
    check(b, w1, "new buffers")
    r.set_camera(cam2)
    r.render(0, 4)
    r.dist_run(4, 5, a.data_ptr(), 3, n_streams=3)   # another culled set: whole assemblies again
    check(a, w2, "after a camera change")
    r.dist_finalize()


def test_bench_group_leg_members_on_one_device():
    """bench.py's pt_create_multi leg with two members
    on device 0: both exchanges timed and each last frame bitwise the
    one-GPU frame; the peer-store probe check is not armed on one device."""
    env = dict(os.environ)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--no-scene-legs",
           "--no-cpu-baseline", "--group-devices", "0,0"]
    res = _run(cmd, env)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-4000:]
    out = _record(res)
    g = out["group_leg"]
    assert g["devices"] == [0, 0]
    for k in ("exchange0", "exchange1"):
        assert g[k]["verified_bitwise_vs_single_gpu"] is True, g
        assert g[k]["ms_per_step"] > 0
    assert g["exchange0"]["exchange"].startswith("peer stores")
    assert g["exchange1"]["exchange"].startswith("staged")
