"""Multi-rank path on CPU (gloo, world_size 2 and 4), built from the
product's own partition and exchange tables.

Each rank takes its share from libptamd's host code -- pt_partition_items
(the item lists pt_render_packed launches and pt_items_pack writes, with the
kernels' item -> pixel map) and pt_primary_cull_rects -- renders exactly those
pixels with the CPU oracle (the GPU's stand-in here; the GPU runs of the same
exchange are tests/test_gpu_multi.py), packs its live items into the
pt_items_pack slot layout, and gloo-gathers the slots to rank 0.  Rank 0
assembles the frame as pt_items_unpack_all does: every rank's live items
scattered by its table, culled items written as (0,0,0,1).  The frame must
be the single-rank frame bit for bit.  A second test covers the reduce
alternative: each rank's -0/+0 cleared share (partition_owned), SUM-reduced.
This is the exchange bench.py runs over RCCL for N > 1."""
import os
import sys
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
import ptamd
import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

W, H, SPP, SPL = 72, 40, 2, 4
CAM = scenes.camera((3.0, 2.0, 4.0))   # the box off-centre: live and culled items on every rank


def _scene():
    v, i, _ = O.obj_parse(open(scenes.BOX_OBJ, "rb").read())
    ri, nodes = O.bvh_build(v, i)
    return v, ri, nodes


def _rects(nodes):
    n = nodes.reshape(-1, 8)
    return ptamd.primary_cull_rects(CAM, W, H, n[0, 0:3], n[0, 4:7], scenes.REFERENCE_LIGHT)


def _pack_share(rank, world, slots, slot_items):
    """This rank's live items rendered and packed as pt_items_pack lays them out."""
    v, ri, nodes = _scene()
    live, culled, pix = ptamd.partition_items(W, H, SPL, world, rank, slots, _rects(nodes))
    lp = pix[:len(live)].reshape(-1)
    frame, _ = O.render_pixels(v, ri, nodes, CAM, scenes.REFERENCE_LIGHT, W, H, lp, n_batches=SPP, nthreads=2)
    frame = frame.reshape(-1, 4)
    send = np.zeros((slot_items * (256 // SPL), 4), np.float32)
    ok = lp >= 0
    send[:lp.size][ok] = frame[lp[ok]]   # pixels past the frame edge stay zero, as on the device
    return send.reshape(-1)


def _assemble(slots_data, world, slots):
    """pt_items_unpack_all on the host: live items from each rank's slot,
    culled items (0,0,0,1)."""
    _, _, nodes = _scene()
    frame = np.full((W * H, 4), np.nan, np.float32)
    for r in range(world):
        live, culled, pix = ptamd.partition_items(W, H, SPL, world, r, slots, _rects(nodes))
        src = slots_data[r].reshape(-1, 4)
        lp = pix[:len(live)].reshape(-1)
        ok = lp >= 0
        frame[lp[ok]] = src[:lp.size][ok]
        cp = pix[len(live):].reshape(-1)
        frame[cp[cp >= 0]] = (0.0, 0.0, 0.0, 1.0)
    return frame.reshape(-1)


def _slot_items(world, slots):
    _, _, nodes = _scene()
    return max(len(ptamd.partition_items(W, H, SPL, world, r, slots, _rects(nodes))[0]) for r in range(world))


def _gather_worker(rank, world, port, slots, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.from_numpy(_pack_share(rank, world, slots, _slot_items(world, slots)))
    got = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, got, dst=0)
    if rank == 0:
        q.put(_assemble([g.numpy() for g in got], world, slots).tobytes())
    dist.barrier()
    dist.destroy_process_group()


def _reduce_worker(rank, world, port, slots, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    v, ri, nodes = _scene()
    owned = ptamd.partition_owned(W, H, world, rank, slots)
    acc = np.repeat(np.where(owned[..., None], np.float32(0.0), np.float32(-0.0)), 4, axis=2)
    acc = np.ascontiguousarray(acc, np.float32).reshape(-1)   # pt_clear_accum: +0 owned, -0 elsewhere
    O.render_pixels(v, ri, nodes, CAM, scenes.REFERENCE_LIGHT, W, H, np.flatnonzero(owned.reshape(-1)),
                    n_batches=SPP, accum=acc, nthreads=2)
    t = torch.from_numpy(acc)
    dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)
    if rank == 0:
        q.put(t.numpy().tobytes())
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    """A free port below the ephemeral range (32768+), so no client socket
    of an earlier run can be holding it (a port picked in that range can be
    taken before the store binds it: EADDRINUSE)."""
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


def _run(worker, world, slots):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, slots, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = np.frombuffer(q.get(timeout=240), np.float32)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return got


def _want():
    v, ri, nodes = _scene()
    want, _ = O.render(v, ri, nodes, CAM, scenes.REFERENCE_LIGHT, W, H, n_batches=SPP)
    return want


@pytest.mark.parametrize("world,slots", [(2, None), (4, None), (4, [2, 4, 4, 4])])
def test_sparse_gather_with_product_tables_is_bit_exact(world, slots):
    got = _run(_gather_worker, world, slots)
    want = _want()
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_culled_items_hold_exactly_the_fill_value():
    """The premise of the sparse exchange: every pixel of a culled item is
    (0,0,0,1) in a frame rendered from batch 0."""
    _, _, nodes = _scene()
    want = _want().reshape(-1, 4)
    n_culled = 0
    for r in range(3):
        live, culled, pix = ptamd.partition_items(W, H, SPL, 3, r, None, _rects(nodes))
        cp = pix[len(live):].reshape(-1)
        cp = cp[cp >= 0]
        n_culled += cp.size
        assert np.all(want[cp] == np.array([0, 0, 0, 1], np.float32))
    assert n_culled > 0


@pytest.mark.parametrize("world,slots", [(2, None), (4, [3, 2, 2, 1])])
def test_tile_split_reduce_is_bit_exact(world, slots):
    got = _run(_reduce_worker, world, slots)
    want = _want()
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_negative_zero_is_the_additive_identity():
    x = np.array([0.0, -0.0, 1.5, -2.0, np.inf, -np.inf, 1e-45], np.float32)
    s = (x + np.float32(-0.0)).astype(np.float32)
    assert np.array_equal(s.view(np.uint32), x.view(np.uint32))
    # +0 is not: -0 + +0 = +0
    assert (np.float32(-0.0) + np.float32(0.0)).view(np.uint32) == 0


def test_rccl_standin_exports_the_entry_points_pt_dist_resolves():
    """tests/dist_shim.cpp (loaded by libptamd through PT_RCCL_LIB in the
    two-process GPU test of pt_dist_run) defines every RCCL entry point
    rccl_api() resolves (pt_api.cpp), and libptamd names that variable."""
    import ctypes
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = os.path.join(root, "tests", "_build", "libptdistshim.so")
    subprocess.check_call(["make", "-s", "-C", os.path.join(root, "tests")])
    lib = ctypes.CDLL(so)
    for name in ("ncclGetUniqueId", "ncclCommInitRank", "ncclCommDestroy", "ncclCommAbort", "ncclGroupStart",
                 "ncclGroupEnd", "ncclSend", "ncclRecv", "ncclGetErrorString"):
        assert hasattr(lib, name), name
    api = open(os.path.join(root, "discovering-path-tracer_amd", "csrc", "pt_api.cpp")).read()
    assert 'getenv("PT_RCCL_LIB")' in api
    uid = ctypes.create_string_buffer(128)
    assert lib.ncclGetUniqueId(uid) == 0 and uid.value.startswith(b"/ptshim-")


def test_bench_spawns_ranks_without_a_launcher():
    """`python bench.py --gpus 2` with no WORLD_SIZE starts
    its two ranks itself (torch.distributed.run as a child process, never an
    exec) and reaches the two-rank path; --dry-run stops before any GPU call."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"], cwd=ROOT,
                         env=env, capture_output=True, text=True, timeout=180)
    assert res.returncode == 0, res.stderr[-3000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert {k: out[k] for k in ("dry_run", "n_gpus", "ranks_seen", "launcher", "backend_requested")} == \
        {"dry_run": True, "n_gpus": 2, "ranks_seen": [0, 1], "launcher": "spawned", "backend_requested": "nccl"}


def test_bench_stuck_rank_fails_fast():
    """a rank that never reaches a collective (the shape
    of the round-4 two-rank hang, killed after 180 s with nothing said) must
    end the run with an error within the process-group timeout
    (PT_BENCH_PG_TIMEOUT_S), naming where each rank was; it must not hold the
    other ranks for gloo's / RCCL's default 30 minutes."""
    import subprocess
    import time as _t
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PT_BENCH_DRY_STALL_RANK="1", PT_BENCH_PG_TIMEOUT_S="5")
    t0 = _t.perf_counter()
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"], cwd=ROOT,
                         env=env, capture_output=True, text=True, timeout=120)
    dt = _t.perf_counter() - t0
    assert res.returncode != 0, res.stdout[-2000:]
    assert dt < 90, dt
    assert "imed out" in res.stderr or "Timeout" in res.stderr or "timeout" in res.stderr, res.stderr[-3000:]
