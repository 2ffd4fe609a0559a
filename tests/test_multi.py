"""Multi-rank path on CPU (gloo, world_size 2 and 4): each rank renders its
screen tiles (pt_set_partition's block-interleaved ownership) with -0 in the
pixels it does not own, exactly as the device clear kernel leaves them; a SUM
reduction over ranks must reproduce the single-rank frame bit for bit.  This
is the collective bench.py runs over RCCL for N > 1."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
import ptamd
import scenes

W, H, SPP = 72, 40, 2


def _scene():
    v, i, _ = O.obj_parse(open(scenes.BOX_OBJ, "rb").read())
    ri, nodes = O.bvh_build(v, i)
    return v, ri, nodes


def _rank_frame(rank, world):
    v, ri, nodes = _scene()
    owned = ptamd.partition_owned(W, H, world, rank)
    acc = np.repeat(np.where(owned[..., None], np.float32(0.0), np.float32(-0.0)), 4, axis=2)
    acc = np.ascontiguousarray(acc, np.float32).reshape(-1)
    O.render(v, ri, nodes, scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, W, H, n_batches=SPP,
             tile=16, nranks=world, rank=rank, accum=acc, nthreads=2)
    return acc


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.from_numpy(_rank_frame(rank, world))
    dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)
    if rank == 0:
        q.put(t.numpy().tobytes())
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 4])
def test_tile_split_reduce_is_bit_exact(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = np.frombuffer(q.get(timeout=240), np.float32)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    v, ri, nodes = _scene()
    want, _ = O.render(v, ri, nodes, scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, W, H, n_batches=SPP)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_negative_zero_is_the_additive_identity():
    x = np.array([0.0, -0.0, 1.5, -2.0, np.inf, -np.inf, 1e-45], np.float32)
    s = (x + np.float32(-0.0)).astype(np.float32)
    assert np.array_equal(s.view(np.uint32), x.view(np.uint32))
    # +0 is not: -0 + +0 = +0
    assert (np.float32(-0.0) + np.float32(0.0)).view(np.uint32) == 0
