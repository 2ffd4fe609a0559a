"""ctypes binding to oracle/liboracle.so — the CPU parity checker.

Test infrastructure only: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py; never by the product package.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_LIB = None

F32P = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
U32P = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
U64P = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = ctypes.CDLL(path)
        sz = ctypes.c_size_t
        L.oracle_obj_parse.argtypes = [ctypes.c_char_p, sz, ctypes.c_void_p, ctypes.POINTER(sz),
                                       ctypes.c_void_p, ctypes.POINTER(sz), ctypes.c_void_p, ctypes.POINTER(sz)]
        L.oracle_bvh_build.argtypes = [F32P, U32P, sz, U32P, F32P]
        L.oracle_render.argtypes = [F32P, U32P, F32P, sz, F32P, F32P, sz,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    F32P, U64P, ctypes.c_int]
        L.oracle_render_ex.argtypes = L.oracle_render.argtypes + [ctypes.c_uint32]
        L.oracle_render_pixels.argtypes = [F32P, U32P, F32P, sz, F32P, F32P, sz, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                           np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS"), sz,
                                           F32P, U64P, ctypes.c_int, ctypes.c_uint32]
        L.oracle_math.argtypes = [ctypes.c_int, F32P, F32P, sz]
        L.oracle_rng.argtypes = [ctypes.c_uint32, F32P, sz]
        L.oracle_trace.argtypes = [F32P, U32P, F32P, sz, F32P, F32P, F32P, U64P]
        _LIB = L
    return _LIB


def obj_parse(text: bytes):
    L = lib()
    sz = ctypes.c_size_t
    nv, ni, nt = sz(), sz(), sz()
    rc = L.oracle_obj_parse(text, len(text), None, ctypes.byref(nv), None, ctypes.byref(ni), None, ctypes.byref(nt))
    if rc:
        raise ValueError(f"oracle_obj_parse rc={rc}")
    v = np.zeros(nv.value, np.float32)
    i = np.zeros(ni.value, np.uint32)
    t = np.zeros(max(nt.value, 1), np.float32)
    L.oracle_obj_parse(text, len(text), v.ctypes.data, ctypes.byref(nv), i.ctypes.data, ctypes.byref(ni),
                       t.ctypes.data, ctypes.byref(nt))
    return v, i, t[: nt.value]


def bvh_build(verts, idx):
    verts = np.ascontiguousarray(verts, np.float32)
    idx = np.ascontiguousarray(idx, np.uint32)
    T = idx.size // 3
    out_idx = np.zeros_like(idx)
    nodes = np.zeros((2 * T - 1) * 8, np.float32)
    rc = lib().oracle_bvh_build(verts, idx, idx.size, out_idx, nodes)
    if rc:
        raise ValueError(f"oracle_bvh_build rc={rc}")
    return out_idx, nodes


def render(verts, idx, nodes, camera16, lights16, W, H, first_batch=0, n_batches=1,
           max_depth=4, sss_bounces=3, row_stride=1, row_phase=0, tile=16, nranks=1, rank=0,
           accum=None, nthreads=0, int_bits=False):
    """Sequential 1-spp batches of raytrace_comp.comp over the selected pixels.
    int_bits: the nodes' link fields are int32 bit patterns (PT_NODES_INT_BITS,
    the >= 2^24-node layout) instead of float-encoded indices."""
    if accum is None:
        accum = np.zeros(W * H * 4, np.float32)
    stats = np.zeros(3, np.uint64)
    lights16 = np.ascontiguousarray(lights16, np.float32).reshape(-1)
    nodes = np.ascontiguousarray(nodes, np.float32).reshape(-1)
    rc = lib().oracle_render_ex(np.ascontiguousarray(verts, np.float32), np.ascontiguousarray(idx, np.uint32),
                                nodes, nodes.size // 8,
                                np.ascontiguousarray(camera16, np.float32), lights16, lights16.size // 16,
                                W, H, first_batch, n_batches, max_depth, sss_bounces,
                                row_stride, row_phase, tile, nranks, rank, accum, stats, nthreads,
                                1 if int_bits else 0)
    if rc:
        raise ValueError(f"oracle_render rc={rc}")
    return accum, stats


def render_pixels(verts, idx, nodes, camera16, lights16, W, H, pixels, first_batch=0, n_batches=1, max_depth=4,
                  sss_bounces=3, accum=None, nthreads=0, int_bits=False):
    """Like render(), for the listed pixels (y*W+x, negatives skipped) only."""
    if accum is None:
        accum = np.zeros(W * H * 4, np.float32)
    stats = np.zeros(3, np.uint64)
    lights16 = np.ascontiguousarray(lights16, np.float32).reshape(-1)
    nodes = np.ascontiguousarray(nodes, np.float32).reshape(-1)
    pixels = np.ascontiguousarray(pixels, np.int32).reshape(-1)
    rc = lib().oracle_render_pixels(np.ascontiguousarray(verts, np.float32), np.ascontiguousarray(idx, np.uint32),
                                    nodes, nodes.size // 8, np.ascontiguousarray(camera16, np.float32), lights16,
                                    lights16.size // 16, W, H, first_batch, n_batches, max_depth, sss_bounces,
                                    pixels, pixels.size, accum, stats, nthreads, 1 if int_bits else 0)
    if rc:
        raise ValueError(f"oracle_render_pixels rc={rc}")
    return accum, stats


def math(fn, x):
    x = np.ascontiguousarray(x, np.float32)
    y = np.empty_like(x)
    lib().oracle_math(fn, x, y, x.size)
    return y


def rng(seed, n):
    out = np.empty(n, np.float32)
    lib().oracle_rng(seed, out, n)
    return out


def trace(verts, idx, nodes, origin, direction):
    """One reference traceRay: (hit, t, position, normal, [rays, nodes, leaves])."""
    out = np.zeros(8, np.float32)
    ctr = np.zeros(3, np.uint64)
    nodes = np.ascontiguousarray(nodes, np.float32).reshape(-1)
    lib().oracle_trace(np.ascontiguousarray(verts, np.float32), np.ascontiguousarray(idx, np.uint32), nodes,
                       nodes.size // 8, np.asarray(origin, np.float32), np.asarray(direction, np.float32), out, ctr)
    return bool(out[0]), float(out[1]), out[2:5].copy(), out[5:8].copy(), ctr
