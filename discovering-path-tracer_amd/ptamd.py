"""ptamd — Python binding of the MI355X path tracer's C ABI (include/pathtracer.h).

A thin ctypes layer over libptamd.so, mirroring the reference's host-side
objects: Scene (OBJ ingest + BVH, src/BoundingVolumeHierarchy.h), pack_light
(src/Light.cpp), default_camera (src/Camera.cpp) and Renderer — the
replacement for VulkanRayTracer's upload/dispatch/readback
(src/Vulkan/VulkanRayTracer.cpp).  There is no fallback: if the library is
missing or the GPU is absent, calls raise.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PTAMD_LIB") or os.path.join(HERE, "libptamd.so")   # override: A/B of builds

PT_OK = 0
PT_NODES_INT_BITS = 0x1
PT_OPT_SCENE_IN_LDS = 1
PT_OPT_SAMPLE_LANES = 2
PT_OPT_FRESH_BATCH0 = 3
PT_OPT_KERNEL = 4
PT_OPT_SM_BATCH = 5
PT_OPT_PRIMARY_CULL = 6
PT_OPT_WF_PATHS = 7
PT_OPT_ITEM_ORDER = 8
PT_OPT_LAUNCH_TIMING = 9
PT_OPT_COUNT_TRACED = 10
PT_OPT_PAIRS = 11
PT_OPT_WIDE = 12
PT_OPT_WF_STREAMS = 13
PT_OPT_WIDE_BUILD = 14
PT_OPT_WF_FUSE = 15
PT_OPT_WIDE_NODE = 16
PT_OPT_WF_TAIL = 17
PT_OPT_GROUP_EXCHANGE = 18
PT_OPT_GROUP_CHECK = 19
PT_OPT_WF_GRID = 20
PT_OPT_WF_REFILL = 21
PT_OPT_MIXED_LANES = 22
KERNEL_AUTO, KERNEL_RECURSIVE, KERNEL_WAVEFRONT = 0, 1, 3   # 2 (lane state machine) was removed

# Every symbol include/pathtracer.h declares (tests check the .so exports them).
EXPORTS = [
    "pt_abi_version", "pt_last_error", "pt_create", "pt_destroy", "pt_set_stream", "pt_synchronize",
    "pt_upload_scene", "pt_upload_lights", "pt_set_camera", "pt_set_params", "pt_resize_and_clear",
    "pt_bind_accum", "pt_clear_accum", "pt_accum_device_ptr", "pt_read_accum", "pt_dispatch", "pt_render",
    "pt_set_partition", "pt_tiles_owned", "pt_tiles_pack", "pt_tiles_unpack", "pt_set_option", "pt_last_kernel", "pt_set_stats_mode", "pt_get_stats", "pt_reset_stats", "pt_last_launch_ms",
    "pt_launch_times_ms", "pt_reset_launch_times", "pt_selftest_math", "pt_selftest_exhaustive",
    "pt_scene_load_obj", "pt_scene_parse_obj", "pt_scene_from_arrays", "pt_scene_build_bvh",
    "pt_scene_counts", "pt_scene_copy", "pt_scene_upload", "pt_scene_free", "pt_pack_light",
    "pt_default_camera", "pt_primary_cull_rects", "pt_scene_save", "pt_scene_load_cache",
    "pt_progressive_camera", "pt_progressive_advance", "pt_readback_begin", "pt_readback_end", "pt_write_image",
    "pt_items_live", "pt_items_pack", "pt_items_unpack_all", "pt_render_packed", "pt_launch_span_ms",
    "pt_set_partition_slots", "pt_get_traced", "pt_wide_info", "pt_partition_items",
    "pt_dist_unique_id", "pt_dist_init", "pt_dist_run", "pt_dist_slot_floats", "pt_dist_finalize",
    "pt_dist_set_streams", "pt_dist_wait", "pt_dist_abort", "pt_create_multi", "pt_group_info",
    "pt_group_check", "pt_dist_info", "pt_mixed_info",
]


class PTError(RuntimeError):
    pass


class Params(ctypes.Structure):
    _fields_ = [("max_depth", ctypes.c_int), ("sss_bounces", ctypes.c_int)]


class Stats(ctypes.Structure):
    _fields_ = [("rays", ctypes.c_uint64), ("nodes", ctypes.c_uint64), ("leaf_tests", ctypes.c_uint64),
                ("samples", ctypes.c_uint64)]


class Traced(ctypes.Structure):
    _fields_ = [("closest_walks", ctypes.c_uint64), ("shadow_walks", ctypes.c_uint64), ("nodes", ctypes.c_uint64),
                ("tri_tests", ctypes.c_uint64), ("primaries", ctypes.c_uint64)]


_lib = None


def lib():
    """Load libptamd.so (build it with `make -C discovering-path-tracer_amd`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PTError(f"{LIB_PATH} not built; run __graft_entry__.build() or make -C {HERE}")
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int
        psz = ctypes.POINTER(sz)
        sig = {
            "pt_abi_version": ([], i32), "pt_last_error": ([], ctypes.c_char_p),
            "pt_create": ([i32, ctypes.POINTER(vp)], i32), "pt_destroy": ([vp], i32),
            "pt_create_multi": ([vp, i32, ctypes.POINTER(vp)], i32),
            "pt_group_info": ([vp, ctypes.POINTER(i32), vp, i32, ctypes.POINTER(i32)], i32),
            "pt_group_check": ([vp, ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_float),
                                ctypes.POINTER(ctypes.c_float)], i32),
            "pt_dist_info": ([vp, ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(i32)], i32),
            "pt_set_stream": ([vp, vp], i32), "pt_synchronize": ([vp], i32),
            "pt_upload_scene": ([vp, vp, sz, vp, sz, vp, sz, vp, sz, vp, sz, u32], i32),
            "pt_upload_lights": ([vp, vp, sz], i32), "pt_set_camera": ([vp, vp], i32),
            "pt_set_params": ([vp, ctypes.POINTER(Params)], i32),
            "pt_resize_and_clear": ([vp, i32, i32], i32), "pt_bind_accum": ([vp, vp, i32, i32], i32),
            "pt_clear_accum": ([vp], i32), "pt_accum_device_ptr": ([vp], vp),
            "pt_read_accum": ([vp, vp, sz], i32), "pt_dispatch": ([vp, u32], i32),
            "pt_render": ([vp, u32, u32], i32), "pt_set_partition": ([vp, i32, i32], i32),
            "pt_set_partition_slots": ([vp, i32, i32, vp], i32),
            "pt_set_stats_mode": ([vp, i32], i32), "pt_set_option": ([vp, i32, i32], i32), "pt_last_kernel": ([vp, ctypes.POINTER(ctypes.c_int)], i32),
            "pt_tiles_owned": ([vp, ctypes.POINTER(i32)], i32), "pt_tiles_pack": ([vp, vp], i32),
            "pt_tiles_unpack": ([vp, vp, i32, vp], i32), "pt_get_stats": ([vp, ctypes.POINTER(Stats)], i32),
            "pt_reset_stats": ([vp], i32), "pt_get_traced": ([vp, ctypes.POINTER(Traced)], i32),
            "pt_wide_info": ([vp, ctypes.POINTER(ctypes.c_int)], i32),
            "pt_mixed_info": ([vp, ctypes.POINTER(ctypes.c_int)], i32),
            "pt_partition_items": ([i32, i32, i32, i32, i32, vp, vp, i32, i32, vp, psz, vp, psz, vp], i32),
            "pt_dist_unique_id": ([vp, sz], i32), "pt_dist_init": ([vp, vp, i32, i32], i32),
            "pt_dist_run": ([vp, u32, i32, i32, vp, i32], i32), "pt_dist_slot_floats": ([vp, psz], i32),
            "pt_dist_finalize": ([vp], i32), "pt_dist_set_streams": ([vp, vp, vp, vp], i32),
            "pt_dist_wait": ([vp, i32], i32), "pt_dist_abort": ([vp], i32), "pt_last_launch_ms": ([vp, ctypes.POINTER(ctypes.c_float)], i32),
            "pt_launch_times_ms": ([vp, vp, sz, psz], i32), "pt_reset_launch_times": ([vp], i32),
            "pt_launch_span_ms": ([vp, ctypes.POINTER(ctypes.c_float), psz], i32),
            "pt_selftest_math": ([i32, i32, vp, vp, sz], i32),
            "pt_selftest_exhaustive": ([i32, i32, ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(u32)], i32),
            "pt_scene_load_obj": ([ctypes.c_char_p, ctypes.POINTER(vp)], i32),
            "pt_scene_parse_obj": ([ctypes.c_char_p, sz, ctypes.POINTER(vp)], i32),
            "pt_scene_from_arrays": ([vp, sz, vp, sz, ctypes.POINTER(vp)], i32),
            "pt_scene_build_bvh": ([vp, u32, i32], i32),
            "pt_scene_counts": ([vp, psz, psz, psz, psz, psz], i32),
            "pt_scene_copy": ([vp, vp, vp, vp, vp, vp], i32), "pt_scene_upload": ([vp, vp], i32),
            "pt_scene_free": ([vp], i32), "pt_pack_light": ([vp, vp, vp, vp, vp], i32),
            "pt_default_camera": ([vp], i32),
            "pt_primary_cull_rects": ([vp, i32, i32, vp, vp, vp, i32, vp, i32, ctypes.POINTER(i32)], i32),
            "pt_scene_save": ([vp, ctypes.c_char_p], i32),
            "pt_progressive_camera": ([vp, vp, ctypes.POINTER(i32)], i32),
            "pt_progressive_advance": ([vp, u32, u32, ctypes.POINTER(u32), ctypes.POINTER(u32)], i32),
            "pt_readback_begin": ([vp, ctypes.POINTER(i32)], i32),
            "pt_readback_end": ([vp, i32, vp, sz], i32),
            "pt_write_image": ([ctypes.c_char_p, vp, i32, i32, i32], i32),
            "pt_items_live": ([vp, i32, ctypes.POINTER(i32), ctypes.POINTER(i32)], i32),
            "pt_items_pack": ([vp, vp], i32),
            "pt_items_unpack_all": ([vp, vp, sz, vp], i32),
            "pt_render_packed": ([vp, u32, vp, vp, sz, vp], i32),
            "pt_scene_load_cache": ([ctypes.c_char_p, ctypes.POINTER(vp)], i32),
        }
        for name, (args, res) in sig.items():
            if not hasattr(L, name):   # older library (A/B timing); calls to it fail loudly
                continue
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


def _check(rc, what):
    if rc != PT_OK:
        raise PTError(f"{what} failed ({rc}): {lib().pt_last_error().decode()}")


def _ptr(a):
    return a.ctypes.data if a is not None and a.size else None


class Scene:
    """OBJ (or raw arrays) + BVH, built by the native host layer."""

    def __init__(self, handle):
        self._h = ctypes.c_void_p(handle) if not isinstance(handle, ctypes.c_void_p) else handle

    @classmethod
    def load_obj(cls, path):
        h = ctypes.c_void_p()
        _check(lib().pt_scene_load_obj(path.encode(), ctypes.byref(h)), "pt_scene_load_obj")
        return cls(h)

    @classmethod
    def parse_obj(cls, text: bytes):
        h = ctypes.c_void_p()
        _check(lib().pt_scene_parse_obj(text, len(text), ctypes.byref(h)), "pt_scene_parse_obj")
        return cls(h)

    @classmethod
    def from_arrays(cls, vertices, indices):
        v = np.ascontiguousarray(vertices, np.float32).reshape(-1)
        i = np.ascontiguousarray(indices, np.uint32).reshape(-1)
        h = ctypes.c_void_p()
        _check(lib().pt_scene_from_arrays(_ptr(v), v.size, _ptr(i), i.size, ctypes.byref(h)), "pt_scene_from_arrays")
        return cls(h)

    @classmethod
    def load_cache(cls, path):
        """pt_scene_load_cache: a scene written by save() (BVH included)."""
        h = ctypes.c_void_p()
        _check(lib().pt_scene_load_cache(str(path).encode(), ctypes.byref(h)), "pt_scene_load_cache")
        return cls(h)

    def save(self, path):
        _check(lib().pt_scene_save(self._h, str(path).encode()), "pt_scene_save")
        return self

    def build_bvh(self, int_bits=False, threads=0):
        self.int_bits = int_bits
        _check(lib().pt_scene_build_bvh(self._h, PT_NODES_INT_BITS if int_bits else 0, threads), "pt_scene_build_bvh")
        return self

    def counts(self):
        c = [ctypes.c_size_t() for _ in range(5)]
        _check(lib().pt_scene_counts(self._h, *[ctypes.byref(x) for x in c]), "pt_scene_counts")
        return tuple(x.value for x in c)

    def arrays(self):
        """(vertices, indices [BVH order once built], nodes (N,8) float32, uvs, mat_indices)."""
        nvf, ni, nn, nuv, nmat = self.counts()
        v = np.zeros(nvf, np.float32)
        i = np.zeros(ni, np.uint32)
        n = np.zeros((nn, 8), np.float32)
        uv = np.zeros(nuv, np.float32)
        m = np.zeros(nmat, np.uint32)
        _check(lib().pt_scene_copy(self._h, _ptr(v), _ptr(i), _ptr(n), _ptr(uv), _ptr(m)), "pt_scene_copy")
        return v, i, n, uv, m

    def close(self):
        if self._h:
            lib().pt_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pack_light(position, normal, intensity, size):
    """Light::packData (src/Light.cpp:16-33) -> 16 float32."""
    out = np.zeros(16, np.float32)
    args = [np.ascontiguousarray(a, np.float32) for a in (position, normal, intensity, size)]
    _check(lib().pt_pack_light(*[a.ctypes.data for a in args], out.ctypes.data), "pt_pack_light")
    return out


def reference_light():
    """The scene light of VulkanRayTracer.cpp:149-162."""
    return pack_light([0, 2, 0], [0, -1, 0], [10, 10, 10], [2.5, 2.5])


def device_math(fn, x, device=0):
    """Evaluate the kernel's math function `fn` on the GPU (pt_selftest_math)."""
    x = np.ascontiguousarray(x, np.float32)
    y = np.empty_like(x)
    _check(lib().pt_selftest_math(device, fn, x.ctypes.data, y.ctypes.data, x.size), "pt_selftest_math")
    return y


def device_math_exhaustive(fn, device=0):
    """pt_selftest_exhaustive: (mismatching inputs, smallest such bit pattern)
    of the device's fast-quotient fn (0 rcp, 1 log, 2 exp, 3 acos)
    against its IEEE definition over all 2^32 inputs."""
    bad = ctypes.c_ulonglong(0)
    first = ctypes.c_uint32(0)
    _check(lib().pt_selftest_exhaustive(device, fn, ctypes.byref(bad), ctypes.byref(first)),
           "pt_selftest_exhaustive")
    return bad.value, first.value


def partition_slot_positions(nranks, rank, slots=None):
    """(m, positions) of rank's slots in a period of the slotted partition
    (pt_api.cpp part_of): slots ordered by (k + 1/2) / slots[r] for each
    rank's k-th slot, ties by rank."""
    s = [1] * nranks if slots is None else [int(x) for x in slots]
    seq = sorted(((k + 0.5) / s[r], r) for r in range(nranks) for k in range(s[r]))
    return len(seq), [v for v, (_, r) in enumerate(seq) if r == rank]


def partition_owned(width, height, nranks, rank, slots=None):
    """Pixels a rank renders under pt_set_partition(_slots): 16x16 blocks,
    block (bx, by) is tile b = by*blocks_x + (bx - by) mod blocks_x (rows
    rotated); the rank owns tile b iff b % m is one of its slot positions
    (partition_slot_positions; one slot per rank: b % nranks == rank).
    Returns a (H, W) bool mask."""
    m, pos = partition_slot_positions(nranks, rank, slots)
    nbx = (width + 15) // 16
    ys, xs = np.mgrid[0:height, 0:width]
    by, bx = ys // 16, xs // 16
    return np.isin((by * nbx + (bx - by) % nbx) % m, pos)


def partition_items(width, height, sample_lanes, nranks, rank, slots=None, cull_rects=None, item_order=1):
    """pt_partition_items: the product's item tables for `rank` (host only).
    Returns (live, culled, pixel_of) -- live and culled item ids in launch /
    table order, and pixel_of[(len(live) + len(culled)), 256 // sample_lanes]
    with the pixel index y*W+x of each item slot (-1 past the frame edge)."""
    sl = None if slots is None else np.ascontiguousarray(slots, np.int32)
    if cull_rects is None:
        cr, nc = None, -1
    else:
        cr = np.ascontiguousarray(cull_rects, np.float32).reshape(-1, 4)
        nc = cr.shape[0]
    nl, nu = ctypes.c_size_t(0), ctypes.c_size_t(0)
    args = (width, height, sample_lanes, nranks, rank, None if sl is None else sl.ctypes.data,
            None if cr is None else cr.ctypes.data, nc, item_order)
    _check(lib().pt_partition_items(*args, None, ctypes.byref(nl), None, ctypes.byref(nu), None), "pt_partition_items")
    live = np.zeros(max(nl.value, 1), np.int32)
    culled = np.zeros(max(nu.value, 1), np.int32)
    per = 256 // sample_lanes
    pix = np.zeros(max((nl.value + nu.value) * per, 1), np.int32)
    _check(lib().pt_partition_items(*args, live.ctypes.data, ctypes.byref(nl), culled.ctypes.data, ctypes.byref(nu),
                                    pix.ctypes.data), "pt_partition_items")
    return live[:nl.value], culled[:nu.value], pix[:(nl.value + nu.value) * per].reshape(-1, per)


def primary_cull_rects(camera_ubo, width, height, root_min, root_max, lights16, max_rects=8):
    """pt_primary_cull_rects: NDC rectangles {x0,x1,y0,y1} outside which no
    primary ray reaches the root box or a light; None when not derivable."""
    cam = np.ascontiguousarray(camera_ubo, np.float32).reshape(16)
    lo = np.ascontiguousarray(root_min, np.float32).reshape(3)
    hi = np.ascontiguousarray(root_max, np.float32).reshape(3)
    l = np.ascontiguousarray(lights16, np.float32).reshape(-1)
    out = np.zeros((max_rects, 4), np.float32)
    n = ctypes.c_int(0)
    _check(lib().pt_primary_cull_rects(cam.ctypes.data, width, height, lo.ctypes.data, hi.ctypes.data,
                                       l.ctypes.data if l.size else None, l.size // 16, out.ctypes.data,
                                       max_rects, ctypes.byref(n)), "pt_primary_cull_rects")
    return None if n.value < 0 else out[:n.value].copy()


def write_image(path, rgba, width, height, fmt="png"):
    """pt_write_image: PFM (float) or 8-bit sRGB PNG of an accumulation image."""
    a = np.ascontiguousarray(rgba, np.float32).reshape(-1)
    if a.size != width * height * 4:
        raise PTError("rgba must hold width*height*4 floats")
    _check(lib().pt_write_image(str(path).encode(), a.ctypes.data, width, height, 1 if fmt == "png" else 0),
           "pt_write_image")


def default_camera():
    ubo = np.zeros(16, np.float32)
    _check(lib().pt_default_camera(ubo.ctypes.data), "pt_default_camera")
    return ubo


class Renderer:
    """One GPU's path tracer: upload, dispatch/render, read back."""

    def __init__(self, device=0, devices=None):
        """One GPU (pt_create), or with `devices` (a list of ordinals) one
        context over all of them (pt_create_multi: tile split, the frame on
        devices[0])."""
        self._c = ctypes.c_void_p()
        if devices is None:
            _check(lib().pt_create(device, ctypes.byref(self._c)), "pt_create")
        else:
            d = np.ascontiguousarray(devices, np.int32)
            _check(lib().pt_create_multi(d.ctypes.data, d.size, ctypes.byref(self._c)), "pt_create_multi")
        self.width = self.height = 0

    def group_info(self):
        """(device ordinals, members store straight into the frame)."""
        n, peer = ctypes.c_int(0), ctypes.c_int(0)
        devs = np.zeros(64, np.int32)
        _check(lib().pt_group_info(self._c, ctypes.byref(n), devs.ctypes.data, devs.size, ctypes.byref(peer)),
               "pt_group_info")
        return [int(x) for x in devs[:n.value]], bool(peer.value)

    def group_check(self):
        """The peer-store check (PT_OPT_GROUP_CHECK): (state, ms_peer,
        ms_staged); state -2 armed, -1 not run, 0 matched, 1 mismatch (staged
        copies in force)."""
        st, a, b = ctypes.c_int(0), ctypes.c_float(0), ctypes.c_float(0)
        _check(lib().pt_group_check(self._c, ctypes.byref(st), ctypes.byref(a), ctypes.byref(b)), "pt_group_check")
        return st.value, a.value, b.value

    def upload_scene(self, vertices, indices, nodes, uvs=None, mat=None, int_bits=False):
        v = np.ascontiguousarray(vertices, np.float32).reshape(-1)
        i = np.ascontiguousarray(indices, np.uint32).reshape(-1)
        n = np.ascontiguousarray(nodes, np.float32).reshape(-1)
        uv = None if uvs is None else np.ascontiguousarray(uvs, np.float32).reshape(-1)
        m = None if mat is None else np.ascontiguousarray(mat, np.uint32).reshape(-1)
        _check(lib().pt_upload_scene(self._c, _ptr(v), v.size, _ptr(i), i.size, _ptr(n), n.size // 8,
                                     _ptr(uv), 0 if uv is None else uv.size, _ptr(m), 0 if m is None else m.size,
                                     PT_NODES_INT_BITS if int_bits else 0), "pt_upload_scene")

    def upload(self, scene: Scene):
        _check(lib().pt_scene_upload(self._c, scene._h), "pt_scene_upload")

    def upload_lights(self, lights16):
        l = np.ascontiguousarray(lights16, np.float32).reshape(-1)
        _check(lib().pt_upload_lights(self._c, _ptr(l), l.size // 16), "pt_upload_lights")

    def set_camera(self, ubo16):
        u = np.ascontiguousarray(ubo16, np.float32).reshape(16)
        _check(lib().pt_set_camera(self._c, u.ctypes.data), "pt_set_camera")

    def set_params(self, max_depth=4, sss_bounces=3):
        p = Params(max_depth, sss_bounces)
        _check(lib().pt_set_params(self._c, ctypes.byref(p)), "pt_set_params")

    def set_partition(self, nranks, rank, slots=None):
        """Tile split over nranks (pt_set_partition); `slots` (one int per
        rank) gives unequal shares (pt_set_partition_slots)."""
        if slots is None:
            _check(lib().pt_set_partition(self._c, nranks, rank), "pt_set_partition")
            return
        sl = np.ascontiguousarray(slots, np.int32)
        if sl.size != nranks:
            raise PTError("one slot count per rank")
        _check(lib().pt_set_partition_slots(self._c, nranks, rank, sl.ctypes.data), "pt_set_partition_slots")

    def tiles_owned(self):
        n = ctypes.c_int()
        _check(lib().pt_tiles_owned(self._c, ctypes.byref(n)), "pt_tiles_owned")
        return n.value

    def tiles_pack(self, dst_device_ptr):
        _check(lib().pt_tiles_pack(self._c, dst_device_ptr), "pt_tiles_pack")

    def tiles_unpack(self, src_device_ptr, src_rank, frame_device_ptr):
        _check(lib().pt_tiles_unpack(self._c, src_device_ptr, src_rank, frame_device_ptr), "pt_tiles_unpack")

    def progressive_camera(self, ubo16):
        """Camera for the progressive loop; True if it reset the sample counter."""
        u = np.ascontiguousarray(ubo16, np.float32).reshape(16)
        reset = ctypes.c_int(0)
        _check(lib().pt_progressive_camera(self._c, u.ctypes.data, ctypes.byref(reset)), "pt_progressive_camera")
        return bool(reset.value)

    def progressive_advance(self, max_new, limit=1024):
        first, count = ctypes.c_uint32(0), ctypes.c_uint32(0)
        _check(lib().pt_progressive_advance(self._c, max_new, limit, ctypes.byref(first), ctypes.byref(count)),
               "pt_progressive_advance")
        return first.value, count.value

    def readback_begin(self):
        t = ctypes.c_int(0)
        _check(lib().pt_readback_begin(self._c, ctypes.byref(t)), "pt_readback_begin")
        return t.value

    def readback_end(self, ticket):
        out = np.empty(self.width * self.height * 4, np.float32)
        _check(lib().pt_readback_end(self._c, ticket, out.ctypes.data, out.size), "pt_readback_end")
        return out

    def items_live(self, rank):
        """(live items of `rank` in the last rendered frame, pixels per item)."""
        n, per = ctypes.c_int(0), ctypes.c_int(0)
        _check(lib().pt_items_live(self._c, rank, ctypes.byref(n), ctypes.byref(per)), "pt_items_live")
        return n.value, per.value

    def items_pack(self, dst_ptr):
        _check(lib().pt_items_pack(self._c, dst_ptr), "pt_items_pack")

    def render_packed(self, n_batches, dst_ptr, gathered_ptr=None, slot_floats=0, frame_ptr=None):
        """Fresh frame's live items into dst; optionally assemble the previous
        frame's gathered slots into frame in the same launch."""
        _check(lib().pt_render_packed(self._c, n_batches, dst_ptr, gathered_ptr, slot_floats, frame_ptr),
               "pt_render_packed")

    def items_unpack_all(self, src_ptr, slot_floats, frame_ptr):
        _check(lib().pt_items_unpack_all(self._c, src_ptr, slot_floats, frame_ptr), "pt_items_unpack_all")

    def set_option(self, key, value):
        _check(lib().pt_set_option(self._c, key, value), "pt_set_option")

    def last_kernel(self):
        """Kernel of the last render: KERNEL_RECURSIVE or KERNEL_WAVEFRONT."""
        k = ctypes.c_int(0)
        _check(lib().pt_last_kernel(self._c, ctypes.byref(k)), "pt_last_kernel")
        return k.value

    def set_stream(self, stream_handle):
        _check(lib().pt_set_stream(self._c, stream_handle), "pt_set_stream")

    def resize_and_clear(self, w, h):
        _check(lib().pt_resize_and_clear(self._c, w, h), "pt_resize_and_clear")
        self.width, self.height = w, h

    def bind_accum(self, device_ptr, w, h):
        _check(lib().pt_bind_accum(self._c, device_ptr, w, h), "pt_bind_accum")
        self.width, self.height = w, h

    def clear(self):
        _check(lib().pt_clear_accum(self._c), "pt_clear_accum")

    def accum_ptr(self):
        return lib().pt_accum_device_ptr(self._c)

    def dispatch(self, sample_batch):
        _check(lib().pt_dispatch(self._c, sample_batch), "pt_dispatch")

    def render(self, first_batch, n_batches):
        _check(lib().pt_render(self._c, first_batch, n_batches), "pt_render")

    def synchronize(self):
        _check(lib().pt_synchronize(self._c), "pt_synchronize")

    def read_accum(self):
        out = np.empty(self.width * self.height * 4, np.float32)
        _check(lib().pt_read_accum(self._c, out.ctypes.data, out.size), "pt_read_accum")
        return out

    def set_stats_mode(self, on):
        _check(lib().pt_set_stats_mode(self._c, 1 if on else 0), "pt_set_stats_mode")

    def reset_stats(self):
        _check(lib().pt_reset_stats(self._c), "pt_reset_stats")

    def stats(self):
        s = Stats()
        _check(lib().pt_get_stats(self._c, ctypes.byref(s)), "pt_get_stats")
        return {"rays": s.rays, "nodes": s.nodes, "leaf_tests": s.leaf_tests, "samples": s.samples}

    # ---- native multi-GPU step loop (pt_dist_*) ----
    @staticmethod
    def dist_unique_id():
        """128-byte RCCL communicator id (rank 0 makes it, every rank gets a copy)."""
        buf = (ctypes.c_char * 128)()
        _check(lib().pt_dist_unique_id(buf, 128), "pt_dist_unique_id")
        return bytes(buf)

    def dist_init(self, uid, nranks, rank):
        b = (ctypes.c_char * 128).from_buffer_copy(uid)
        _check(lib().pt_dist_init(self._c, b, nranks, rank), "pt_dist_init")

    def dist_info(self):
        """(ranks the RCCL communicator reports via ncclCommCount, or -1;
        nranks and rank given to pt_dist_init)."""
        c, n, r = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
        _check(lib().pt_dist_info(self._c, ctypes.byref(c), ctypes.byref(n), ctypes.byref(r)), "pt_dist_info")
        return c.value, n.value, r.value

    def dist_run(self, n_batches, n_frames, frames_ptr=None, n_frame_bufs=1, n_streams=2):
        _check(lib().pt_dist_run(self._c, n_batches, n_frames, n_streams, frames_ptr, n_frame_bufs), "pt_dist_run")

    def dist_set_streams(self, render0=None, render1=None, gather=None):
        _check(lib().pt_dist_set_streams(self._c, render0, render1, gather), "pt_dist_set_streams")

    def dist_slot_floats(self):
        n = ctypes.c_size_t(0)
        _check(lib().pt_dist_slot_floats(self._c, ctypes.byref(n)), "pt_dist_slot_floats")
        return n.value

    def dist_wait(self, timeout_ms):
        _check(lib().pt_dist_wait(self._c, timeout_ms), "pt_dist_wait")

    def dist_abort(self):
        _check(lib().pt_dist_abort(self._c), "pt_dist_abort")

    def dist_finalize(self):
        _check(lib().pt_dist_finalize(self._c), "pt_dist_finalize")

    def traced(self):
        """Work the fast kernels actually did while PT_OPT_COUNT_TRACED was on
        (pt_get_traced), since the last reset_stats."""
        t = Traced()
        _check(lib().pt_get_traced(self._c, ctypes.byref(t)), "pt_get_traced")
        return {k: int(getattr(t, k)) for k, _ in Traced._fields_}

    def wide_info(self):
        """(wide nodes, stack bound) of the culled wide walk, or (0, 0, reason)."""
        info = (ctypes.c_int * 2)()
        _check(lib().pt_wide_info(self._c, info), "pt_wide_info")
        if info[0] == 0:
            return 0, 0, lib().pt_last_error().decode()
        return info[0], info[1]

    def mixed_info(self):
        """(schedule, live workgroups, measured launches) of the last launch:
        schedule 0 none, 1 static, 2 measured (PT_OPT_MIXED_LANES)."""
        info = (ctypes.c_int * 3)()
        _check(lib().pt_mixed_info(self._c, info), "pt_mixed_info")
        return info[0], info[1], info[2]

    def last_launch_ms(self):
        ms = ctypes.c_float()
        _check(lib().pt_last_launch_ms(self._c, ctypes.byref(ms)), "pt_last_launch_ms")
        return ms.value

    def launch_times_ms(self):
        n = ctypes.c_size_t()
        out = np.zeros(512, np.float32)
        _check(lib().pt_launch_times_ms(self._c, out.ctypes.data, out.size, ctypes.byref(n)), "pt_launch_times_ms")
        return out[: n.value].copy()

    def launch_span_ms(self):
        """(device ms from the first launch's start to the last end, launches)
        since reset_launch_times -- the busy span of overlapping launches."""
        ms, n = ctypes.c_float(), ctypes.c_size_t()
        _check(lib().pt_launch_span_ms(self._c, ctypes.byref(ms), ctypes.byref(n)), "pt_launch_span_ms")
        return ms.value, n.value

    def reset_launch_times(self):
        _check(lib().pt_reset_launch_times(self._c), "pt_reset_launch_times")

    def close(self):
        if self._c:
            lib().pt_destroy(self._c)
            self._c = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
