import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "discovering-path-tracer_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa
import ptamd, scenes
s = ptamd.Scene.load_obj(scenes.BOX_OBJ).build_bvh()
v, i, n, _, _ = s.arrays()
W, H, SPP = int(sys.argv[1]), int(sys.argv[2]), 8
def mk(nr, rk, opts):
    r = ptamd.Renderer(0)
    r.upload_scene(v, i, n); r.upload_lights(scenes.REFERENCE_LIGHT); r.set_camera(scenes.DEFAULT_CAMERA); r.set_params(4, 3)
    r.set_partition(nr, rk)
    for k, val in opts: r.set_option(k, val)
    r.resize_and_clear(W, H)
    return r
ref = mk(1, 0, []); ref.render(0, SPP); want = ref.read_accum()
for name, opts in [("default", []), ("nocull", [(ptamd.PT_OPT_PRIMARY_CULL, 0)]), ("spl2", [(ptamd.PT_OPT_SAMPLE_LANES, 2)]),
                   ("spl4", [(ptamd.PT_OPT_SAMPLE_LANES, 4)])]:
    acc = np.full(W * H * 4, -0.0, np.float32)
    for rk in range(2):
        r = mk(2, rk, opts); r.clear(); r.render(0, SPP); acc = (acc + r.read_accum()).astype(np.float32)
    bad = np.flatnonzero(acc.view(np.uint32) != want.view(np.uint32))
    print(name, "mismatches", bad.size, (bad[:5] // 4, acc[bad[:5]], want[bad[:5]]) if bad.size else "")
