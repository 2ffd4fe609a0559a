"""Regenerates tests/golden/oracle_frames.json — SHA-256 of oracle frames of
box.obj plus their traversal counters.  Run only when the oracle is changed
on purpose (and say why in the commit).  History: v1 frames used mul+add
polynomials; v2 (fma Horner chains) changed low-order bits only — identical
traversal counters and mean colour to 7 digits."""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402
import scenes  # noqa: E402

v, i, _ = O.obj_parse(open(scenes.BOX_OBJ, "rb").read())
ri, nodes = O.bvh_build(v, i)
cases = []
for W, H, spp, depth, sss in [(256, 256, 1, 1, 3), (256, 256, 1, 4, 3), (160, 90, 8, 4, 3)]:
    acc, st = O.render(v, ri, nodes, scenes.DEFAULT_CAMERA, scenes.REFERENCE_LIGHT, W, H, n_batches=spp,
                       max_depth=depth, sss_bounces=sss)
    cases.append({"W": W, "H": H, "spp": spp, "depth": depth, "sss": sss,
                  "sha256": hashlib.sha256(acc.tobytes()).hexdigest(), "stats": st.tolist(),
                  "mean_rgb": float(acc.reshape(-1, 4)[:, :3].mean())})
json.dump({"generator": "tests/golden/make_golden.py",
           "math_definition": "oracle/glsl_math.h v2: fdlibm float kernels, polynomials as fma Horner chains",
           "cases": cases}, open(os.path.join(HERE, "oracle_frames.json"), "w"),
          indent=1)
print(json.dumps(cases, indent=1))
