import sys, os
sys.path.insert(0, "/root/repo")
os.chdir(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
sys.argv = ["bench.py"]
import torch  # noqa
import bench
# LEG_CONTEXTS="3 4 3 4" (default: 1 2 3 3 2); LEG_FRAMES (default 12)
ctx = [int(x) for x in os.environ.get("LEG_CONTEXTS", "1 2 3 3 2").split()]
for c in ctx:
    out = bench.scene_leg("sphere", 1920, 1080, 8, 4, 3, int(os.environ.get("LEG_FRAMES", "12")), 0, "sphere_1080p8",
                          contexts=c)
    print("contexts", c, out["ms_per_step"], out["ms_per_frame"], flush=True)
