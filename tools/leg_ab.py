import sys, os
sys.path.insert(0, "/root/repo")
os.chdir(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
sys.argv = ["bench.py"]
import torch  # noqa
import bench
for c in (1, 2, 3, 3, 2):
    out = bench.scene_leg("sphere", 1920, 1080, 8, 4, 3, 12, 0, "sphere_1080p8", contexts=c)
    print("contexts", c, out["ms_per_step"], out["ms_per_frame"], flush=True)
