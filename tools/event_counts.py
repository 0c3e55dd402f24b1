"""Traversal event counts of the render kernel (diagnostic; never the product).

Loads build/librt_mi355x_cnt.so (make -C tinyraytracerinrust_amd diag NAME=cnt DIAG=-DRT_COUNT),
renders the 4K globes frame once and prints, per ray category, lane-events per frame: rays,
object box tests, objects entered, leaf box tests, leaf evaluations (by kind), CSG filter calls,
plus shade waterfall iterations (per wave).
"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("RT_LIB_PATH", os.path.join(ROOT, "tinyraytracerinrust_amd", "build", "librt_mi355x_cnt.so"))
sys.path.insert(0, ROOT)
import torch
import tinyraytracerinrust_amd as T
from tinyraytracerinrust_amd import _lib

S = os.path.join(ROOT, "tests", "golden", "scenes")
L = _lib.lib()
L.rt_diag_cnt.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 32)()
EV = ["rays", "obj box tests", "obj entered", "leaf box tests", "leaf evals", "  sphere", "  plane", "  cube",
      "filter calls"]
for W, H, d in [(3840, 2160, 10), (3840, 2160, 0)]:
    rt = T.RayTracer(W, H)
    rt.load_scene(open(os.path.join(S, "globes.scene")).read(), 0.0, asset_dir=S)
    r = rt.renderer
    out = r.render_rows(0, H, max_depth=d)
    torch.cuda.synchronize()
    L.rt_diag_cnt(buf)
    r.render_rows(0, H, max_depth=d, out=out)
    torch.cuda.synchronize()
    L.rt_diag_cnt(buf)
    print(f"globes {W}x{H} d={d}  (lane-events per frame; per-ray in brackets)")
    for c, nm in enumerate(["primary", "secondary", "shadow"]):
        rays = buf[c * 9] or 1
        print(f"  {nm}:")
        for i, e in enumerate(EV):
            v = buf[c * 9 + i]
            print(f"    {e:16s} {v:14d}  [{v / rays:7.3f}]")
    print(f"  shade waterfall iterations (per wave): {buf[27]}  waves {W * H // 64}")
