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
buf = (ctypes.c_ulonglong * 64)()
EV = ["rays", "obj box tests", "obj entered", "leaf box tests", "leaf evals", "  sphere", "  plane", "  cube",
      "filter calls"]
# usage: event_counts.py [SCENE WxH TIME DEPTH[,DEPTH...]]   (default: globes 3840x2160 0 10,0)
SCENE = sys.argv[1] if len(sys.argv) > 1 else "globes"
W0, H0 = (int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "3840x2160").split("x"))
TIME = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
DEPTHS = [int(v) for v in (sys.argv[4] if len(sys.argv) > 4 else "10,0").split(",")]
for W, H, d in [(W0, H0, dd) for dd in DEPTHS]:
    rt = T.RayTracer(W, H)
    rt.load_scene(open(os.path.join(S, SCENE + ".scene")).read(), TIME, asset_dir=S)
    r = rt.renderer
    out = r.render_rows(0, H, max_depth=d)
    torch.cuda.synchronize()
    L.rt_diag_cnt(buf)
    r.render_rows(0, H, max_depth=d, out=out)
    torch.cuda.synchronize()
    L.rt_diag_cnt(buf)
    print(f"{SCENE} {W}x{H} t={TIME:g} d={d}  (lane-events per frame; per-ray in brackets)")
    for c, nm in enumerate(["primary", "secondary", "shadow"]):
        rays = buf[c * 9] or 1
        print(f"  {nm}:")
        for i, e in enumerate(EV):
            v = buf[c * 9 + i]
            print(f"    {e:16s} {v:14d}  [{v / rays:7.3f}]")
    print(f"  shade waterfall iterations (per wave): {buf[27]}  waves {W * H // 64}")
    # SIMD lane utilisation: lane-events / (wave-events x 64)
    for c, nm in enumerate(["primary", "secondary", "shadow"]):
        wc, wl = buf[32 + c], buf[35 + c]
        print(f"  {nm:9s} traversal calls: {buf[c * 9] / max(1, 64 * wc):.3f} of lanes active; "
              f"leaf evaluations: {buf[c * 9 + 4] / max(1, 64 * wl):.3f} of lanes active ({wc} wave calls, {wl} wave leaf evals)")
    # per-object leaf evaluations (lane-events; objects in draw order, index mod 8)
    for c, nm in enumerate(["primary", "secondary", "shadow"]):
        print(f"  {nm:9s} leaf evals by object: " + " ".join(f"{o}:{buf[40 + c * 8 + o]}" for o in range(8)))

