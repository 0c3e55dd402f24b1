"""Section cost split of the render kernel (diagnostic; never the product).

Loads build/librt_mi355x_prof.so (make -C tinyraytracerinrust_amd profile-sections), renders the
4K globes frame, and prints the wave-cycles spent in each part of trace() as a share of the
whole-kernel wave-cycles.  Sections: primary nearest_hit, secondary nearest_hit, shadow rays,
shade_inputs (normal/UV/material), everything between nearest_hit and the combine (includes
shadows + shading), whole trace per wave.
"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("RT_LIB_PATH", os.path.join(ROOT, "tinyraytracerinrust_amd", "build", "librt_mi355x_prof.so"))
sys.path.insert(0, ROOT)
import torch
import tinyraytracerinrust_amd as T
from tinyraytracerinrust_amd import _lib

NAMES = ["primary nearest_hit", "secondary nearest_hit", "shadow_transparency", "shade_inputs",
         "hit->combine (incl. shadows+shade)", "whole trace"]
S = os.path.join(ROOT, "tests", "golden", "scenes")
CASES = [(3840, 2160, 10, "globes"), (3840, 2160, 0, "globes")]
L = _lib.lib()
L.rt_diag_prof.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 8)()
for W, H, d, scene in CASES:
    rt = T.RayTracer(W, H)
    rt.load_scene(open(os.path.join(S, scene + ".scene")).read(), 0.0, asset_dir=S)
    r = rt.renderer
    out = r.render_rows(0, H, max_depth=d)
    torch.cuda.synchronize()
    L.rt_diag_prof(buf)                          # reset after warm-up
    n = 5
    for _ in range(n):
        r.render_rows(0, H, max_depth=d, out=out)
    ms = r.last_kernel_ms()
    L.rt_diag_prof(buf)
    tot = buf[5] or 1
    print(f"{scene} {W}x{H} d={d}: kernel {ms:.3f} ms (instrumented)")
    for i, nm in enumerate(NAMES):
        print(f"  {nm:38s} {buf[i] / n:16.0f} wave-cycles/frame  {100 * buf[i] / tot:6.1f} %")
