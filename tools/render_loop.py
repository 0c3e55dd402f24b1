"""Render the 4K globes frame N times (profiling driver: PC sampling, counters)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import tinyraytracerinrust_amd as T
S = os.path.join(ROOT, "tests", "golden", "scenes")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
d = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rt = T.RayTracer(3840, 2160)
rt.load_scene(open(os.path.join(S, "globes.scene")).read(), 0.0, asset_dir=S)
r = rt.renderer
out = r.render_rows(0, 2160, max_depth=d)
for _ in range(n):
    r.render_rows(0, 2160, max_depth=d, out=out)
torch.cuda.synchronize()
print("frames", n, "last kernel ms", r.last_kernel_ms())
