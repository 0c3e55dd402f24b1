"""Quick timing of the 4K globes frame on one GPU (diagnostic; bench.py is the contract)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import tinyraytracerinrust_amd as T
S = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "scenes")
CASES = [(3840, 2160, 10, "globes"), (3840, 2160, 0, "globes"), (1920, 1080, 5, "globes"), (1920, 1080, 0, None)]
for (W, H, d, scene) in CASES:
    rt = T.RayTracer(W, H)
    if scene:
        rt.load_scene(open(os.path.join(S, scene + ".scene")).read(), 0.0, asset_dir=S)
    else:
        rt.load_scene("draw(sphere(<0, 0, 0>, 30, red))", 0.0)
    r = rt.renderer
    out = r.render_rows(0, H, max_depth=d)
    torch.cuda.synchronize()
    ms = []
    for i in range(5):
        r.render_rows(0, H, max_depth=d, out=out)
        ms.append(r.last_kernel_ms())
    print(f"{scene or 'sphere'} {W}x{H} d={d}: kernel ms {['%.2f' % m for m in ms]}  "
          f"Mrays/s {W * H / (min(ms) * 1e-3) / 1e6:.1f}", flush=True)
