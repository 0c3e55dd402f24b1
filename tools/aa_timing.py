"""Time the anti-aliasing pass on the 4K globes frame (diagnostic)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import tinyraytracerinrust_amd as T
S = os.path.join(ROOT, "tests", "golden", "scenes")
for W, H in [(1920, 1080), (3840, 2160)]:
    rt = T.RayTracer(W, H)
    rt.load_scene(open(os.path.join(S, "globes.scene")).read(), 0.0, asset_dir=S)
    r = rt.renderer
    frame = r.render_rows(0, H)
    out, rays = r.antialias(frame, 0.01, 3)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        out, rays = r.antialias(frame, 0.01, 3, out=out)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    print(f"AA globes {W}x{H}: {min(ts):.2f} ms wall (kernels {r.last_kernel_ms():.2f} ms), "
          f"{rays} sub-pixel rays = {rays / (W * H):.3f}/px, {rays / (min(ts) * 1e-3) / 1e6:.0f} Mrays/s", flush=True)
