"""Frames in flight (diagnostic): render N frames of one scene round-robin over K HIP streams and
print ms per frame.  Independent frames on separate streams let one kernel's last waves share the
GPU with the next kernel's first ones."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import tinyraytracerinrust_amd as T
S = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "scenes")
for (W, H, d, scene) in [(3840, 2160, 10, "globes"), (1920, 1080, 5, "globes"), (1920, 1080, 10, "spinning_globes")]:
    rt = T.RayTracer(W, H)
    rt.load_scene(open(os.path.join(S, scene + ".scene")).read(), 0.0, asset_dir=S)
    r = rt.renderer
    outs = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(4)]
    for K in (1, 2, 3, 4):
        st = [torch.cuda.current_stream()] if K == 1 else [torch.cuda.Stream() for _ in range(K)]
        for i in range(8):
            r.render_rows(0, H, max_depth=d, out=outs[i % 4], stream=st[i % K])
        torch.cuda.synchronize()
        res = []
        for rep in range(5):
            t0 = time.perf_counter()
            for i in range(40):
                r.render_rows(0, H, max_depth=d, out=outs[i % 4], stream=st[i % K])
            torch.cuda.synchronize()
            res.append((time.perf_counter() - t0) * 1e3 / 40)
        res.sort()
        print(f"{scene} {W}x{H} d={d} streams={K}: ms/frame median {res[2]:.4f} min {res[0]:.4f}", flush=True)
