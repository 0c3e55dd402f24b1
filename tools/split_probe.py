"""One frame as several launches on several HIP streams (diagnostic): the frame's rows are split
into K contiguous parts, part k launched on stream k (after an event on the current stream), and
the current stream waits for all parts.  Prints ms per frame against K."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import tinyraytracerinrust_amd as T
S = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "scenes")
for (W, H, d, scene) in [(3840, 2160, 10, "globes"), (1920, 1080, 5, "globes"), (1920, 1080, 10, "spinning_globes")]:
    rt = T.RayTracer(W, H)
    rt.load_scene(open(os.path.join(S, scene + ".scene")).read(), 0.0, asset_dir=S)
    r = rt.renderer
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    ref = r.render_rows(0, H, max_depth=d).clone()
    cur = torch.cuda.current_stream()
    for K in (1, 2, 3, 4, 8):
        st = [torch.cuda.Stream() for _ in range(K)]
        cuts = [H * k // K for k in range(K + 1)]
        def frame():
            ev = torch.cuda.Event(); ev.record(cur)
            for k in range(K):
                st[k].wait_event(ev)
                r.render_rows(cuts[k], cuts[k + 1], max_depth=d, out=out[cuts[k]:cuts[k + 1]], stream=st[k])
            for k in range(K):
                e = torch.cuda.Event(); e.record(st[k]); cur.wait_event(e)
        for i in range(5):
            frame()
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
        res = []
        for rep in range(5):
            t0 = time.perf_counter()
            for i in range(20):
                frame()
            torch.cuda.synchronize()
            res.append((time.perf_counter() - t0) * 1e3 / 20)
        res.sort()
        print(f"{scene} {W}x{H} d={d} parts={K}: ms/frame median {res[2]:.4f} min {res[0]:.4f}", flush=True)
