"""Lone-frame kernel time of a bundled scene at several depths and kernel choices (diagnostic;
bench.py is the contract).  One context per (depth, kernel); the first launch calibrates, then
REPS ordered launches are timed with the library's launch events (median printed).
usage: python tools/scene_timing.py SCENE WxH TIME DEPTHS [KERNELS] [REPS]
  e.g. python tools/scene_timing.py fractal 1920x1080 0 0,1,2,4,10 auto,mega,wavefront:p0,wavefront:p2 5"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import tinyraytracerinrust_amd as T  # noqa: E402

S = os.path.join(ROOT, "tests", "golden", "scenes")
scene, size, t, depths = sys.argv[1], sys.argv[2], float(sys.argv[3]), [int(v) for v in sys.argv[4].split(",")]
kernels = sys.argv[5].split(",") if len(sys.argv) > 5 else ["auto"]
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
W, H = (int(v) for v in size.split("x"))
text = open(os.path.join(S, scene + ".scene")).read()
for d in depths:
    for k in kernels:
        rt = T.RayTracer(W, H)
        rt.max_depth = d
        rt.load_scene(text, t, asset_dir=S)
        r = rt.renderer
        kn, _, pm = k.partition(":p")                     # e.g. wavefront:p0 = RT_OPT_WAVEFRONT_PAIRS 0
        r.set_kernel(kn)
        if pm:
            r.set_wavefront_pairs(int(pm))
        out = r.render_rows(0, H)
        torch.cuda.synchronize()
        cal = r.last_kernel_ms()
        ms = []
        for _ in range(reps):
            r.render_rows(0, H, out=out)
            ms.append(r.last_kernel_ms())
        print(f"{scene} {W}x{H} t={t} d={d} kernel={k}: calibration {cal:.3f} ms, ordered median "
              f"{statistics.median(ms):.4f} min {min(ms):.4f} ms", flush=True)
