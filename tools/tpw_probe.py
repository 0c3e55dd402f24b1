"""Diagnostic (round 5): the specialised megakernel's tiles per wave
(rt_ctx_set_option RT_OPT_TILES_PER_WAVE: a wave takes its 8x8 tiles grid-stride) on the BASELINE
configs, one frame at a time on one stream (bench.py's N = 1 arrangement), settings interleaved over
rounds after a 300 ms settle.  Prints the ms per frame (one event pair around `--frames` launches)
and checks every frame buffer against a single-launch render.
usage: python tools/tpw_probe.py [--configs sphere1080d0,globes1080d5,globes4k] [--tpw 1,2,3,4,6,8]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
S = os.path.join(ROOT, "tests", "golden", "scenes")
CONFIGS = {"sphere1080d0": (None, 1920, 1080, 0), "globes1080d5": ("globes", 1920, 1080, 5),
           "globes4k": ("globes", 3840, 2160, 10)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="sphere1080d0,globes1080d5,globes4k")
    ap.add_argument("--tpw", default="1,2,3,4,6,8")
    ap.add_argument("--frames", type=int, default=0, help="frames per measurement (0: ~40 ms worth)")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    import tinyraytracerinrust_amd as T
    tpws = [int(v) for v in a.tpw.split(",")]
    for cfg in a.configs.split(","):
        scene, W, H, depth = CONFIGS[cfg]
        text = open(os.path.join(S, scene + ".scene")).read() if scene else "draw(sphere(<0, 0, 0>, 30, red))"
        r = T.Renderer(0, specialize=1)
        r.upload(T.Scene.compile(text, 0.0, W, H, asset_dir=S))
        r.spec_wait()
        r.set_timing(False)
        out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        whole = r.render_rows(0, H, max_depth=depth)        # calibration
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        ts = time.perf_counter()
        while time.perf_counter() - ts < 0.3:
            r.render_rows(0, H, max_depth=depth, out=out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            r.render_rows(0, H, max_depth=depth, out=out)
        torch.cuda.synchronize()
        n = a.frames or max(20, int(40.0 / ((time.perf_counter() - t0) * 100.0)))
        res = {t: [] for t in tpws}
        for rd in range(a.rounds):
            for t in tpws:
                r.set_tiles_per_wave(t)
                for _ in range(3):
                    r.render_rows(0, H, max_depth=depth, out=out)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(n):
                    r.render_rows(0, H, max_depth=depth, out=out)
                e1.record(st)
                torch.cuda.synchronize()
                res[t].append(e0.elapsed_time(e1) / n)
                if not torch.equal(out, whole):
                    raise SystemExit(f"{cfg} tpw {t}: frame differs from the single-launch render")
        print(f"{cfg}: {n} frames per measurement, ms per frame (median of {a.rounds} rounds) -- {r.kernel_info()}")
        for t in tpws:
            v = sorted(res[t])
            print(f"  tiles/wave {t}: {v[len(v) // 2]:.4f}   ({' '.join(f'{x:.4f}' for x in res[t])})", flush=True)
        r.free()


if __name__ == "__main__":
    main()
