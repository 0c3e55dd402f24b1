"""Interleaved A/B of librt_mi355x.so builds on a BASELINE config, one frame at a time on one stream
(bench.py's N = 1 arrangement), each library through its own ctypes handle, context and upload, with
the specialised kernels loaded (RT_OPT_SPECIALIZE 1, rt_ctx_spec_wait) unless --generic.  Prints the
ms per frame (one event pair around --frames launches) per library, median over --rounds.
usage: python tools/ab_libs.py LIB [LIB ...] [--config sphere1080d0|globes1080d5|globes4k] [--generic]"""
import argparse
import ctypes
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
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--config", default="sphere1080d0")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=0)
    ap.add_argument("--generic", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="ablation libraries: do not require equal frames")
    ap.add_argument("--levels", default="", help="per library (in order): its RT_OPT_SPECIALIZE level, e.g. 1,2 "
                                                   "(a library path may repeat); default 1 (0 with --generic)")
    a = ap.parse_args()
    import torch
    scene, W, H, depth = CONFIGS[a.config]
    text = (open(os.path.join(S, scene + ".scene")).read() if scene else "draw(sphere(<0, 0, 0>, 30, red))").encode()
    ctxs, outs = [], []
    levels = [int(v) for v in a.levels.split(",")] if a.levels else [0 if a.generic else 1] * len(a.libs)
    for path, level in zip(a.libs, levels):
        L = ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL)
        L.rt_ctx_spec_wait.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        sc, cx = ctypes.c_void_p(), ctypes.c_void_p()
        assert L.rt_scene_compile(text, S.encode(), ctypes.c_double(0.0), W, H, ctypes.byref(sc)) == 0
        assert L.rt_ctx_create(0, ctypes.byref(cx)) == 0
        assert L.rt_ctx_set_option(cx, 6, level) == 0
        assert L.rt_ctx_upload(cx, sc) == 0
        assert L.rt_ctx_spec_wait(cx, -1) == 0
        assert L.rt_ctx_set_option(cx, 1, 0) == 0                  # RT_OPT_TIMING off, as bench.py
        ctxs.append((L, cx))
        outs.append(torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda"))
    st = torch.cuda.current_stream()

    def launch(i):
        L, cx = ctxs[i]
        assert L.rt_render_rows(cx, 0, H, depth, ctypes.c_void_p(outs[i].data_ptr()), ctypes.c_size_t(W * 4),
                                ctypes.c_void_p(st.cuda_stream)) == 0
    for i in range(len(ctxs)):
        launch(i)                                                   # calibration
    torch.cuda.synchronize()
    ts = time.perf_counter()
    while time.perf_counter() - ts < 0.3:
        for i in range(len(ctxs)):
            launch(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        launch(0)
    torch.cuda.synchronize()
    n = a.frames or max(20, int(0.04 / ((time.perf_counter() - t0) / 10)))
    res = [[] for _ in ctxs]
    for _ in range(a.rounds):
        for i in range(len(ctxs)):
            for _ in range(3):
                launch(i)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(n):
                launch(i)
            e1.record(st)
            torch.cuda.synchronize()
            res[i].append(e0.elapsed_time(e1) / n)
    for i in range(1, len(outs)):
        if not a.no_check and not torch.equal(outs[i], outs[0]):
            raise SystemExit(f"{a.libs[i]}: frame differs from {a.libs[0]}'s")
    print(f"{a.config} ({'generic' if a.generic else 'specialised'}), {n} frames per measurement, ms per frame, median of {a.rounds}:")
    for path, level, v in zip(a.libs, levels, res):
        w = sorted(v)
        print(f"  {w[len(w) // 2]:.4f}  ({' '.join(f'{x:.4f}' for x in v)})  {path} (RT_OPT_SPECIALIZE {level})", flush=True)


if __name__ == "__main__":
    main()
