"""Diagnostic: a rank's share of the 4K globes frame at N ranks (rank 0's cyclic 8-row bands),
rendered with K frames in flight on K HIP streams on ONE GPU -- the render part of bench.py's
N-GPU step without the all-gather.  Prints the wall time per frame for each (N, K).
usage: python tools/inflight_probe.py LIB [LIB ...] [--frames F]"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
S = os.path.join(ROOT, "tests", "golden", "scenes")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--depth", type=int, default=10)
    a = ap.parse_args()
    import torch
    W, H = 3840, 2160
    text = open(os.path.join(S, "globes.scene")).read().encode()
    for path in a.libs:
        L = ctypes.CDLL(os.path.abspath(path))
        sc, cx = ctypes.c_void_p(), ctypes.c_void_p()
        assert L.rt_scene_compile(text, S.encode(), ctypes.c_double(0.0), W, H, ctypes.byref(sc)) == 0
        assert L.rt_ctx_create(0, ctypes.byref(cx)) == 0
        assert L.rt_ctx_upload(cx, sc) == 0
        for n in (1, 2, 4, 8):
            band = 8
            n_bands = len(range(0, -(-H // band), n))
            outs = [torch.empty((n_bands * band, W, 4), dtype=torch.uint8, device="cuda") for _ in range(4)]
            for k in (1, 2, 3, 4):
                streams = [torch.cuda.Stream() for _ in range(k)]

                def issue(i):
                    s = streams[i % k]
                    rc = L.rt_render_row_bands(cx, 0, band, band * n, n_bands, a.depth,
                                               ctypes.c_void_p(outs[i % k].data_ptr()), ctypes.c_size_t(W * 4),
                                               ctypes.c_void_p(s.cuda_stream))
                    assert rc == 0
                for i in range(2 * k + 2):            # calibration + warm-up
                    issue(i)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(a.frames):
                    issue(i)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) * 1e3 / a.frames
                print(f"N={n} K={k}: {dt:.4f} ms per frame share  ({path})", flush=True)


if __name__ == "__main__":
    sys.exit(main())
