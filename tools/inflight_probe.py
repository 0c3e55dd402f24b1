"""Diagnostic: a rank's share of the 4K globes frame at N ranks (rank 0's cyclic 8-row bands),
rendered with K frames in flight on K HIP streams on ONE GPU -- the render part of bench.py's
N-GPU step without the all-gather.  Prints the wall time per frame for each (N, K).
usage: python tools/inflight_probe.py LIB [LIB ...] [--frames F] [--kernel bench|auto|mega|deferred]
--kernel bench (default) is bench.py's choice: the library's automatic choice at K = 1, the
megakernel (rt_ctx_set_option RT_OPT_KERNEL) with frames in flight."""
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
    ap.add_argument("--kernel", default="bench", choices=["bench", "auto", "mega", "deferred", "wavefront"])
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--ks", default="1,2,3,4")
    ap.add_argument("--reps", type=int, default=1, help="repeat each (N, K) with a fresh context (new calibration)")
    ap.add_argument("--measures", type=int, default=1, help="timed runs per calibration")
    ap.add_argument("--fixed-streams", action="store_true", help="the same K streams for every repetition")
    ap.add_argument("--same-ctx", action="store_true", help="one context (one calibration) for every repetition")
    ap.add_argument("--streams", default="hw", choices=["hw", "pool"],
                    help="hw: rt_stream_create (a hardware queue each, as bench.py); pool: torch.cuda.Stream()")
    ap.add_argument("--options", nargs="*", default=["-"],
                    help="context option sets to compare, each OPT=VAL[,OPT=VAL] by number (rt_abi.h rt_option: 6 = "
                         "RT_OPT_SPECIALIZE, 7 = RT_OPT_TAIL_TILES); '-' for none")
    a = ap.parse_args()
    import torch
    W, H = 3840, 2160
    text = open(os.path.join(S, "globes.scene")).read().encode()
    for path, opts in [(p, o) for p in a.libs for o in a.options]:
        L = ctypes.CDLL(os.path.abspath(path))
        for n in (int(v) for v in a.ns.split(",")):
            band = 8
            n_bands = len(range(0, -(-H // band), n))
            kmax = max(int(v) for v in a.ks.split(","))
            outs = [torch.empty((n_bands * band, W, 4), dtype=torch.uint8, device="cuda") for _ in range(max(4, kmax))]
            for k in (int(v) for v in a.ks.split(",")):
                sys.path.insert(0, ROOT)
                import tinyraytracerinrust_amd as T
                hold = []

                def new_streams():
                    if a.streams == "pool":
                        return [torch.cuda.Stream() for _ in range(k)]
                    hs = [T.HwStream(0) for _ in range(k)]
                    hold.extend(hs)
                    return [h.torch for h in hs]
                fixed = new_streams()
                cx0 = None
                for rep in range(a.reps):
                    sc, cx = ctypes.c_void_p(), ctypes.c_void_p()
                    if cx0 is None or not a.same_ctx:
                        assert L.rt_scene_compile(text, S.encode(), ctypes.c_double(0.0), W, H, ctypes.byref(sc)) == 0
                        assert L.rt_ctx_create(0, ctypes.byref(cx)) == 0
                        assert L.rt_ctx_upload(cx, sc) == 0
                        cx0 = (cx, sc)
                    cx, sc = cx0
                    streams = fixed if a.fixed_streams else new_streams()
                    mode = ("auto" if k == 1 else "mega") if a.kernel == "bench" else a.kernel
                    assert L.rt_ctx_set_option(cx, 0, {"auto": 0, "mega": 1, "deferred": 2, "wavefront": 3}[mode]) == 0   # RT_OPT_KERNEL
                    if opts != "-":
                        for kv in opts.split(","):
                            o, v = (int(x) for x in kv.split("="))
                            assert L.rt_ctx_set_option(cx, o, v) == 0, kv

                    def issue(i):
                        s = streams[i % k]
                        rc = L.rt_render_row_bands(cx, 0, band, band * n, n_bands, a.depth,
                                                   ctypes.c_void_p(outs[i % k].data_ptr()), ctypes.c_size_t(W * 4),
                                                   ctypes.c_void_p(s.cuda_stream))
                        assert rc == 0
                    for i in range(2 * k + 2):            # calibration + warm-up
                        issue(i)
                    torch.cuda.synchronize()
                    res = []
                    for _ in range(a.measures):
                        t0 = time.perf_counter()
                        for i in range(a.frames):
                            issue(i)
                        torch.cuda.synchronize()
                        res.append((time.perf_counter() - t0) * 1e3 / a.frames)
                    if not a.same_ctx:
                        L.rt_ctx_free(cx)
                        L.rt_scene_free(sc)
                    print(f"N={n} K={k}: {' '.join(f'{v:.4f}' for v in res)} ms per frame share, {mode} kernel, {a.streams} streams, options {opts}  ({path})",
                          flush=True)


if __name__ == "__main__":
    sys.exit(main())
