"""Interleaved A/B kernel timing of several builds of librt_mi355x.so in ONE process (diagnostic).

Each library is loaded with its own ctypes handle (RTLD_LOCAL, so identical symbol names do not
clash), gets its own context and scene upload, and the 4K globes frame is rendered round-robin
over the libraries REPS times; the median / min kernel ms per library are printed.  Interleaving
cancels clock drift (DVFS) between variants, which separate runs do not.
usage: python tools/ab_interleaved.py LIB [LIB ...] [--reps N] [--depth D] [--size WxH] [--scene NAME]
"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(ROOT, "tests", "golden", "scenes")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--size", default="3840x2160")
    ap.add_argument("--scene", default="globes")
    ap.add_argument("--time", type=float, default=0.0)
    ap.add_argument("--burst", type=int, default=1,
                    help="launches back to back per measurement (sustained clocks); the time per launch is "
                         "the burst's wall time / burst")
    ap.add_argument("--upload-env", nargs="*", default=[],
                    help="per library (in order): KEY=VAL set in the environment while its scene is compiled and "
                         "uploaded (host-side flattening switches of a `make diag DIAG=-DRT_DIAG_ENV` build, e.g. RT_NO_LIT_ORDER=1); '-' for none")
    ap.add_argument("--check", action="store_true",
                    help="after timing, render once more per library and require every frame to equal the first's")
    ap.add_argument("--kernel", nargs="*", default=[],
                    help="per library (in order): RT_OPT_KERNEL auto / mega / deferred for its context; '-' keeps auto. "
                         "A library path may repeat with different kernels")
    ap.add_argument("--option", nargs="*", default=[],
                    help="per library (in order): OPT=VAL[,OPT=VAL] context options by number (rt_abi.h rt_option, "
                         "e.g. 6=1 for RT_OPT_SPECIALIZE); '-' for none")
    ap.add_argument("--family", nargs="*", default=[],
                    help="per library (in order): F registers the scene's F-frame animation (time f / F) as scene "
                         "families (rt_spec_family_register) before its options are set; '-' for none")
    a = ap.parse_args()
    import time
    import torch
    W, H = (int(v) for v in a.size.split("x"))
    # "sphere": bench.py's one-line scene of BASELINE config 2
    text = (b"draw(sphere(<0, 0, 0>, 30, red))" if a.scene == "sphere"
            else open(os.path.join(SCENES, a.scene + ".scene")).read().encode())
    out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ctxs = []
    for li, path in enumerate(a.libs):
        env = a.upload_env[li] if li < len(a.upload_env) and a.upload_env[li] != "-" else None
        if env:
            k, v = env.split("=", 1)
            os.environ[k] = v
        L = ctypes.CDLL(os.path.abspath(path))
        sc, cx = ctypes.c_void_p(), ctypes.c_void_p()
        assert L.rt_scene_compile(text, SCENES.encode(), ctypes.c_double(a.time), W, H, ctypes.byref(sc)) == 0
        assert L.rt_ctx_create(0, ctypes.byref(cx)) == 0
        assert L.rt_ctx_upload(cx, sc) == 0
        if env:
            del os.environ[env.split("=", 1)[0]]
        kern = a.kernel[li] if li < len(a.kernel) and a.kernel[li] != "-" else None
        if kern:
            assert L.rt_ctx_set_option(cx, 0, {"auto": 0, "mega": 1, "deferred": 2}[kern]) == 0
        fam = int(a.family[li]) if li < len(a.family) and a.family[li] != "-" else 0
        if fam:
            L.rt_spec_family_clear()
            fs = []
            for f in range(fam):
                s = ctypes.c_void_p()
                tf = a.time if fam == 1 else f / fam         # a family of one: the scene itself
                assert L.rt_scene_compile(text, SCENES.encode(), ctypes.c_double(tf), W, H, ctypes.byref(s)) == 0
                fs.append(s)
            arr = (ctypes.c_void_p * fam)(*[s.value for s in fs])
            ms = ctypes.c_double()
            assert L.rt_spec_family_register(arr, fam, ctypes.byref(ms)) == 0
            print(f"{path}: {fam}-frame families registered, {ms.value:.0f} ms", flush=True)
        opt = a.option[li] if li < len(a.option) and a.option[li] != "-" else None
        if opt:
            for kv in opt.split(","):
                k, v = (int(x) for x in kv.split("="))
                t0 = time.perf_counter()
                rc = L.rt_ctx_set_option(cx, k, v)
                assert rc == 0, (kv, rc)
                print(f"{path}: option {k}={v} in {(time.perf_counter() - t0) * 1e3:.0f} ms", flush=True)
        ctxs.append((path + (f" family{fam}" if fam else "") + (f" [{env}]" if env else "") + (f" <{kern}>" if kern else "") + (f" {{{opt}}}" if opt else ""),
                     L, cx, []))
    for rep in range(a.reps + 3):
        for path, L, cx, ms in ctxs:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.burst):
                rc = L.rt_render_rows(cx, 0, H, a.depth, ctypes.c_void_p(out.data_ptr()), ctypes.c_size_t(W * 4),
                                      ctypes.c_void_p(st))
                assert rc == 0, rc
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3 / a.burst
            v = ctypes.c_float()
            L.rt_ctx_last_kernel_ms(cx, ctypes.byref(v))
            if rep >= 3:
                ms.append(v.value if a.burst == 1 else dt)
    if a.check:
        frames = []
        for path, L, cx, ms in ctxs:
            o = torch.zeros_like(out)
            assert L.rt_render_rows(cx, 0, H, a.depth, ctypes.c_void_p(o.data_ptr()), ctypes.c_size_t(W * 4),
                                    ctypes.c_void_p(st)) == 0
            torch.cuda.synchronize()
            frames.append(o)
        for (path, *_), f in zip(ctxs[1:], frames[1:]):
            same = bool(torch.equal(f, frames[0]))
            print(f"check: {path} frame {'==' if same else '!='} {ctxs[0][0]} frame", flush=True)
            if not same:
                return 1
    base = None
    for path, L, cx, ms in ctxs:
        med = statistics.median(ms)
        base = base or med
        print(f"{a.scene} {W}x{H} d={a.depth}  median {med:.4f} ms  min {min(ms):.4f}  ({med / base:.3f}x of first)  {path}",
              flush=True)


if __name__ == "__main__":
    sys.exit(main())
