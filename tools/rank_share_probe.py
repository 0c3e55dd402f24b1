"""Per-rank render at N ranks, emulated on one GPU (diagnostic): rank 0's cyclic 8-row bands of the
4K globes frame (the bench's default multi-GPU layout), timed with the context's kernel events for
each library given (longest-first tiles calibrated on the first launch)."""
import ctypes, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
S = os.path.join(ROOT, "tests", "golden", "scenes")
W, H, D = 3840, 2160, 10
text = open(os.path.join(S, "globes.scene")).read().encode()
SPEC = "--spec" in sys.argv                       # RT_OPT_SPECIALIZE = 1 on every context
for path in [a for a in sys.argv[1:] if a != "--spec"]:
    L = ctypes.CDLL(os.path.abspath(path))
    sc, cx = ctypes.c_void_p(), ctypes.c_void_p()
    assert L.rt_scene_compile(text, S.encode(), ctypes.c_double(0.0), W, H, ctypes.byref(sc)) == 0
    assert L.rt_ctx_create(0, ctypes.byref(cx)) == 0
    assert L.rt_ctx_upload(cx, sc) == 0
    if SPEC:
        assert L.rt_ctx_set_option(cx, 6, 1) == 0
    st = torch.cuda.current_stream().cuda_stream
    for n in (1, 2, 4, 8):
        band = 8
        n_bands = -(-(-(-H // band)) // n)          # bands dealt cyclically: ceil(ceil(H/8)/n)
        n_bands = min(n_bands, (H - 0 + band * n - 1) // (band * n))
        out = torch.empty((n_bands * band, W, 4), dtype=torch.uint8, device="cuda")
        ms = []
        for rep in range(23):
            rc = L.rt_render_row_bands(cx, 0, band, band * n, n_bands, D, ctypes.c_void_p(out.data_ptr()),
                                       ctypes.c_size_t(W * 4), ctypes.c_void_p(st))
            assert rc == 0, rc
            torch.cuda.synchronize()
            v = ctypes.c_float()
            L.rt_ctx_last_kernel_ms(cx, ctypes.byref(v))
            if rep >= 3:
                ms.append(v.value)
        print(f"N={n}: rank 0 renders {n_bands * band} rows: kernel median {statistics.median(ms):.4f} ms "
              f"min {min(ms):.4f}  ({path})", flush=True)
