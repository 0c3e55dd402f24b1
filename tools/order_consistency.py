"""Ordered launches reproduce the calibration launch bit-for-bit (diagnostic, per library given):
4K globes d10 and 1080p spinning_globes, full frame and rank-0 cyclic bands at N=8."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import torch
S = os.path.join(ROOT, "tests", "golden", "scenes")
for path in sys.argv[1:]:
    L = ctypes.CDLL(os.path.abspath(path))
    for scene, W, H in (("globes", 3840, 2160), ("spinning_globes", 1920, 1080)):
        text = open(os.path.join(S, scene + ".scene")).read().encode()
        sc, cx = ctypes.c_void_p(), ctypes.c_void_p()
        assert L.rt_scene_compile(text, S.encode(), ctypes.c_double(0.0), W, H, ctypes.byref(sc)) == 0
        assert L.rt_ctx_create(0, ctypes.byref(cx)) == 0
        assert L.rt_ctx_upload(cx, sc) == 0
        st = torch.cuda.current_stream().cuda_stream
        for (bands, pitch, n) in ((H, H, 1), (8, 64, 34)):
            outs = []
            for rep in range(3):
                o = torch.zeros((bands * n, W, 4), dtype=torch.uint8, device="cuda")
                assert L.rt_render_row_bands(cx, 0, bands, pitch, n, 10, ctypes.c_void_p(o.data_ptr()),
                                             ctypes.c_size_t(W * 4), ctypes.c_void_p(st)) == 0
                torch.cuda.synchronize()
                outs.append(o)
            ok = all(torch.equal(outs[0], o) for o in outs[1:])
            print(f"{os.path.basename(path)} {scene} {W}x{H} bands {bands}/{pitch}x{n}: ordered == calibration: {ok}", flush=True)
            if not ok:
                sys.exit(1)
