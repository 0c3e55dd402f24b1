"""The library's DEFAULT render path (RT_OPT_SPECIALIZE 1, round 5): rt_ctx_upload requests the scene's
specialised program from the library's compile pool and returns at once; launches run the generic
kernels until the code object is ready and the specialised ones from the next launch on.  A host shaped
like the reference's (upload, then render frame after frame: debug_window.rs:53-87, gui.rs:78-89) never
blocks on the compile.  Every frame -- before, across and after the swap -- against the CPU oracle (a
restatement of src/raytracer/raytracer.rs:132-287), RGBA8 bit-identical.

Also here: the context's completion events (rt_ctx_synchronize / rt_ctx_free never touch a caller's
stream, which may be destroyed by then), and a compile that fails keeps the generic kernels."""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

from tests.conftest import ROOT, SCENES, scene_text
from tests.test_gpu_parity import assert_close

pytestmark = pytest.mark.gpu


def _oracle(text, t, W, H, depth):
    from oracle import oracle as O
    return O.OracleScene(text, t, W, H, max_depth=depth).render(0, H)[1]


def test_default_upload_renders_at_once_then_swaps(worldmap):
    """A scene no other test compiles (a random fuzz scene), the library's default option value:
    the first frame renders on the generic kernels while the program compiles, later frames on the
    specialised kernel once loaded, each exact.  Upload + first frame take far less than a compile."""
    import torch
    import tinyraytracerinrust_amd as T
    from tests.scene_fuzz import random_scene
    W, H = 320, 240
    text = random_scene(7771)
    ref = _oracle(text, 0.0, W, H, 10)
    sc = T.Scene.compile(text, 0.0, W, H, asset_dir=SCENES)
    r = T.Renderer(0, specialize=T.Renderer.LIBRARY_DEFAULT)     # the library's own default (1)
    t0 = time.perf_counter()
    r.upload(sc)
    f = r.render_rows(0, H)
    torch.cuda.synchronize()
    first_ms = (time.perf_counter() - t0) * 1e3
    info0 = r.kernel_info()
    assert_close(f.cpu().numpy(), None, ref, None, f"first frame ({info0})")
    assert info0.startswith("generic") and "compiling in the background" in info0, info0
    kinds = set()
    deadline = time.time() + 300
    while time.time() < deadline:
        f = r.render_rows(0, H)
        torch.cuda.synchronize()
        info = r.kernel_info()
        assert_close(f.cpu().numpy(), None, ref, None, f"frame during the compile ({info})")
        kinds.add(info.split("last launch: ")[1])
        if info.startswith("scene-specialised") and "(specialised)" in info:
            break
        time.sleep(0.05)
    assert info.startswith("scene-specialised") and "(specialised)" in info, info
    for _ in range(3):
        f = r.render_rows(0, H)
        torch.cuda.synchronize()
        assert_close(f.cpu().numpy(), None, ref, None, f"frame after the swap ({r.kernel_info()})")
    print(f"first frame after upload {first_ms:.1f} ms; kernels seen {sorted(kinds)}; {info}")
    assert first_ms < 1000, first_ms


def test_spec_wait_pending_then_loaded(worldmap):
    """rt_ctx_spec_wait: 0 ms right after the upload of an uncompiled scene -> pending (False); no
    limit -> loaded; the next launch is specialised and exact."""
    import tinyraytracerinrust_amd as T
    from tests.scene_fuzz import random_scene
    W, H = 160, 120
    text = random_scene(7772)
    sc = T.Scene.compile(text, 0.0, W, H, asset_dir=SCENES)
    r = T.Renderer(0, specialize=1)
    r.upload(sc)
    assert r.spec_wait(0) is False
    assert r.spec_wait() is True
    a = r.render_rows_host(0, H)
    assert "megakernel (specialised)" in r.kernel_info() or "deferred (specialised)" in r.kernel_info(), r.kernel_info()
    assert_close(a, None, _oracle(text, 0.0, W, H, 10), None, f"after spec_wait ({r.kernel_info()})")


def test_swap_recalibrates_deferred_orders(worldmap):
    """1080p globes d5 (a tail-bound launch: the generic path's choice is the deferred kernel with split
    tiles): ordered launches before the specialised program is loaded, then after it (the deferred order
    is dropped at the swap and the geometry calibrates again for the specialised megakernel); every frame
    exact."""
    import torch
    import tinyraytracerinrust_amd as T
    W, H = 1920, 1080
    text = scene_text("globes")
    ref = _oracle(text, 0.0, W, H, 5)
    r = T.Renderer(0, specialize=0)
    r.upload(T.Scene.compile(text, 0.0, W, H, asset_dir=SCENES))
    seen = []
    for _ in range(3):
        f = r.render_rows(0, H, max_depth=5)
        torch.cuda.synchronize()
        seen.append(r.kernel_info().split("last launch: ")[1])
        assert_close(f.cpu().numpy(), None, ref, None, f"generic ({seen[-1]})")
    r.set_specialize(1, wait=True)
    for _ in range(3):
        f = r.render_rows(0, H, max_depth=5)
        torch.cuda.synchronize()
        seen.append(r.kernel_info().split("last launch: ")[1])
        assert_close(f.cpu().numpy(), None, ref, None, f"specialised ({seen[-1]})")
    assert "specialised" in seen[-1] and all("specialised" not in k for k in seen[:3]), seen


def test_synchronize_and_free_after_the_stream_is_gone(worldmap):
    """Launches on own-queue streams that are destroyed right after: rt_ctx_synchronize and rt_ctx_free
    wait on the context's own completion events, never on the (destroyed) streams -- round 4 crashed at
    exit synchronising a destroyed stream.  The frames are exact."""
    import torch
    import tinyraytracerinrust_amd as T
    W, H = 320, 240
    text = scene_text("globes")
    ref = _oracle(text, 0.0, W, H, 10)
    r = T.Renderer(0, specialize=0)
    r.upload(T.Scene.compile(text, 0.0, W, H, asset_dir=SCENES))
    outs = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(6)]
    for i in range(6):
        h = T.HwStream(0)
        r.render_rows(0, H, out=outs[i], stream=h.torch)
        h.close()                                        # the stream is gone before the render is waited for
    r.synchronize()
    for o in outs:
        assert_close(o.cpu().numpy(), None, ref, None, "frame on a destroyed stream")
    r.free()


def test_failed_compile_keeps_generic_kernels():
    """A compile that cannot happen (the pool stopped by rt_spec_shutdown, in a fresh process so the rest
    of the suite keeps its pool): the upload succeeds, the kernel info says why specialisation is off,
    rt_ctx_spec_wait reports the failure, and the frame is the oracle's through the generic kernels."""
    code = f"""
import sys; sys.path.insert(0, {ROOT!r})
import numpy as np, torch
import tinyraytracerinrust_amd as T
from oracle import oracle as O
S = {SCENES!r}
O.register_texture_file("worldmap.png", S + "/worldmap.png")
text = open(S + "/globes.scene").read()
T.lib().rt_spec_shutdown()
r = T.Renderer(0, specialize=1)
r.upload(T.Scene.compile(text, 0.0, 160, 120, asset_dir=S))
try:
    r.spec_wait()
    raise SystemExit("spec_wait did not report the failure")
except T.RtError as e:
    assert "shut down" in e.message, e.message
a = r.render_rows_host(0, 120)
info = r.kernel_info()
assert info.startswith("generic") and "specialisation failed" in info, info
ref = O.OracleScene(text, 0.0, 160, 120).render(0, 120)[1]
assert np.array_equal(a, ref), int((a != ref).sum())
print("ok", info)
"""
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, RT_SPEC_CACHE_DIR=""))
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-3000:]
    assert "ok generic" in res.stdout


@pytest.mark.parametrize("case", ["globes_d10", "globes_d5_bands", "globes_f64", "spinning_chain",
                                  "fuzz_tree", "globes_deferred", "fractal_wavefront"])
def test_library_default_parity_subset(worldmap, case):
    """the rest of the suite pins RT_OPT_SPECIALIZE 0 (conftest), so a representative
    subset runs here with the option as the LIBRARY sets it (specialize=LIBRARY_DEFAULT, i.e. 1), after
    rt_ctx_spec_wait: whatever kernel the default path then picks -- the specialised megakernel, the
    deferred or wavefront requests, row bands, f64 rows (generic: option level 1 keeps f64 generic) --
    every launch (calibration and ordered) is the oracle's, RGBA8 bit-identical / f64 within 1e-9."""
    import torch
    import tinyraytracerinrust_amd as T
    from oracle import oracle as O
    from tests.scene_fuzz import random_scene
    W, H, depth, t, kernel = 320, 240, 10, 0.0, None
    if case.startswith("globes"):
        text = scene_text("globes")
        depth = 5 if case == "globes_d5_bands" else 10
        kernel = "deferred" if case == "globes_deferred" else None
    elif case == "spinning_chain":
        text, t = scene_text("spinning_globes"), 0.35
    elif case == "fuzz_tree":
        text = random_scene(7773)
    else:
        text, W, H, kernel = scene_text("fractal"), 160, 120, "wavefront"
    osc = O.OracleScene(text, t, W, H, max_depth=depth)
    ref8 = osc.render(0, H)[1]
    r = T.Renderer(0, specialize=T.Renderer.LIBRARY_DEFAULT)
    r.upload(T.Scene.compile(text, t, W, H, asset_dir=SCENES))
    if kernel:
        r.set_kernel(kernel)
    r.spec_wait()
    for launch in ("calibration", "ordered", "ordered again"):
        if case == "globes_f64":
            got = r.render_rows_host(0, H, max_depth=depth, f64=True)
            ref64 = osc.render(0, H, f64=True)[0]
            assert np.array_equal(np.isnan(got), np.isnan(ref64))
            assert np.nanmax(np.abs(got - ref64)) <= 1e-9, f"{case} {launch} ({r.kernel_info()})"
        elif case == "globes_d5_bands":
            band, n = 8, H // 8
            slot = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
            r.render_row_bands(0, band, band, n, slot, max_depth=depth)
            torch.cuda.synchronize()
            assert np.array_equal(slot.cpu().numpy(), ref8), f"{case} {launch} ({r.kernel_info()})"
        else:
            got = r.render_rows_host(0, H, max_depth=depth)
            assert np.array_equal(got, ref8), f"{case} {launch}: {int((got != ref8).sum())} channels ({r.kernel_info()})"
    print(case, r.kernel_info())
