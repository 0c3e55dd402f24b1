"""The deferred-shadow path (rt_device.h trace_deferred: chain phase, wave-wide shadow
phase through an LDS window, post-order fold) on EVERY tile -- rt_ctx_set_option(RT_OPT_KERNEL,
RT_KERNEL_DEFERRED) -- against the oracle (src/raytracer/raytracer.rs:132-287): small frames (no
ordered launch, lanes outside the frame trace other lanes' shadow rays) and ordered frames whose
costliest tiles are split over several waves."""
import numpy as np
import pytest

from tests.conftest import SCENES, scene_text

pytestmark = pytest.mark.gpu

CASES = [("globes", 0.0, 64, 48, 10), ("globes", 0.25, 161, 121, 10), ("globes", 0.0, 640, 480, 10),
         ("globes", 0.5, 640, 480, 3), ("three_cubes", 0.0, 160, 120, 10), ("spinning_cube", 0.3, 160, 120, 10),
         ("ground_star", 0.2, 160, 120, 10), ("spinning_gimbals", 0.4, 160, 120, 10), ("fractal", 0.0, 96, 72, 10),
         # refraction chains (glass shells of reflectivity 0): the deferred kernel's REFR path
         ("spinning_globes", 0.3, 160, 120, 10), ("spinning_globes", 0.7, 640, 480, 10),
         ("spinning_globes", 0.05, 640, 480, 4)]


@pytest.mark.parametrize("name,t,W,H,d", CASES)
def test_every_tile_on_the_deferred_path(worldmap, name, t, W, H, d):
    import tinyraytracerinrust_amd as T
    from oracle import oracle as O
    rt = T.RayTracer(W, H)
    rt.max_depth = d
    rt.load_scene(scene_text(name), t, asset_dir=SCENES)
    rt.renderer.set_kernel("deferred")
    frames = [rt.renderer.render_rows_host(0, H) for _ in range(2)]     # calibration (if ordered), ordered
    f64 = rt.renderer.render_rows_host(0, H, f64=True)
    rf, ru = O.OracleScene(scene_text(name), t, W, H, max_depth=d).render(0, H, f64=True)
    for u in frames:
        assert np.array_equal(u, ru), (name, t, W, H, int((u != ru).sum()))
    assert np.nanmax(np.abs(f64 - rf)) <= 1e-9, name


def test_deferred_request_beyond_split_encoding_takes_megakernel():
    """The deferred kernel's order entries hold a tile index in 20 bits: a launch of more than 2^20
    tiles must fall back to the megakernel even when the deferred kernel is requested (same pixels)."""
    import torch
    import tinyraytracerinrust_amd as T
    W, H = 8200, 8200                                # 1025 x 1025 = 1 050 625 tiles > 2^20
    text = "draw(sphere(<0, 0, 0>, 30, red))"
    frames = {}
    for mode in ("mega", "deferred"):
        rt = T.RayTracer(W, H)
        rt.max_depth = 0
        rt.load_scene(text, 0.0)
        rt.renderer.set_kernel(mode)
        frames[mode] = rt.renderer.render_rows(0, H)
        torch.cuda.synchronize()
    assert torch.equal(frames["mega"], frames["deferred"])
    assert int((frames["mega"][..., 0] > 0).sum()) > 0


def test_kernel_option_same_pixels():
    """rt_ctx_set_option(RT_OPT_KERNEL): auto / megakernel / deferred give identical frames on one
    context, including after switching back and forth (tile orders are rebuilt per kernel)."""
    import tinyraytracerinrust_amd as T
    W, H = 640, 480                                  # >= 2048 tiles: ordered (and split) launches
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text("globes"), 0.25, asset_dir=SCENES)
    r = rt.renderer
    frames = {}
    for mode in ("auto", "mega", "deferred", "mega", "auto", "deferred"):
        r.set_kernel(mode)
        frames.setdefault(mode, []).extend(r.render_rows_host(0, H) for _ in range(2))
    ref = frames["auto"][0]
    for mode, fs in frames.items():
        for f in fs:
            assert np.array_equal(f, ref), mode
    from tinyraytracerinrust_amd import _lib
    with pytest.raises(T.RtError):
        _lib.check(T.lib().rt_ctx_set_option(r.h, 0, 7))


def test_timing_option():
    """rt_ctx_set_option(RT_OPT_TIMING): with the launch events off the frames are the same and
    rt_ctx_last_kernel_ms fails; turned back on, the next launch is timed again."""
    import tinyraytracerinrust_amd as T
    from tinyraytracerinrust_amd import _lib
    W, H = 320, 240
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text("globes"), 0.0, asset_dir=SCENES)
    r = rt.renderer
    ref = r.render_rows_host(0, H)
    assert r.last_kernel_ms() > 0.0
    r.set_timing(False)
    assert np.array_equal(r.render_rows_host(0, H), ref)
    with pytest.raises(T.RtError):
        r.last_kernel_ms()
    r.set_timing(True)
    assert np.array_equal(r.render_rows_host(0, H), ref)
    assert r.last_kernel_ms() > 0.0
    with pytest.raises(T.RtError):
        _lib.check(T.lib().rt_ctx_set_option(r.h, _lib.RT_OPT_TIMING, 2))
