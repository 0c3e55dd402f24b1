"""GPU parity of the adaptive anti-aliasing pass (rt_antialias) against the oracle's depth-first
restatement of antialiaser.rs (itself pinned bit-for-bit to oracle/pyref.py in test_oracle.py).

Both sides anti-alias the SAME quantised frame (the GPU render), so the test isolates the pass.
Bar: the same sub-pixel rays (the reference's ray_counter), f64 colours within 1e-9, RGBA8
bit-identical (the north star's 1-LSB bound is only reported)."""
import numpy as np
import pytest

from tests.conftest import SCENES, scene_text

pytestmark = pytest.mark.gpu

F64_TOL = 1e-9


@pytest.fixture(scope="module")
def T():
    import torch
    import tinyraytracerinrust_amd as T
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return T


def run_pair(T, name, time, W, H, threshold, level, depth=10):
    from oracle import oracle as O
    text = scene_text(name)
    rt = T.RayTracer(W, H)
    rt.max_depth = depth
    rt.load_scene(text, time, asset_dir=SCENES)
    frame = rt.renderer.render_rows_host(0, H)
    gf, grays = rt.renderer.antialias(frame, threshold, level, f64=True)
    gu, grays2 = rt.renderer.antialias(frame, threshold, level)
    ref = O.OracleScene(text, time, W, H, max_depth=depth)
    rf, ru, rrays = ref.antialias(frame, threshold, level)
    return frame, gf, gu, grays, grays2, rf, ru, rrays


CASES = [
    ("globes", 0.0, 160, 120, 0.01, 3),
    ("globes", 0.25, 96, 72, 0.01, 4),
    ("globes", 0.0, 64, 48, 0.0, 2),          # threshold 0: every non-flat pixel is an edge
    ("globes", 0.0, 64, 48, 0.1, 1),
    ("globes", 0.0, 64, 48, 0.01, 0),         # level 0: corner averages only, no rays
    ("spinning_globes", 0.3, 96, 72, 0.01, 3),   # refraction chains
    ("three_cubes", 0.0, 96, 72, 0.01, 3),
    ("fractal", 0.0, 64, 48, 0.01, 3),
]


@pytest.mark.parametrize("name,time,W,H,threshold,level", CASES)
def test_antialias_parity(T, worldmap, name, time, W, H, threshold, level):
    frame, gf, gu, grays, grays2, rf, ru, rrays = run_pair(T, name, time, W, H, threshold, level)
    print(f"{name} {W}x{H} th={threshold} level={level}: rays gpu={grays} oracle={rrays}")
    assert grays == rrays == grays2
    if level == 0:
        assert grays == 0
    fd = np.abs(gf - rf)
    assert fd.max() <= F64_TOL, f"f64 max |d| {fd.max():.3e}"
    d = np.abs(gu.astype(np.int16) - ru.astype(np.int16))
    print(f"aa: max|d| {d.max()} exact {100 * np.mean(d == 0):.4f}%")
    assert np.array_equal(gu, ru)
    assert np.array_equal(gu[-1], frame[-1]) and np.array_equal(gu[:, -1], frame[:, -1])


def test_antialias_device_tensors_and_mirror(T, worldmap):
    """Device-tensor path == host path; the AntiAliaser mirror accumulates ray_counter."""
    import torch
    W, H = 128, 96
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text("globes"), 0.0, asset_dir=SCENES)
    dev = rt.renderer.render_rows(0, H)
    out, rays = rt.renderer.antialias(dev, 0.01, 3)
    torch.cuda.synchronize()
    host, hrays = rt.renderer.antialias(dev.cpu().numpy(), 0.01, 3)
    assert out.is_cuda and np.array_equal(out.cpu().numpy(), host) and rays == hrays > 0
    src = dev.cpu().numpy()
    aa = T.AntiAliaser(rt, 0.01, 3)
    a1 = aa.anti_alias_frame(src)
    a2 = aa.anti_alias_frame(src)
    assert aa.ray_counter == 2 * rays
    assert np.array_equal(a1, host) and np.array_equal(a2, host)   # deterministic
    with pytest.raises(T.RtError):
        rt.renderer.antialias(host, 0.01, 5)   # level > 4 unsupported


def test_antialias_640x480(T, worldmap):
    """BASELINE config 1's size, full-frame compare."""
    frame, gf, gu, grays, _, rf, ru, rrays = run_pair(T, "globes", 0.0, 640, 480, 0.01, 3)
    assert grays == rrays
    assert np.abs(gf - rf).max() <= F64_TOL


ORTHO = [("top", (0, 2, 1.0, -1.0)), ("front", (0, 1, 1.0, -1.0)), ("side", (2, 1, -1.0, -1.0))]


@pytest.mark.parametrize("name,time,W,H", [("globes", 0.0, 160, 120), ("three_cubes", 0.0, 128, 96),
                                           ("spinning_gimbals", 0.4, 128, 96), ("fractal", 0.0, 96, 72),
                                           ("ground_star", 0.2, 128, 96)])
def test_ortho_views_parity(T, worldmap, name, time, W, H):
    """Orthogonal previews (debug_window.rs:166-227) against the oracle: bit-exact (no libm)."""
    from oracle import oracle as O
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text(name), time, asset_dir=SCENES)
    ref = O.OracleScene(scene_text(name), time, W, H)
    for area, axes in ORTHO:
        rf, ru = ref.render_ortho(*axes, scale=T.ORTHO_SCALE)
        gf = rt.renderer.render_ortho(T.OrthoAxes.from_area(area), f64=True)
        gu = rt.render_orthogonal_view(area)
        assert np.array_equal(gf, rf), f"{name} {area}: f64 differs"
        assert np.array_equal(gu, ru)
    line = rt.render_orthogonal_view_line(H // 2, T.OrthoAxes.from_area("front"))
    assert np.array_equal(line, ref.render_ortho(0, 1, 1.0, -1.0, 2.0, H // 2, H // 2 + 1)[0][0])
    with pytest.raises(T.RtError):
        rt.renderer.render_ortho(T.OrthoAxes(0, 3, 1.0, 1.0))   # axis out of range


@pytest.mark.parametrize("name,time,W,H,pts", [
    ("globes", 0.0, 160, 120, [(80, 60), (80, 100), (20, 110), (75.5, 40.25), (3, 3)]),
    ("spinning_globes", 0.3, 96, 72, [(48, 36), (40, 30), (60.125, 33.5)]),
    ("three_cubes", 0.0, 96, 72, [(48, 36), (30, 50)]),
])
def test_ray_debugger_records(T, worldmap, name, time, W, H, pts):
    """RayDebugger::record_rays (ray_debugger.rs:92-137): the GPU recorder's rays, in callback order,
    equal the oracle's -- rays, distances, hit objects, raw normals; colours within 1e-9."""
    from oracle import oracle as O
    assert T.RAY_RECORD_DTYPE.itemsize == O.OracleScene(scene_text(name), time, W, H).lib.orc_ray_record_size()
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text(name), time, asset_dir=SCENES)
    ref = O.OracleScene(scene_text(name), time, W, H)
    for x, y in pts:
        got, rgba = rt.renderer.record_rays(x, y)
        raw, ref_rgba = ref.record_rays(x, y)
        want = np.frombuffer(raw.tobytes(), T.RAY_RECORD_DTYPE)
        assert len(got) == len(want) >= 1, (x, y)
        for f in ("depth", "ray_type", "object", "intersected", "has_normal", "point", "direction", "distance",
                  "intersection", "normal"):
            assert np.array_equal(got[f], want[f]), (x, y, f)
        assert np.abs(got["color"] - want["color"]).max() <= 1e-9
        assert np.abs(rgba - ref_rgba).max() <= 1e-9
        assert np.array_equal(rgba, got["color"][-1])          # the primary ray reports last
    dbg = T.RayDebugger(W, H)
    dbg.record_rays(rt, *pts[0])
    n = len(dbg.rays)
    dbg.record_rays(rt, *pts[0])                                # same position: kept, not re-recorded
    assert len(dbg.rays) == n
