"""GPU parity: the HIP render path (through the C ABI) against the CPU oracle.

Bar: the RGBA8 frames are BIT-IDENTICAL to the oracle's (np.array_equal).  The north star allows
1 LSB per channel; that bound is kept only as a reported statistic (max |delta| and the exact
fraction are printed), so a single one-LSB regression fails the test.  The f64 colours agree to
1e-9 (acos/sin may differ from glibc by 1 ulp on the device, DESIGN.md "Parity").
"""
import numpy as np
import pytest

from tests.conftest import SCENES, scene_text

pytestmark = pytest.mark.gpu

U8_TOL = 1            # LSB per channel: the north star's bound, reported, not asserted
F64_TOL = 1e-9        # absolute, pre-quantisation colours in [0, 1]


@pytest.fixture(scope="module")
def T():
    import torch
    import tinyraytracerinrust_amd as T
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    assert T.device_count() >= 1
    return T


def render_pair(T, text, time, W, H, max_depth=10, f64=True, rows=None):
    from oracle import oracle as O
    y0, y1 = rows if rows else (0, H)
    rt = T.RayTracer(W, H)
    rt.max_depth = max_depth
    rt.load_scene(text, time, asset_dir=SCENES)
    r = rt.renderer
    gpu_u8 = r.render_rows_host(y0, y1)
    gpu_f = r.render_rows_host(y0, y1, f64=True) if f64 else None
    ref = O.OracleScene(text, time, W, H, max_depth=max_depth)
    ref_f, ref_u8 = ref.render(y0, y1, f64=f64)
    return gpu_u8, gpu_f, ref_u8, ref_f


def assert_close(gpu_u8, gpu_f, ref_u8, ref_f, label):
    d = np.abs(gpu_u8.astype(np.int16) - ref_u8.astype(np.int16))
    exact = float(np.mean(d == 0))
    print(f"{label}: u8 max|d|={d.max()} (north-star bound {U8_TOL}) exact={100 * exact:.4f}%")
    assert np.array_equal(gpu_u8, ref_u8), \
        f"{label}: {int((d > 0).sum())} channels differ (max {d.max()} LSB, {int((d > U8_TOL).sum())} beyond {U8_TOL})"
    if gpu_f is not None:
        fd = np.abs(gpu_f - ref_f)
        print(f"{label}: f64 max|d|={fd.max():.3e} bit-equal={100 * np.mean(gpu_f == ref_f):.4f}%")
        assert np.nanmax(fd) <= F64_TOL
        assert np.array_equal(np.isnan(gpu_f), np.isnan(ref_f))


CASES = [
    ("globes", 0.0, 64, 48, 10),
    ("globes", 0.25, 160, 120, 10),
    ("globes", 0.5, 160, 120, 10),
    ("globes", 0.0, 320, 240, 5),
    ("spinning_globes", 0.1, 160, 120, 10),
    ("spinning_globes", 0.5, 96, 72, 10),
    ("three_cubes", 0.0, 160, 120, 10),
    ("spinning_cube", 0.3, 160, 120, 10),
    ("ground_star", 0.2, 160, 120, 10),
    ("spinning_gimbals", 0.4, 160, 120, 10),
    ("fractal", 0.0, 96, 72, 10),
]


@pytest.mark.parametrize("name,time,W,H,depth", CASES)
def test_scene_parity(T, worldmap, name, time, W, H, depth):
    gu, gf, ru, rf = render_pair(T, scene_text(name), time, W, H, depth)
    assert_close(gu, gf, ru, rf, f"{name} t={time} {W}x{H} d={depth}")


EDGE_SCENES = {
    # a wall beyond the culling range (|coords| > 1e6): boxes never culled, never grouped
    "huge_wall": "draw(sphere(<0, 0, 2000000>, 1999000, red * 0.8, 0.3))\n"
                 "draw(sphere(<0, 0, 0>, 20, red, 0.5))\ndraw(cube(<25, -10, 0>, 10, red * 0.5, 0.2))",
    # translation-only inverses with -0 entries: the diagonal-affine transform short form
    # materials outside [0, 1] (negative colour, reflectivity > 1, transparency > 1): the kernels
    # must keep the compare/select clamps here (RtDevScene::colour_fast = 0)
    "odd_materials": "draw(sphere(<0, 0, 0>, 25, red * (0 - 0.5), 1.3))\n"   # (-0.5, -0, -0), refl 1.3
                     "draw(plane(<0, 1, 0>, 20, rgb(0.3, 0.3, 0.9), 0.5))\n"
                     "draw(sphere(<30, 0, -10>, 12, rgb(0.8, 0.8, 0.1), 0.2, 1.2))",
    "signed_zero_xf": "translate(0, 5, 0) draw(sphere(<0, 0, 0>, 30, red, 0.3))\n"
                      "translate(0, -30, 0) draw(cube(<0, 0, 0>, 20, red * 0.5, 0.5))\n"
                      "scale(1, 0.5, 1) draw(sphere(<30, 0, 0>, 10, red * 0.2, 0.4, 0.5))",
    # concentric sphere leaves under one transform (RtLeaf::share_prev: a chain of three in a
    # transparent object, so the refraction kernel's shared terms run), concentric spheres under
    # DIFFERENT transforms (no sharing), and planes along x, tilted, and rotated (only the
    # untransformed axis-aligned ones take RtLeaf::plane_axis)
    "shared_spheres_planes": (
        'rotate(0.2, 0.5, 0) do\n'
        '  a = sphere(<-10, 0, 0>, 15)\n'
        '  b = sphere(<-10, 0, 0>, 13)\n'
        '  c = sphere(<-10, 0, 0>, 11)\n'
        "  draw(csg(csg(a, b, 'difference'), c, 'union', rgb(0.9, 0.4, 0.2), 0.3, 0.6))\n"
        'end\n'
        'rotate(0, 0.7, 0) do\n'
        '  d = sphere(<20, 5, 0>, 9)\n'
        'end\n'
        'e = sphere(<20, 5, 0>, 7)\n'
        "draw(csg(d, e, 'difference', rgb(0.2, 0.8, 0.9), 0.4, 0.5))\n"
        'draw(plane(<1, 0, 0>, 45, rgb(0.2, 0.6, 0.2), 0.3))\n'
        'draw(plane(<0, 0, -1>, 80, rgb(0.7, 0.7, 0.7), 0.2))\n'
        'draw(plane(<0.3, 1, 0>, 30, rgb(0.6, 0.6, 0.3), 0.3))\n'
        'rotate(0.3, 0, 0) do\n'
        '  draw(plane(<0, 1, 0>, 60, rgb(0.5, 0.1, 0.6), 0.4))\n'
        'end\n'
        'set camera(<0, 10, -85>)\n'
    ),
}


@pytest.mark.parametrize("name", sorted(EDGE_SCENES))
def test_edge_scene_parity(T, name):
    gu, gf, ru, rf = render_pair(T, EDGE_SCENES[name], 0.0, 160, 120, 10)
    assert_close(gu, gf, ru, rf, name)


def test_single_sphere_primary_only(T):
    """BASELINE config 2 at reduced size: draw(sphere(<0,0,0>, 30, red)), max_depth 0."""
    text = "draw(sphere(<0, 0, 0>, 30, red))"
    gu, gf, ru, rf = render_pair(T, text, 0.0, 192, 108, max_depth=0)
    assert_close(gu, gf, ru, rf, "sphere d=0")


def test_builder_api_matches_dsl(T):
    """The Rust host's path (shape/material calls, no DSL) gives the same frame as the DSL."""
    W, H = 128, 96
    rt = T.RayTracer(W, H)
    rt.add_test_objects()
    s = rt.sphere((0, 0, 0), 30)
    rt.add_object(s, T.solid_material((1, 0, 0, 1)))
    a = rt.sphere((-15, -5, -10), 30)
    b = rt.sphere((-15, -5, -10), 25)
    rt.add_object(rt.csg(a, b, "difference"), T.solid_material((0, 1, 1, 1), 0.0, 0.8))
    gpu = rt.render_frame()
    dsl = T.RayTracer(W, H)
    dsl.load_scene("draw(sphere(<0,0,0>, 30, red))\n"
                   "a = sphere(<-15, -5, -10>, 30)\nb = sphere(<-15, -5, -10>, 25)\n"
                   "draw(csg(a, b, 'difference', rgb(0.0, 1.0, 1.0), 0.0, 0.8))\n", 0.0)
    assert np.array_equal(gpu, dsl.render_frame())


def test_row_tiles_compose(T):
    """Rows [y0, y1) use the full-frame camera: tiles concatenate to the full frame bit-exactly."""
    W, H = 200, 150
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text("globes"), 0.0, asset_dir=SCENES)
    r = rt.renderer
    full = r.render_rows_host(0, H)
    cuts = [0, 1, 17, 64, 65, 149, 150]
    tiles = np.concatenate([r.render_rows_host(a, b) for a, b in zip(cuts[:-1], cuts[1:])])
    assert np.array_equal(full, tiles)
    again = r.render_rows_host(0, H)
    assert np.array_equal(full, again), "render is not deterministic"


def test_points_match_rows(T):
    W, H = 64, 48
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text("globes"), 0.0, asset_dir=SCENES)
    rows = rt.renderer.render_rows_host(0, H, f64=True)
    ys, xs = np.mgrid[0:H, 0:W]
    pts = np.stack([xs.ravel(), ys.ravel()], 1).astype(np.float64)
    out = rt.renderer.render_points(pts)
    assert np.array_equal(out.reshape(H, W, 4), rows)
    # fractional positions (the anti-aliaser's sub-pixels) against the oracle's get_pixel
    from oracle import oracle as O
    ref = O.OracleScene(scene_text("globes"), 0.0, W, H)
    sub = np.array([[10 + 1 / 9, 20 + 5 / 9], [33.5, 7.25], [0.0, 47.875]])
    got = rt.renderer.render_points(sub)
    want = np.stack([ref.get_pixel(x, y) for x, y in sub])
    assert np.max(np.abs(got - want)) <= F64_TOL


def test_trace_pixel_without_context(T):
    """rt_trace_pixel_f64 (SURVEY 8(b)'s scene-level get_pixel): the same doubles as the context's
    points launch and the oracle's get_pixel, and an edited-then-recompiled scene is seen."""
    from oracle import oracle as O
    from tinyraytracerinrust_amd import raytracer as R
    W, H = 64, 48
    text = scene_text("globes")
    sc = R.Scene.compile(text, 0.0, W, H, asset_dir=SCENES)
    rt = T.RayTracer(W, H)
    rt.load_scene(text, 0.0, asset_dir=SCENES)
    ref = O.OracleScene(text, 0.0, W, H)
    for x, y in [(10 + 1 / 9, 20 + 5 / 9), (33.5, 7.25), (0.0, 47.875), (31.0, 30.0)]:
        got = sc.trace_pixel(x, y)
        assert np.array_equal(got, rt.renderer.render_points(np.array([[x, y]]))[0])
        assert np.max(np.abs(got - ref.get_pixel(x, y))) <= F64_TOL
    sc2 = R.Scene.compile("draw(sphere(<0, 0, 0>, 30, red))", 0.0, W, H)
    assert not np.array_equal(sc2.trace_pixel(31.0, 30.0), sc.trace_pixel(31.0, 30.0))


def test_device_output_and_torch_stream(T):
    import torch
    W, H = 96, 64
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text("globes"), 0.0, asset_dir=SCENES)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        out = rt.renderer.render_rows(0, H, stream=s)
    s.synchronize()
    assert out.is_cuda and out.shape == (H, W, 4)
    assert np.array_equal(out.cpu().numpy(), rt.renderer.render_rows_host(0, H))


def test_4k_globes_sampled_rows(T, worldmap):
    """Full BASELINE size (3840x2160, depth 10): render on the GPU, check a stratified sample of
    rows against the oracle, and size-independent properties (alpha, determinism)."""
    import torch
    from oracle import oracle as O
    W, H = 3840, 2160
    text = scene_text("globes")
    rt = T.RayTracer(W, H)
    rt.load_scene(text, 0.0, asset_dir=SCENES)
    frame = rt.renderer.render_rows(0, H)
    torch.cuda.synchronize()
    frame = frame.cpu().numpy()
    assert (frame[..., 3] == 255).all()
    ref = O.OracleScene(text, 0.0, W, H)
    step = 97
    _, ref_u8 = ref.render(0, H, row_step=step)
    got = frame[0:H:step]
    assert_close(got, None, ref_u8, None, "4K globes sampled rows")
    again = rt.renderer.render_rows(0, H).cpu().numpy()
    assert np.array_equal(frame, again)


@pytest.mark.parametrize("world,layout,band", [(2, "contiguous", 0), (3, "cyclic", 8), (8, "cyclic", 8),
                                               (8, "contiguous", 0), (5, "cyclic", 16)])
def test_row_bands_assemble_like_ranks(T, world, layout, band):
    """What each rank of the multi-GPU path does (rt_render_row_bands into its slot of the
    gather buffer) followed by the assembly, simulated on one GPU: equals the plain frame."""
    import torch
    from tinyraytracerinrust_amd import distributed as D
    W, H = 200, 150
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text("globes"), 0.0, asset_dir=SCENES)
    r = rt.renderer
    full = r.render_rows_host(0, H)
    band = band or -(-H // world)
    slot_rows = D.rows_per_rank(H, world, layout, band)
    gath = torch.zeros((world * slot_rows, W, 4), dtype=torch.uint8, device="cuda")
    for rank in range(world):
        y_first, band_rows, pitch, n_bands = D.band_params(H, world, rank, layout, band)
        r.render_row_bands(y_first, band_rows, pitch, n_bands, gath[rank * slot_rows:(rank + 1) * slot_rows])
    frame = D.assemble(gath, H, world, layout, band)                     # rt_assemble_row_bands
    ref = D.assemble_reference(gath, H, world, layout, band)             # torch restatement
    into = D.assemble(gath, H, world, layout, band, out=torch.empty_like(ref))
    torch.cuda.synchronize()
    assert np.array_equal(frame.cpu().numpy(), full)
    assert np.array_equal(ref.cpu().numpy(), full)
    assert np.array_equal(into.cpu().numpy(), full)


@pytest.mark.parametrize("W,world,band", [(3840, 8, 8), (33, 3, 5), (7, 2, 1)])
def test_assemble_row_bands_kernel(T, W, world, band):
    """rt_assemble_row_bands on random bytes against the torch permutation, including row lengths
    that are not a multiple of 16 bytes (byte-copy path) and strided (padded) rows."""
    import torch
    from tinyraytracerinrust_amd import distributed as D
    H = 2160 if W == 3840 else 61
    slot_rows = D.rows_per_rank(H, world, "cyclic", band)
    g = torch.randint(0, 256, (world * slot_rows, W, 4), dtype=torch.uint8, device="cuda")
    want = D.assemble_reference(g, H, world, "cyclic", band).cpu()
    got = D.assemble(g, H, world, "cyclic", band).cpu()
    assert torch.equal(got, want)
    padded = torch.zeros((H, W + 3, 4), dtype=torch.uint8, device="cuda")[:, :W]   # row stride > row bytes
    D._assemble_device(g, H, world, slot_rows, band, out=padded)
    assert torch.equal(padded.cpu(), want)
    with pytest.raises(T.RtError):                                      # slot too small for the layout
        D._assemble_device(g[: world * (slot_rows - band)], H, world, slot_rows - band, band)


@pytest.mark.parametrize("scene,time,W,H,depth", [("globes", 0.25, 160, 120, 10),
                                                   ("spinning_globes", 0.1, 160, 120, 10)])
def test_cost_ordered_dispatch_parity(T, scene, time, W, H, depth):
    """The first launch of a geometry on a context records every tile's wave time (row-major
    dispatch); later launches dispatch the tiles longest-first (DESIGN.md "Tile order").  Every
    launch must give the oracle's bits."""
    from oracle import oracle as O
    rt = T.RayTracer(W, H)
    rt.max_depth = depth
    rt.load_scene(scene_text(scene), time, asset_dir=SCENES)
    r = rt.renderer
    u8 = [r.render_rows_host(0, H) for _ in range(3)]          # calibrate, then ordered twice
    f = [r.render_rows_host(0, H, f64=True) for _ in range(2)]
    assert np.array_equal(u8[0], u8[1]) and np.array_equal(u8[1], u8[2])
    assert np.array_equal(f[0], f[1], equal_nan=True)
    ref_f, ref_u8 = O.OracleScene(scene_text(scene), time, W, H, max_depth=depth).render(0, H, f64=True)
    assert_close(u8[2], f[1], ref_u8, ref_f, f"{scene} t={time} ordered")
    # a new scene on the same context measures again
    rt.load_scene(scene_text(scene), time + 0.125, asset_dir=SCENES)
    a, b = rt.renderer.render_rows_host(0, H), rt.renderer.render_rows_host(0, H)
    assert np.array_equal(a, b)


def test_tile_orders_of_interleaved_geometries_on_two_streams(T):
    """Launches of different row geometries queued on two streams of one context, with new
    geometries calibrated while earlier launches are still queued: every frame must equal the
    synchronous render (an order table is never rewritten while a launch may read it)."""
    import torch
    W, H = 640, 480                                  # 4800 tiles: cost-ordered dispatch is on
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text("globes"), 0.0, asset_dir=SCENES)
    r = rt.renderer
    geoms = [(0, H, 10), (0, H, 5), (0, H - 8, 10), (8, H, 4)]
    want = {g: r.render_rows_host(g[0], g[1], max_depth=g[2]) for g in geoms}
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    rt2 = T.RayTracer(W, H)                         # a fresh context: every geometry calibrates here
    rt2.load_scene(scene_text("globes"), 0.0, asset_dir=SCENES)
    r2 = rt2.renderer
    outs = []
    for it in range(3):
        for k, g in enumerate(geoms):
            s = s1 if (k + it) % 2 == 0 else s2
            outs.append((g, r2.render_rows(g[0], g[1], max_depth=g[2], stream=s)))
    torch.cuda.synchronize()
    for g, o in outs:
        assert np.array_equal(o.cpu().numpy(), want[g]), f"geometry {g}"


@pytest.mark.parametrize("world,layout,band", [(3, "cyclic", 8), (8, "contiguous", 0), (5, "cyclic", 16)])
def test_rgb8_row_bands_assemble_like_ranks(T, world, layout, band):
    """The multi-GPU path with packed RGB8 slots (rt_render_row_bands_rgb8, the all-gather moves 3
    bytes per pixel) assembled into RGBA8 (rt_assemble_row_bands_rgb8): equals the plain frame."""
    import torch
    from tinyraytracerinrust_amd import distributed as D
    W, H = 203, 150                                  # odd width: the RGB rows are not 4-byte multiples
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text("globes"), 0.25, asset_dir=SCENES)
    r = rt.renderer
    full = r.render_rows_host(0, H)
    band = band or -(-H // world)
    slot_rows = D.rows_per_rank(H, world, layout, band)
    gath = torch.zeros((world * slot_rows, W, 3), dtype=torch.uint8, device="cuda")
    for rank in range(world):
        y_first, band_rows, pitch, n_bands = D.band_params(H, world, rank, layout, band)
        r.render_row_bands(y_first, band_rows, pitch, n_bands, gath[rank * slot_rows:(rank + 1) * slot_rows])
    frame = D.assemble(gath, H, world, layout, band)                     # rt_assemble_row_bands_rgb8
    ref = D.assemble_reference(gath, H, world, layout, band)             # torch restatement
    torch.cuda.synchronize()
    assert np.array_equal(frame.cpu().numpy(), full)
    assert np.array_equal(ref.cpu().numpy(), full)


def test_assemble_rgb8_kernel_random(T):
    import torch
    from tinyraytracerinrust_amd import distributed as D
    # 3840 / 1924: the 4-pixel (12-byte load, 16-byte store) path; 33 / 1922: one pixel per thread
    for W, H, world, band in [(3840, 2160, 8, 8), (33, 61, 3, 5), (1924, 100, 8, 8), (1922, 64, 2, 8)]:
        slot_rows = D.rows_per_rank(H, world, "cyclic", band)
        g = torch.randint(0, 256, (world * slot_rows, W, 3), dtype=torch.uint8, device="cuda")
        want = D.assemble_reference(g, H, world, "cyclic", band).cpu()
        got = D.assemble(g, H, world, "cyclic", band).cpu()
        assert torch.equal(got, want)
        assert (got[..., 3] == 255).all()


def test_own_queue_streams_overlapping_frames(T):
    """Frames rendered concurrently on streams with their own hardware queue (rt_stream_create /
    HwStream, as bench.py's frames in flight) equal the synchronous render, including the
    ordered launches that follow the calibration."""
    import torch
    W, H = 640, 480
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text("globes"), 0.1, asset_dir=SCENES)
    r = rt.renderer
    want = r.render_rows(0, H)
    torch.cuda.synchronize()
    hs = [T.HwStream(0) for _ in range(4)]
    outs = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(8)]
    r.set_kernel("mega")
    for i, o in enumerate(outs):
        r.render_rows(0, H, out=o, stream=hs[i % 4].torch)
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, want)
    for h in hs:
        h.close()
    from tinyraytracerinrust_amd import _lib
    with pytest.raises(T.RtError):
        _lib.check(T.lib().rt_stream_destroy(None))
