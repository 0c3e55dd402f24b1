"""Parity fuzzing: seeded random scenes (tests/scene_fuzz.py) compiled by the PRODUCT's
rt_scene_compile and rendered by the HIP kernels, against the oracle's own parse and render of the
same text (src/raytracer/raytracer.rs:132-287 and its callees).  Small frames go through the
one-launch path; larger ones through the calibration launch and the cost-ordered launch that
follows it (and, for tail-bound launches of scenes without a transparent object, the
deferred-shadow kernel with split tiles).  Bar: RGBA8 bit-identical (test_gpu_parity.assert_close;
the north star's 1-LSB bound is only reported), f64 colours within 1e-9."""
import numpy as np
import pytest

from tests.scene_fuzz import random_rod_scene, random_scene
from tests.test_gpu_parity import assert_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def T():
    import torch
    import tinyraytracerinrust_amd as T
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return T


@pytest.mark.parametrize("seed", range(160))
def test_random_scene_small_frame(T, seed):
    from oracle import oracle as O
    text = random_scene(seed)
    W, H, d = 96, 72, 6
    rt = T.RayTracer(W, H)
    rt.max_depth = d
    rt.load_scene(text, 0.0)
    gu = rt.renderer.render_rows_host(0, H)
    gf = rt.renderer.render_rows_host(0, H, f64=True)
    rf, ru = O.OracleScene(text, 0.0, W, H, max_depth=d).render(0, H, f64=True)
    assert_close(gu, gf, ru, rf, f"random scene {seed}")


@pytest.mark.parametrize("seed", range(1000, 1012))
def test_random_scene_ordered_launches(T, seed):
    """512x384 = 3072 tiles: the first launch calibrates the tile order, the next ones use it."""
    from oracle import oracle as O
    text = random_scene(seed)
    W, H, d = 512, 384, 10
    rt = T.RayTracer(W, H)
    rt.max_depth = d
    rt.load_scene(text, 0.0)
    frames = [rt.renderer.render_rows_host(0, H) for _ in range(3)]
    _, ru = O.OracleScene(text, 0.0, W, H, max_depth=d).render(0, H)
    for k, f in enumerate(frames):
        assert_close(f, None, ru, None, f"random scene {seed}, launch {k}")
    assert np.array_equal(frames[1], frames[2])


@pytest.mark.parametrize("seed", range(3000, 3048))
def test_random_chain_scene_small_frame(T, seed):
    """Scenes whose transparent objects are not reflective (ray chains): small frames take the
    deferred kernel's refraction-chain path (no calibration below 2048 tiles)."""
    from oracle import oracle as O
    text = random_scene(seed, chains=True)
    W, H, d = 96, 72, 6
    rt = T.RayTracer(W, H)
    rt.max_depth = d
    rt.load_scene(text, 0.0)
    gu = rt.renderer.render_rows_host(0, H)
    gf = rt.renderer.render_rows_host(0, H, f64=True)
    rf, ru = O.OracleScene(text, 0.0, W, H, max_depth=d).render(0, H, f64=True)
    assert_close(gu, gf, ru, rf, f"random chain scene {seed}")


@pytest.mark.parametrize("seed", range(4000, 4012))
@pytest.mark.parametrize("kernel", ["mega", "deferred", "auto"])
def test_random_chain_scene_ordered_launches(T, seed, kernel):
    """Ray-chain scenes at 512x384 (3072 tiles) through the calibration launch and the cost-ordered
    launches: the refraction chain megakernel (RT_MODE_CHAIN) and the deferred kernel's REFR path with
    its costliest tiles split over several waves."""
    from oracle import oracle as O
    text = random_scene(seed, chains=True)
    W, H, d = 512, 384, 10
    rt = T.RayTracer(W, H)
    rt.max_depth = d
    rt.load_scene(text, 0.0)
    rt.renderer.set_kernel(kernel)
    frames = [rt.renderer.render_rows_host(0, H) for _ in range(3)]
    _, ru = O.OracleScene(text, 0.0, W, H, max_depth=d).render(0, H)
    for k, f in enumerate(frames):
        assert_close(f, None, ru, None, f"random chain scene {seed} {kernel}, launch {k}")


@pytest.mark.parametrize("seed", range(2000, 2024))
def test_random_scene_antialias(T, seed):
    """The adaptive anti-aliasing pass (rt_antialias, antialiaser.rs:87-191) on random scenes:
    the same sub-pixel rays as the oracle's depth-first pass, f64 within 1e-9, RGBA8 exact."""
    from oracle import oracle as O
    text = random_scene(seed)
    W, H, d = 64, 48, 6
    rt = T.RayTracer(W, H)
    rt.max_depth = d
    rt.load_scene(text, 0.0)
    frame = rt.renderer.render_rows_host(0, H)
    level = 1 + seed % 4
    gf, grays = rt.renderer.antialias(frame, 0.01, level, f64=True)
    gu, _ = rt.renderer.antialias(frame, 0.01, level)
    rf, ru, rrays = O.OracleScene(text, 0.0, W, H, max_depth=d).antialias(frame, 0.01, level)
    assert grays == rrays
    assert np.abs(gf - rf).max() <= 1e-9
    assert np.array_equal(gu, ru), int((gu != ru).sum())


@pytest.mark.parametrize("seed", range(3000, 3048))
def test_rod_scene_small_frame(T, seed):
    """Thin rotated rods and slabs (tests/scene_fuzz.py random_rod_scene): objects the kernels
    cull with oriented boxes in a leaf's own frame (scene.cpp obb) -- exactness of that culling."""
    from oracle import oracle as O
    text = random_rod_scene(seed)
    W, H, d = 128, 96, 8
    rt = T.RayTracer(W, H)
    rt.max_depth = d
    rt.load_scene(text, 0.0)
    gu = rt.renderer.render_rows_host(0, H)
    gf = rt.renderer.render_rows_host(0, H, f64=True)
    rf, ru = O.OracleScene(text, 0.0, W, H, max_depth=d).render(0, H, f64=True)
    assert_close(gu, gf, ru, rf, f"rod scene {seed}")


@pytest.mark.parametrize("seed", range(3100, 3106))
def test_rod_scene_ordered_launches(T, seed):
    """640x480: calibration, cost-ordered megakernel and (4800 tiles, tail-bound) deferred-shadow
    launches over rod scenes: the oriented boxes in every traversal, shadow jobs included."""
    from oracle import oracle as O
    text = random_rod_scene(seed)
    W, H, d = 640, 480, 10
    rt = T.RayTracer(W, H)
    rt.max_depth = d
    rt.load_scene(text, 0.0)
    frames = [rt.renderer.render_rows_host(0, H) for _ in range(3)]
    _, ru = O.OracleScene(text, 0.0, W, H, max_depth=d).render(0, H)
    for k, f in enumerate(frames):
        assert_close(f, None, ru, None, f"rod scene {seed}, launch {k}")


_TIE_SCENES = [
    # the same sphere drawn twice in two colours, the larger object listed second: every hit is a tie
    "draw(plane(<0, 1, 0>, 20, white * 0.5, 0.3))\n"
    "draw(sphere(<0, 0, 0>, 12, red, 0.4))\ndraw(sphere(<0, 0, 0>, 12, blue, 0.4))\n"
    "draw(sphere(<-14, 4, -3>, 30, rgb(0.2, 0.8, 0.2)))\nset camera(<0, 10, -90>)\n",
    # a small cube whose front face lies in a big cube's front face; the big cube listed first
    "draw(plane(<0, 1, 0>, 25, red * 0.5, 0.5))\n"
    "draw(cube(<0, 0, 0>, 40, rgb(0.7, 0.7, 0.2), 0.2))\ndraw(cube(<0, 0, -10>, 20, blue, 0.2))\n"
    "set camera(<5, 12, -95>)\n",
    # rotated duplicates (one object through a CSG union with itself) and a shared tilted plane
    "rotate(0.3, 0.5, 0.1) do\n  a = sphere(<3, 0, 0>, 10)\n  draw(csg(a, a, 'union', red, 0.5))\n"
    "  draw(sphere(<3, 0, 0>, 10, white, 0.5))\nend\n"
    "draw(plane(<0.2, 1, 0.1>, 22, blue * 0.6, 0.4))\ndraw(plane(<0.2, 1, 0.1>, 22, red * 0.6, 0.4))\n",
]


@pytest.mark.parametrize("k", range(len(_TIE_SCENES)))
def test_nearest_hit_ties_follow_draw_order(T, k):
    """Objects with coincident surfaces: the reference keeps the first object in draw order that
    reaches the nearest distance (raytracer.rs:141-150); the reflection-only kernels visit objects
    largest-first and resolve equal distances by draw order -- every pixel as the oracle's."""
    from oracle import oracle as O
    text = _TIE_SCENES[k]
    W, H, d = 160, 120, 6
    rt = T.RayTracer(W, H)
    rt.max_depth = d
    rt.load_scene(text, 0.0)
    gu = rt.renderer.render_rows_host(0, H)
    gf = rt.renderer.render_rows_host(0, H, f64=True)
    rf, ru = O.OracleScene(text, 0.0, W, H, max_depth=d).render(0, H, f64=True)
    assert_close(gu, gf, ru, rf, f"tie scene {k}")
    assert np.array_equal(gu, ru)
