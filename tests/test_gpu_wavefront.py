"""The launch-wide wavefront path (k_wavefront.hip wf_trace_kernel / wf_fold_kernel /
wf_fixup_kernel; rt_ctx_set_option(RT_OPT_KERNEL, RT_KERNEL_WAVEFRONT)): one pass per recursion
depth over a dense queue of that depth's rays, then the bottom-up fold of raytracer.rs:256-279.
Every frame against the oracle (src/raytracer/raytracer.rs:132-287): reflection chains, refraction
chains, ray trees (fractal.scene's glass spheres are transparent AND reflective), row bands as the
multi-GPU ranks render them, and pixels whose trees overflow a level (RT_OPT_WAVEFRONT_CAP at 1 %:
the fix-up kernel re-renders them)."""
import numpy as np
import pytest

from tests.conftest import SCENES, scene_text
from tests.test_gpu_parity import assert_close

pytestmark = pytest.mark.gpu

CASES = [("globes", 0.0, 160, 120, 10), ("globes", 0.25, 640, 480, 10), ("globes", 0.0, 320, 240, 3),
         ("spinning_globes", 0.3, 320, 240, 10), ("spinning_globes", 0.7, 160, 120, 4),
         ("three_cubes", 0.0, 160, 120, 10), ("spinning_cube", 0.3, 160, 120, 10), ("ground_star", 0.2, 160, 120, 10),
         ("spinning_gimbals", 0.4, 160, 120, 10), ("fractal", 0.0, 160, 120, 10), ("fractal", 0.0, 96, 72, 2)]


def _render(text, t, W, H, d, cap=None, rows=None, pairs=None):
    import tinyraytracerinrust_amd as T
    rt = T.RayTracer(W, H)
    rt.max_depth = d
    rt.load_scene(text, t, asset_dir=SCENES)
    r = rt.renderer
    r.set_kernel("wavefront")
    if cap is not None:
        r.set_wavefront_cap(cap)
    if pairs is not None:
        r.set_wavefront_pairs(pairs)
    y0, y1 = rows or (0, H)
    return r.render_rows_host(y0, y1), r.render_rows_host(y0, y1, f64=True)


@pytest.mark.parametrize("pairs", [0, 1, 2])
@pytest.mark.parametrize("name,t,W,H,d", CASES)
def test_wavefront_parity(worldmap, name, t, W, H, d, pairs):
    """RT_OPT_WAVEFRONT_PAIRS 0: every level's rays walk the hierarchy a wave at a time; 1: levels >= 1
    go through (ray, object) pairs sorted by object (the wfp_* kernels); 2: level 0 too."""
    from oracle import oracle as O
    gu, gf = _render(scene_text(name), t, W, H, d, pairs=pairs)
    rf, ru = O.OracleScene(scene_text(name), t, W, H, max_depth=d).render(0, H, f64=True)
    assert_close(gu, gf, ru, rf, f"wavefront {name} t={t} {W}x{H} d={d} pairs={pairs}")


def test_wavefront_pairs_one_object_many_hits(worldmap):
    """Shadow rays through several glass shells of one transparency (the pair path folds a count: T^k)
    and rays that meet coincident surfaces (the nearest-hit tie goes to the first object drawn)."""
    from oracle import oracle as O
    text = ("draw(sphere(<0, 0, 0>, 30, rgb(0.9, 0.9, 0.9), 0, 0.7))\n"
            "draw(sphere(<0, 0, 0>, 20, rgb(0.9, 0.5, 0.5), 0, 0.7))\n"
            "draw(sphere(<0, 0, 0>, 10, rgb(0.5, 0.9, 0.5), 0.3, 0.7))\n"
            "draw(sphere(<25, 0, 0>, 10, rgb(0.5, 0.5, 0.9), 0.5))\n"
            "draw(sphere(<25, 0, 0>, 10, rgb(0.9, 0.9, 0.1), 0.5))\n"
            "draw(plane(<0, 1, 0>, 40, blue, 0.3))\n"
            "append light(<0, 80, -60>, rgb(0.6, 0.6, 0.6), 100)\n")
    W, H, d = 160, 120, 10
    for pairs in (0, 1, 2):
        gu, gf = _render(text, 0.0, W, H, d, pairs=pairs)
        rf, ru = O.OracleScene(text, 0.0, W, H, max_depth=d).render(0, H, f64=True)
        assert_close(gu, gf, ru, rf, f"wavefront shells pairs={pairs}")


HUGE_T_SCENE = (
    "b = (1000000000 * 1000000000)\n"
    "t = ((b * b) * (b * b))\n"                           # 1e72: T^k overflows to inf after 5 hits
    "draw(sphere(<0, 0, -40>, 30, rgb(0.9, 0.9, 0.9), 0, t))\n"
    "draw(sphere(<0, 0, -40>, 25, rgb(0.9, 0.5, 0.5), 0, t))\n"
    "draw(sphere(<0, 0, -40>, 20, rgb(0.5, 0.9, 0.5), 0, t))\n"
    "draw(sphere(<0, 0, 10>, 12, rgb(0.5, 0.5, 0.9), 0.5))\n"
    "draw(plane(<0, 1, 0>, 40, blue, 0.3))\n"
    "append light(<0, 80, -160>, rgb(0.6, 0.6, 0.6), 100)\n")


def test_wavefront_huge_transparency_shadow_order(worldmap):
    """Shadow rays through shells of transparency 1e72 and an opaque sphere: in draw order the product
    reaches inf before or after the opaque factor (inf * 0 = NaN, which is not 0: the light still
    counts), so it is not a function of the hit counts and the pair path must not fold counts
    (scene.cpp shadow_pow).  Every pair setting against the oracle."""
    from oracle import oracle as O
    W, H, d = 160, 120, 6
    rf, ru = O.OracleScene(HUGE_T_SCENE, 0.0, W, H, max_depth=d).render(0, H, f64=True)
    for pairs in (0, 1, 2):
        gu, gf = _render(HUGE_T_SCENE, 0.0, W, H, d, pairs=pairs)
        assert_close(gu, gf, ru, rf, f"wavefront huge transparency pairs={pairs}")


@pytest.mark.parametrize("pairs", [0, 2])
@pytest.mark.parametrize("name,t", [("fractal", 0.0), ("spinning_globes", 0.3), ("globes", 0.0)])
def test_wavefront_level_overflow_fixup(worldmap, name, t, pairs):
    """Levels of 1 % of the pixel slots: most trees overflow, and their pixels come from the fix-up."""
    from oracle import oracle as O
    W, H, d = 128, 96, 10
    gu, gf = _render(scene_text(name), t, W, H, d, cap=1, pairs=pairs)
    rf, ru = O.OracleScene(scene_text(name), t, W, H, max_depth=d).render(0, H, f64=True)
    assert_close(gu, gf, ru, rf, f"wavefront overflow {name}")


def test_wavefront_rows_and_bands(worldmap):
    """Row ranges and cyclic row bands (a multi-GPU rank's share) through the wavefront path."""
    import torch
    import tinyraytracerinrust_amd as T
    from tinyraytracerinrust_amd import distributed as D
    from oracle import oracle as O
    W, H = 200, 150
    text = scene_text("fractal")
    ref_f, ref_u8 = O.OracleScene(text, 0.0, W, H).render(0, H, f64=True)
    gu, gf = _render(text, 0.0, W, H, 10, rows=(17, 131))
    assert_close(gu, gf, ref_u8[17:131], ref_f[17:131], "wavefront rows 17..131")
    rt = T.RayTracer(W, H)
    rt.load_scene(text, 0.0, asset_dir=SCENES)
    r = rt.renderer
    r.set_kernel("wavefront")
    world, band = 3, 8
    slot_rows = D.rows_per_rank(H, world, "cyclic", band)
    gath = torch.zeros((world * slot_rows, W, 4), dtype=torch.uint8, device="cuda")
    for rank in range(world):
        y_first, band_rows, pitch, n_bands = D.band_params(H, world, rank, "cyclic", band)
        r.render_row_bands(y_first, band_rows, pitch, n_bands, gath[rank * slot_rows:(rank + 1) * slot_rows])
    frame = D.assemble(gath, H, world, "cyclic", band)
    torch.cuda.synchronize()
    assert np.array_equal(frame.cpu().numpy(), ref_u8)


@pytest.mark.parametrize("pairs", [0, 2])
@pytest.mark.parametrize("seed", range(5000, 5032))
def test_wavefront_random_scenes(seed, pairs):
    """Seeded random scenes (trees and chains, odd materials) through the wavefront path."""
    from tests.scene_fuzz import random_scene
    from oracle import oracle as O
    text = random_scene(seed, chains=seed % 2 == 1)
    W, H, d = 96, 72, 6
    gu, gf = _render(text, 0.0, W, H, d, pairs=pairs)
    rf, ru = O.OracleScene(text, 0.0, W, H, max_depth=d).render(0, H, f64=True)
    assert_close(gu, gf, ru, rf, f"wavefront random scene {seed}")


def test_wavefront_option_bounds():
    import tinyraytracerinrust_amd as T
    rt = T.RayTracer(64, 48)
    rt.load_scene("draw(sphere(<0, 0, 0>, 30, red))", 0.0)
    for bad in (0, 401):
        with pytest.raises(T.RtError):
            rt.renderer.set_wavefront_cap(bad)
    for bad in (-1, 3, 8):
        with pytest.raises(T.RtError):
            rt.renderer.set_wavefront_pairs(bad)


@pytest.mark.parametrize("name,t", [("fractal", 0.0), ("fractal", 0.5)])
def test_ray_tree_autotune_same_pixels(worldmap, name, t):
    """Ray-tree scenes under RT_KERNEL_AUTO: the calibration launch, the first ordered launch (timed
    against one wavefront launch of the same rows) and the launches after it (whichever path won)
    all give the oracle's pixels."""
    import tinyraytracerinrust_amd as T
    from oracle import oracle as O
    W, H = 640, 480                                  # 4800 tiles: calibrated, ordered, autotuned
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text(name), t, asset_dir=SCENES)
    frames = [rt.renderer.render_rows_host(0, H) for _ in range(4)]
    _, ru = O.OracleScene(scene_text(name), t, W, H).render(0, H)
    for k, f in enumerate(frames):
        assert_close(f, None, ru, None, f"{name} t={t} auto launch {k}")


@pytest.mark.parametrize("pairs", [1, 2])
@pytest.mark.parametrize("text,d", [
    ("draw(sphere(<0, 0, 0>, 30, red, 0.3, 0.6))", 10),                         # one object: a ray tree
    ("draw(sphere(<0, 0, 0>, 30, red, 0.3, 0.6))\ndraw(plane(<0, 1, 0>, 35, blue, 0.5))", 1),   # depth 1
    ("draw(plane(<0, 1, 0>, 35, blue, 0.5))", 10),                                # unbounded object only
])
def test_wavefront_pairs_small_scenes(text, d, pairs):
    """Pair-path edge cases: a single object (one bucket), depth 1 (one pair level), an unbounded
    object (no culling box) -- every frame against the oracle."""
    from oracle import oracle as O
    W, H = 96, 72
    gu, gf = _render(text, 0.0, W, H, d, pairs=pairs)
    rf, ru = O.OracleScene(text, 0.0, W, H, max_depth=d).render(0, H, f64=True)
    assert_close(gu, gf, ru, rf, f"wavefront pairs={pairs} small scene d={d}")


def _sphere_field(n, seed):
    """n small spheres spread over the default camera's view, glass spheres that also reflect among
    them (ray trees), and a reflective floor: a hierarchy of ~2n nodes."""
    import random
    r = random.Random(seed)
    lines = ["draw(plane(<0, 1, 0>, 32, white * 0.6, 0.3))"]
    mats = ["red, 0.3, 0.6", "blue, 0, 0.6", "white * 0.8, 0.5, 0", "rgb(0.2, 0.9, 0.4), 0, 0"]   # one transparency: shadow_pow
    for k in range(n):
        c = f"<{r.uniform(-40, 40):.2f}, {r.uniform(-28, 28):.2f}, {r.uniform(-25, 45):.2f}>"
        lines.append(f"draw(sphere({c}, {r.uniform(0.8, 3.5):.2f}, {mats[k % len(mats)]}))")
    return "\n".join(lines)


@pytest.mark.parametrize("n", [400, 2100])
def test_wavefront_pairs_large_hierarchies(n):
    """Scenes past the candidate walks' LDS hierarchy (> 640 nodes: the walks read the node array from
    global memory) and, at 2100 objects, past the fused-scan sorts (> 2048 buckets: the candidate
    kernels count no pairs, the sorts launch their histogram and scan): every pixel against the oracle."""
    from oracle import oracle as O
    text = _sphere_field(n, 7000 + n)
    W, H, d = 96, 72, 6
    gu, gf = _render(text, 0.0, W, H, d, pairs=2)
    rf, ru = O.OracleScene(text, 0.0, W, H, max_depth=d).render(0, H, f64=True)
    assert_close(gu, gf, ru, rf, f"wavefront pairs, {n} objects")
