"""Scene-specialised row kernels (tinyraytracerinrust_amd/csrc/spec.hip, RT_OPT_SPECIALIZE): the same
device code as the generic kernels, compiled by hipRTC with the uploaded scene's tables as constants.
Every frame against the CPU oracle (a restatement of src/raytracer/raytracer.rs:132-287), RGBA8
bit-identical -- and at level 2 (f64 and calibration launches specialised too) the f64 colours
bit-identical to the generic kernels' (the same operations in the same order, constants folded only
where the host computed them already).  The kernel info names which kernel every launch ran."""
import numpy as np
import pytest

from tests.conftest import SCENES, scene_text
from tests.test_gpu_parity import assert_close

pytestmark = pytest.mark.gpu


def _renderer(text, t, W, H, depth, level, kernel="auto"):
    import tinyraytracerinrust_amd as T
    rt = T.RayTracer(W, H)
    rt.max_depth = depth
    rt.load_scene(text, t, asset_dir=SCENES)
    r = rt.renderer
    r.set_kernel(kernel)
    r.set_specialize(level)
    assert r.kernel_variant() == "spec", r.kernel_info()
    return rt, r


def _oracle(text, t, W, H, depth, f64=False, y0=0, y1=None):
    from oracle import oracle as O
    return O.OracleScene(text, t, W, H, max_depth=depth).render(y0, H if y1 is None else y1, f64=f64)


def test_globes4k_specialised_full_frame(worldmap):
    """The headline frame: the calibration launch (generic at level 1) and the cost-ordered launch
    (specialised megakernel), every pixel against the oracle."""
    import torch
    W, H = 3840, 2160
    rt, r = _renderer(scene_text("globes"), 0.0, W, H, 10, 1)
    _, ref = _oracle(scene_text("globes"), 0.0, W, H, 10)
    for launch in ("calibration", "ordered"):
        f = r.render_rows(0, H)
        torch.cuda.synchronize()
        info = r.kernel_info()
        assert_close(f.cpu().numpy(), None, ref, None, f"spec 4K globes {launch} launch ({info})")
    assert "megakernel (specialised)" in info


@pytest.mark.parametrize("world", [8, 4])
def test_globes4k_rank_bands_specialised(worldmap, world):
    """A rank's share of the 4K frame at N = 8 / 4: the ordered launches take the specialised
    megakernel (the library's choice once it is loaded, k_rows.hip launch_bands)."""
    import torch
    from tinyraytracerinrust_amd import distributed as D
    W, H = 3840, 2160
    rt, r = _renderer(scene_text("globes"), 0.0, W, H, 10, 1)
    _, ref = _oracle(scene_text("globes"), 0.0, W, H, 10)
    slot_rows = D.rows_per_rank(H, world, "cyclic", 8)
    kinds = set()
    for launch in range(2):
        gath = torch.zeros((world * slot_rows, W, 3), dtype=torch.uint8, device="cuda")
        for rank in range(world):
            y_first, band_rows, pitch, n_bands = D.band_params(H, world, rank, "cyclic", 8)
            r.render_row_bands(y_first, band_rows, pitch, n_bands, gath[rank * slot_rows:(rank + 1) * slot_rows])
            kinds.add(r.kernel_info().split("last launch: ")[1])
        frame = D.assemble(gath, H, world, "cyclic", 8).cpu().numpy()
        assert_close(frame, None, ref, None, f"spec 4K globes N={world} bands, launch {launch} ({sorted(kinds)})")
    assert any("specialised" in k for k in kinds), kinds


def test_sphere1080_d0_specialised_full_frame():
    """BASELINE config 2 as `bench.py --config sphere1080d0` runs it (RT_OPT_SPECIALIZE 1, timing
    events off): the calibration launch and the cost-ordered launches of the specialised primary-ray
    kernel (rt_spec_prim_00: max_depth 0 at compile time, write-back stores, XCD line order), 1920x1080
    primary rays only, every pixel against the oracle."""
    import torch
    W, H = 1920, 1080
    text = "draw(sphere(<0, 0, 0>, 30, red))"
    rt, r = _renderer(text, 0.0, W, H, 0, 1)
    r.set_timing(False)
    _, ref = _oracle(text, 0.0, W, H, 0)
    for launch in ("calibration", "ordered", "ordered again"):
        f = r.render_rows(0, H, max_depth=0)
        torch.cuda.synchronize()
        info = r.kernel_info()
        assert_close(f.cpu().numpy(), None, ref, None, f"spec sphere 1080p d0 {launch} launch ({info})")
    assert "primary-ray (specialised)" in info, info


@pytest.mark.parametrize("scene,t,level", [("globes", 0.0, 1), ("globes", 0.3, 2), ("spinning_globes", 0.45, 1),
                                           ("fuzz_tree", 0.0, 1), ("fuzz_tree", 0.0, 2)])
def test_primary_ray_kernel_every_mode(worldmap, scene, t, level):
    """The primary-ray kernel of every kernel mode (reflection-only, refraction chains, ray trees) for
    max_depth 0 launches: calibration and ordered launches (level 2: the calibration launch is the
    primary-ray kernel's CAL form, and f64 rows too), full frames and row bands, against the oracle."""
    import torch
    from tests.scene_fuzz import random_scene
    from tinyraytracerinrust_amd import distributed as D
    W, H = 640, 360
    text = random_scene(7774) if scene == "fuzz_tree" else scene_text(scene)
    rt, r = _renderer(text, t, W, H, 0, level)
    f64ref, ref = _oracle(text, t, W, H, 0, f64=level == 2)
    for launch in ("calibration", "ordered"):
        f = r.render_rows(0, H, max_depth=0)
        torch.cuda.synchronize()
        info = r.kernel_info()
        assert_close(f.cpu().numpy(), None, ref, None, f"prim {scene} {launch} ({info})")
        assert launch == "calibration" and level == 1 or "primary-ray (specialised)" in info, info
    if level == 2:
        got = r.render_rows_host(0, H, max_depth=0, f64=True)
        assert "primary-ray (specialised)" in r.kernel_info(), r.kernel_info()
        assert np.nanmax(np.abs(got - f64ref)) <= 1e-9 and np.array_equal(np.isnan(got), np.isnan(f64ref))
    world = 4
    slot_rows = D.rows_per_rank(H, world, "cyclic", 8)
    gath = torch.zeros((world * slot_rows, W, 3), dtype=torch.uint8, device="cuda")
    for rank in range(world):
        y_first, band_rows, pitch, n_bands = D.band_params(H, world, rank, "cyclic", 8)
        r.render_row_bands(y_first, band_rows, pitch, n_bands, gath[rank * slot_rows:(rank + 1) * slot_rows], max_depth=0)
    frame = D.assemble(gath, H, world, "cyclic", 8).cpu().numpy()
    assert np.array_equal(frame[..., :3], ref[..., :3]), f"prim {scene} bands"


@pytest.mark.parametrize("kernel", ["auto", "deferred", "mega"])
def test_globes1080_d5_specialised(worldmap, kernel):
    import torch
    W, H = 1920, 1080
    rt, r = _renderer(scene_text("globes"), 0.0, W, H, 5, 1, kernel)
    _, ref = _oracle(scene_text("globes"), 0.0, W, H, 5)
    for _ in range(2):
        f = r.render_rows(0, H)
        torch.cuda.synchronize()
        assert_close(f.cpu().numpy(), None, ref, None, f"spec 1080p d5 {kernel} ({r.kernel_info()})")


@pytest.mark.parametrize("name,t,W,H,depth", [("spinning_globes", 0.3, 640, 480, 10), ("three_cubes", 0.0, 320, 240, 10),
                                              ("spinning_gimbals", 0.4, 320, 240, 10), ("ground_star", 0.2, 320, 240, 10),
                                              ("spinning_cube", 0.3, 320, 240, 10)])
def test_reference_scenes_specialised_level2(worldmap, name, t, W, H, depth):
    """Level 2: every row launch specialised (calibration, ordered, f64), against the oracle in RGBA8,
    and the f64 colours bit-equal to the generic kernels' -- refraction chains (spinning_globes), cubes,
    CSG gimbals and stars."""
    import tinyraytracerinrust_amd as T
    text = scene_text(name)
    rt, r = _renderer(text, t, W, H, depth, 2)
    su = r.render_rows_host(0, H)
    sf = r.render_rows_host(0, H, f64=True)
    assert "(specialised)" in r.kernel_info()
    g = T.RayTracer(W, H)
    g.max_depth = depth
    g.load_scene(text, t, asset_dir=SCENES)
    gf = g.renderer.render_rows_host(0, H, f64=True)
    rf, ru = _oracle(text, t, W, H, depth, f64=True)
    assert_close(su, sf, ru, rf, f"spec {name}")
    same = (sf == gf) | (np.isnan(sf) & np.isnan(gf))
    assert same.all(), f"{name}: {int((~same).sum())} f64 channels differ from the generic kernels"


@pytest.mark.parametrize("seed", [11, 23, 37, 3001, 3002])
def test_fuzz_scenes_specialised(worldmap, seed):
    """Random scenes of the parity fuzz suite (tests/scene_fuzz.py): nested CSG, tilted planes,
    transparent objects, colours outside [0, 1], random transforms and lights (3001+: thin rotated rods
    and slabs with oriented boxes)."""
    from tests.scene_fuzz import random_scene, random_rod_scene
    W, H = 96, 72
    text = random_rod_scene(seed) if seed >= 3000 else random_scene(seed)
    rt, r = _renderer(text, 0.0, W, H, 6, 2)
    su = r.render_rows_host(0, H)
    sf = r.render_rows_host(0, H, f64=True)
    rf, ru = _oracle(text, 0.0, W, H, 6, f64=True)
    assert_close(su, sf, ru, rf, f"spec fuzz seed {seed}")


def test_large_scene_keeps_generic_kernels(worldmap):
    """fractal.scene (171 objects) is beyond the unrolling limits: the option leaves the generic kernels
    in place, says so, and the frame is unchanged."""
    import tinyraytracerinrust_amd as T
    W, H = 96, 72
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text("fractal"), 0.0, asset_dir=SCENES)
    r = rt.renderer
    a = r.render_rows_host(0, H)
    r.set_specialize(1)
    assert r.kernel_variant() == "generic" and "too large to specialise" in r.kernel_info()
    assert np.array_equal(a, r.render_rows_host(0, H))


def test_specialise_option_round_trip(worldmap):
    """Off again: the generic kernels; on: the process cache returns the compiled programs at once."""
    import tinyraytracerinrust_amd as T
    text = scene_text("globes")
    rt, r = _renderer(text, 0.0, 160, 120, 10, 1)
    a = r.render_rows_host(0, 120)
    r.set_specialize(0)
    assert r.kernel_variant() == "generic"
    b = r.render_rows_host(0, 120)
    r.set_specialize(1)
    assert "[process cache]" in r.kernel_info()
    c = r.render_rows_host(0, 120)
    assert np.array_equal(a, b) and np.array_equal(b, c)
