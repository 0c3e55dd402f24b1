"""Full-frame parity at every BASELINE configuration's real size (BASELINE.json configs 2-5):
every pixel of the HIP render, through the C ABI, against the CPU oracle (a restatement of
src/raytracer/raytracer.rs:132-287 and its callees) on all usable host cores.

* 3840x2160 globes.scene, depth 10: the calibration launch (row-major, records tile costs) AND the
  cost-ordered launch that follows it;
* 1920x1080 globes.scene, depth 5;
* 1920x1080 single sphere, depth 0 (config 2);
* all 120 frames of the spinning_globes animation at 1920x1080, time = f / 120;
* the DSL-quirk scenes of tests/test_oracle.py compiled by the PRODUCT's rt_scene_compile and
  rendered on the GPU.

Bar: RGBA8 bit-identical (the north star's 1-LSB bound is reported, the count of differing channels
printed on failure).  These pin the exactness of
the kernels' culling (rt_device.h "conservative culling") over whole frames.
"""
import numpy as np
import pytest

from tests.conftest import SCENES, scene_text
from tests.test_gpu_parity import assert_close

pytestmark = pytest.mark.gpu

SPHERE = "draw(sphere(<0, 0, 0>, 30, red))"


@pytest.fixture(scope="module")
def T():
    import torch
    import tinyraytracerinrust_amd as T
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return T


def gpu_frames(T, text, time, W, H, depth, launches=2):
    """`launches` whole-frame renders on one context into device buffers (the first of a
    geometry of >= 2048 tiles is the calibration launch, later ones are cost-ordered)."""
    import torch
    rt = T.RayTracer(W, H)
    rt.max_depth = depth
    rt.load_scene(text, time, asset_dir=SCENES)
    out = []
    for _ in range(launches):
        f = rt.renderer.render_rows(0, H)
        torch.cuda.synchronize()
        out.append(f.cpu().numpy())
    return out


def oracle_frame(text, time, W, H, depth):
    from oracle import oracle as O
    _, u8 = O.OracleScene(text, time, W, H, max_depth=depth).render(0, H)
    return u8


@pytest.mark.parametrize("name,text,W,H,depth", [
    ("globes4k_d10", "globes", 3840, 2160, 10),
    ("globes1080_d5", "globes", 1920, 1080, 5),
    ("sphere1080_d0", None, 1920, 1080, 0),
])
def test_baseline_config_full_frame(T, worldmap, name, text, W, H, depth):
    text = scene_text(text) if text else SPHERE
    cal, ordered = gpu_frames(T, text, 0.0, W, H, depth)
    ref = oracle_frame(text, 0.0, W, H, depth)
    assert_close(cal, None, ref, None, f"{name} calibration launch")
    assert_close(ordered, None, ref, None, f"{name} ordered launch")
    print(f"{name}: {int((cal != ref).sum())} / {ref.size} channels differ (calibration), "
          f"{int((ordered != ref).sum())} (ordered)")
    assert (ordered[..., 3] == 255).all()


@pytest.fixture(scope="module")
def globes4k_oracle(worldmap):
    return oracle_frame(scene_text("globes"), 0.0, 3840, 2160, 10)


@pytest.mark.parametrize("world,channels", [(8, 3), (4, 4), (2, 3)])
def test_globes4k_rank_bands_full_frame(T, globes4k_oracle, world, channels):
    """BASELINE config 4 as the multi-GPU path renders it: every rank's cyclic 8-row bands
    (rt_render_row_bands: the calibration launch, then the ordered launch -- at N = 8 the
    deferred-shadow kernel with the costliest tiles split over several waves, at N <= 4 the
    megakernel), assembled (rt_assemble_row_bands): all 8.3 M pixels against the oracle."""
    import torch
    from tinyraytracerinrust_amd import distributed as D
    W, H = 3840, 2160
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text("globes"), 0.0, asset_dir=SCENES)
    r = rt.renderer
    slot_rows = D.rows_per_rank(H, world, "cyclic", 8)
    frames = []
    for launch in range(2):
        gath = torch.zeros((world * slot_rows, W, channels), dtype=torch.uint8, device="cuda")   # 3: packed RGB8 slots
        for rank in range(world):
            y_first, band_rows, pitch, n_bands = D.band_params(H, world, rank, "cyclic", 8)
            r.render_row_bands(y_first, band_rows, pitch, n_bands, gath[rank * slot_rows:(rank + 1) * slot_rows])
        frames.append(D.assemble(gath, H, world, "cyclic", 8).cpu().numpy())
    assert_close(frames[0], None, globes4k_oracle, None, f"4K globes N={world} bands, calibration launches")
    assert_close(frames[1], None, globes4k_oracle, None, f"4K globes N={world} bands, ordered launches")


@pytest.fixture(scope="module")
def anim_families(T):
    """The scene families exactly as `bench.py --config anim120` registers them: all 120 frames of
    spinning_globes.scene at 1920x1080, time f / 120 (rt_spec_family_register; two families, 63 + 57
    frames).  Yields the family size each frame's program must report."""
    text = scene_text("spinning_globes")
    scenes = [T.Scene.compile(text, f / 120, 1920, 1080, asset_dir=SCENES) for f in range(120)]
    T.Scene.clear_families()
    T.Scene.register_family(scenes)
    yield text
    T.Scene.clear_families()


@pytest.mark.parametrize("chunk", list(range(8)))
def test_spinning_globes_animation_frames(T, anim_families, chunk):
    """BASELINE config 5, ALL 120 frames (15 per test case): frame f at time f / 120, 1920x1080,
    depth 10 (refraction chains), against the oracle frame (the reference's per-frame scene build,
    src/raydebugger/debug_window.rs:53-62, and render, raytracer.rs:132-287), through BOTH code paths
    the library has for it:
      * the generic chain megakernel: calibration launch, then the cost-ordered launch;
      * the code objects `bench.py --config anim120` times: the frame's scene-family program
        (RT_OPT_SPECIALIZE 1 after the bench's own 120-frame registration, `anim_families`) -- the
        ordered launch is the family's specialised megakernel, and the kernel info must name a family
        of 63 or 57 frames."""
    import torch
    text = anim_families
    W, H = 1920, 1080
    families = set()
    for frame in range(chunk * 15, chunk * 15 + 15):
        ref = oracle_frame(text, frame / 120, W, H, 10)
        cal, ordered = gpu_frames(T, text, frame / 120, W, H, 10)
        assert_close(cal, None, ref, None, f"spinning_globes f={frame} calibration launch")
        assert_close(ordered, None, ref, None, f"spinning_globes f={frame} ordered launch")
        r = T.Renderer(0)
        r.set_specialize(1)
        r.upload(T.Scene.compile(text, frame / 120, W, H, asset_dir=SCENES))
        r.set_timing(False)
        for launch in ("calibration", "ordered"):
            f = r.render_rows(0, H, max_depth=10)
            torch.cuda.synchronize()
            info = r.kernel_info()
            assert_close(f.cpu().numpy(), None, ref, None, f"spinning_globes f={frame} family program, {launch} ({info})")
        assert "megakernel (specialised)" in info and ("family of 63 scenes" in info or "family of 57 scenes" in info), info
        families.add(info.split("family of ")[1].split(" ")[0])
        r.free()
    print(f"frames {chunk * 15}..{chunk * 15 + 14}: families {sorted(families)}")


def test_dsl_quirk_scenes_through_product_compiler(T):
    """The DSL-quirk cases (operator-chain dropping, locals/globals, while, camera transformed
    twice, default arguments, appended lights, ...) compiled by rt_scene_compile and rendered by
    the HIP kernels, against the oracle's own parse + render of the same text."""
    from tests.test_oracle import DSL_CASES
    from oracle import oracle as O
    W, H = 160, 120
    for key, text in sorted(DSL_CASES.items()):
        rt = T.RayTracer(W, H)
        rt.load_scene(text, 0.0, asset_dir=SCENES)
        gu = rt.renderer.render_rows_host(0, H)
        gf = rt.renderer.render_rows_host(0, H, f64=True)
        rf, ru = O.OracleScene(text, 0.0, W, H).render(0, H, f64=True)
        assert_close(gu, gf, ru, rf, f"DSL {key}")
