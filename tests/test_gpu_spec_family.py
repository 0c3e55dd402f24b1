"""Scene families (rt_spec_family_register, csrc/spec.hip; rt_device.h RT_REC): one specialised program
per family of scenes of the same structure -- the frames of an animation (the reference's animate
mode, gui.rs:78-89, builds every frame's scene anew) -- the words every member shares compiled in,
the others read from the rendering scene's own tables.  Every frame against the CPU oracle (a
restatement of raytracer.rs:132-287), RGBA8 bit-identical, and the kernel info names the family
program; a scene that was not registered but shares the family's constant words renders through
it exactly as well, and one that does not keeps its own program."""
import pytest

from tests.conftest import SCENES, scene_text
from tests.test_gpu_parity import assert_close

pytestmark = pytest.mark.gpu

W, H, DEPTH, F = 640, 480, 10, 12


@pytest.fixture(scope="module")
def family():
    import tinyraytracerinrust_amd as T
    text = scene_text("spinning_globes")
    scenes = [T.Scene.compile(text, f / F, W, H, asset_dir=SCENES) for f in range(F)]
    T.Scene.clear_families()
    T.Scene.register_family(scenes)
    yield text, scenes
    T.Scene.clear_families()


def _render(text, t):
    import tinyraytracerinrust_amd as T
    sc = T.Scene.compile(text, t, W, H, asset_dir=SCENES)
    r = T.Renderer(0)
    r.set_specialize(1)
    r.upload(sc)                       # requests the program: a registered family's (compiled), or its own
    r.spec_wait()
    frames = [r.render_rows_host(0, H) for _ in range(2)]          # calibration, then the ordered launch
    return frames, r.kernel_info()


@pytest.mark.parametrize("f", [0, 1, 5, 6, 11])
def test_family_frames(worldmap, family, f):
    from oracle import oracle as O
    text, _ = family
    (cal, ordered), info = _render(text, f / F)
    _, ref = O.OracleScene(text, f / F, W, H, max_depth=DEPTH).render(0, H)
    assert_close(cal, None, ref, None, f"frame {f} calibration")
    assert_close(ordered, None, ref, None, f"frame {f} ({info})")
    assert "family of" in info and "(specialised)" in info, info


def test_unregistered_time(worldmap, family):
    """t = 0.37 is not one of the registered frames: either a family holds its structure and shared
    words (then its program renders it) or it compiles its own -- the pixels are the oracle's."""
    from oracle import oracle as O
    text, _ = family
    (_, ordered), info = _render(text, 0.37)
    _, ref = O.OracleScene(text, 0.37, W, H, max_depth=DEPTH).render(0, H)
    assert_close(ordered, None, ref, None, f"t = 0.37 ({info})")
    assert "(specialised)" in info, info


def test_other_scene_keeps_its_program(worldmap, family):
    import tinyraytracerinrust_amd as T
    sc = T.Scene.compile(scene_text("globes"), 0.0, 160, 120, asset_dir=SCENES)
    r = T.Renderer(0)
    r.set_specialize(1)
    r.upload(sc)
    r.spec_wait()
    assert r.kernel_variant() == "spec" and "family" not in r.kernel_info(), r.kernel_info()
