"""The min/max colour clamps (rt_device.h in_limit<FC>, taken when rt::flatten proves every
colour-op operand finite and >= +0) against the compare/select clamps of color.rs:36-53 as the
reference writes them: the f64 colours of whole frames must be BIT-identical.  The two forms are
selected per context with rt_ctx_set_option(RT_OPT_FAST_CLAMP)."""
import numpy as np
import pytest

from tests.conftest import SCENES, scene_text

pytestmark = pytest.mark.gpu

CASES = [("globes", 0.0, 320, 240, 10), ("globes", 0.25, 640, 480, 10), ("spinning_globes", 0.3, 320, 240, 10),
         ("three_cubes", 0.0, 160, 120, 10), ("ground_star", 0.2, 160, 120, 10),
         ("spinning_gimbals", 0.4, 160, 120, 10), ("fractal", 0.0, 96, 72, 10)]


@pytest.mark.parametrize("name,t,W,H,d", CASES)
def test_fast_clamps_bit_identical(name, t, W, H, d):
    import tinyraytracerinrust_amd as T
    out = {}
    for fast in (True, False):
        rt = T.RayTracer(W, H)
        rt.max_depth = d
        rt.load_scene(scene_text(name), t, asset_dir=SCENES)
        rt.renderer.set_fast_clamp(fast)
        out[fast] = (rt.renderer.render_rows_host(0, H, f64=True), rt.renderer.render_rows_host(0, H))
    (fa, ua), (fb, ub) = out[True], out[False]
    assert np.array_equal(fa.view(np.uint64), fb.view(np.uint64))   # bit patterns, signs of zero included
    assert np.array_equal(ua, ub)
