"""The min/max colour clamps (render_kernels.hip in_limit<FC>, taken when rt::flatten proves every
colour-op operand finite and >= +0) against the compare/select clamps of color.rs:36-53 as the
reference writes them: the f64 colours of whole frames must be BIT-identical (RT_FAST_CLAMP=0,
read once per process, so each setting renders in its own child process)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

CHILD = r"""
import sys
sys.path.insert(0, ROOT)
import numpy as np
import tinyraytracerinrust_amd as T
from tests.conftest import SCENES, scene_text
out = {}
for name, t, W, H, d in [("globes", 0.0, 320, 240, 10), ("globes", 0.25, 640, 480, 10), ("spinning_globes", 0.3, 320, 240, 10),
                         ("three_cubes", 0.0, 160, 120, 10), ("ground_star", 0.2, 160, 120, 10),
                         ("spinning_gimbals", 0.4, 160, 120, 10), ("fractal", 0.0, 96, 72, 10)]:
    rt = T.RayTracer(W, H)
    rt.max_depth = d
    rt.load_scene(scene_text(name), t, asset_dir=SCENES)
    out[f"{name}_{t}_{W}"] = rt.renderer.render_rows_host(0, H, f64=True)
    out[f"{name}_{t}_{W}_u8"] = rt.renderer.render_rows_host(0, H)
np.savez(OUT, **out)
print("ok")
"""


def _render(tmp_path, fast):
    out = str(tmp_path / f"fc{fast}.npz")
    env = dict(os.environ, RT_FAST_CLAMP=str(fast))
    p = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\nOUT = {out!r}\n" + CHILD], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-4000:]
    return np.load(out)


def test_fast_clamps_bit_identical(tmp_path):
    a, b = _render(tmp_path, 1), _render(tmp_path, 0)
    assert sorted(a.files) == sorted(b.files)
    for k in a.files:
        x, y = a[k], b[k]
        if x.dtype == np.float64:
            assert np.array_equal(x.view(np.uint64), y.view(np.uint64)), k   # bit patterns, signs of zero included
        else:
            assert np.array_equal(x, y), k
