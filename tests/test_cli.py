"""Headless driver (python -m tinyraytracerinrust_amd render ...), which replaces the reference's
GUI entry point for producing a frame (src/main.rs:7-9, src/raydebugger/debug_window.rs:53-62):
argument handling and the no-fallback rule on CPU; on the GPU, the written PNG read back with
rt_read_png_rgba8 against the oracle's u8 frame."""
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.conftest import ROOT, SCENES


def _cli(*args, timeout=300):
    return subprocess.run([sys.executable, "-m", "tinyraytracerinrust_amd", *args], capture_output=True, text=True,
                          cwd=ROOT, timeout=timeout)


def test_cli_parses_and_rejects_bad_size():
    from tinyraytracerinrust_amd.__main__ import _parse
    a = _parse(["render", "x.scene", "--size", "64x48", "--frame", "75"])
    assert (a.width, a.height, a.t) == (64, 48, 0.25)          # time = frame / 300 (debug_window.rs:57)
    p = _cli("render", os.path.join(SCENES, "globes.scene"), "--size", "64by48")
    assert p.returncode != 0 and "--size" in p.stderr


def test_cli_fails_loudly_without_a_gpu(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    out = tmp_path / "x.png"
    p = _cli("render", os.path.join(SCENES, "globes.scene"), "--size", "32x24", "-o", str(out))
    assert p.returncode != 0
    assert "no CPU fallback" in p.stderr or "HIP" in p.stderr
    assert not out.exists()


@pytest.mark.gpu
@pytest.mark.parametrize("channels", [3, 4])
def test_cli_png_matches_oracle(tmp_path, worldmap, channels):
    import tinyraytracerinrust_amd as T
    from oracle import oracle as O
    out = tmp_path / "globes.png"
    p = _cli("render", os.path.join(SCENES, "globes.scene"), "--size", "96x72", "--time", "0.25",
             "--channels", str(channels), "-o", str(out), timeout=120)
    assert p.returncode == 0, p.stderr
    got = T.read_png_rgba8(str(out))
    text = open(os.path.join(SCENES, "globes.scene")).read()
    _, want = O.OracleScene(text, 0.25, 96, 72).render()
    assert got.shape == want.shape
    assert np.array_equal(got[..., :3], want[..., :3])
    assert (got[..., 3] == 255).all()
