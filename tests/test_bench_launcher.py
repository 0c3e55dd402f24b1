"""bench.py's N-rank launcher on CPU: ``python bench.py --gpus N`` started WITHOUT
torch.distributed.run must start its own N ranks (as the driver may launch it), and each rank
must own its band layout, all-gather it and assemble the frame.  ``--launcher-check`` runs that
machinery under gloo with a per-pixel pattern in place of the renderer (the reference's row loop
being tiled is src/raydebugger/debug_window.rs:74-87)."""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT


def _run(*args):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       env=env, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout           # exactly one JSON line, from rank 0
    return json.loads(lines[0])


@pytest.mark.parametrize("world,layout,gather", [(2, "cyclic", "rgb"), (2, "contiguous", "rgb"), (3, "cyclic", "rgb"),
                                                 (2, "cyclic", "rgba")])
def test_self_launch_gloo(world, layout, gather):
    line = _run("--gpus", str(world), "--launcher-check", "--layout", layout, "--steps", "2", "--gather", gather)
    d = line["distributed"]
    assert line["n_gpus"] == world
    assert d["world_size_seen"] == world and d["backend"] == "gloo" and d["gather"] == gather
    assert d["frame_check"] is True
    assert len(d["rows_per_rank"]) == world and sum(d["rows_per_rank"]) == line["config"]["height"]
    if layout == "cyclic":                          # the single-frame phase's chunked gathers (default 4)
        assert d["chunks"] == 4 and d["chunks_check"] is True


def test_self_launch_gloo_chunks():
    """Sub-frame gathers at other chunk counts, world 3 (a partial last slot band)."""
    for c in (2, 3):
        d = _run("--gpus", "3", "--launcher-check", "--layout", "cyclic", "--steps", "1", "--chunks", str(c))["distributed"]
        assert d["frame_check"] is True and d["chunks"] == c and d["chunks_check"] is True


def test_host_cpus_reports_usable_cores():
    sys.path.insert(0, ROOT)
    import bench
    cores, model, aff, quota = bench.host_cpus()
    assert 1 <= cores <= aff
    assert isinstance(model, str) and model
