"""bench.py's N > 1 frame pipeline on one GPU: the RCCL path at world size 1 (torch.distributed.run,
--force-collective) with 4 frames in flight on own-queue streams -- band renders, all-gathers of
packed RGB8 (and RGBA8) slots, assemblies on their own stream, buffer reuse ordered by events.
After its timed region bench.py compares EVERY frame buffer with a single-launch render of the
frame and exits non-zero on a difference, so a stream-ordering or buffer-reuse mistake fails here.
The tiled row loop this stands for is src/raydebugger/debug_window.rs:74-87."""
import json
import os
import socket
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("gather,layout", [("rgb", "cyclic"), ("rgba", "contiguous")])
def test_collective_pipeline_frames_in_flight(gather, layout):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--force-collective",
           "--inflight", "4", "--steps", "12", "--warmup", "3", "--settle-ms", "0", "--no-cpu-baseline",
           "--gather", gather, "--layout", layout]
    p = subprocess.run(cmd, capture_output=True, text=True, env=env, cwd=ROOT, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([l for l in p.stdout.splitlines() if l.strip()][-1])
    d = line["distributed"]
    assert d["frames_in_flight"] == 4 and d["gather"] == gather
    assert d["frame_check"].startswith("all 5 frame buffers")
    assert "own hardware queue" in line["config"]["streams"]


@pytest.mark.parametrize("world,inflight,layout", [(2, 0, "cyclic"), (4, 1, "cyclic"), (8, 0, "cyclic"),
                                                    (3, 2, "contiguous")])
def test_rehearsal_n_ranks_on_one_gpu(world, inflight, layout):
    """The driver's N-GPU form (`python bench.py --gpus N`: bench.py starts its own N ranks) with
    every rank on the one GPU of this box: N processes each render their cyclic bands with the
    HIP library (megakernel with 4 frames in flight at the default K, the deferred-shadow kernel
    with split tiles at K = 1 for N >= 4), the gathers run over a real 2..8-rank process group
    (gloo, host-staged: RCCL refuses two ranks on one device), the assembly kernel builds every
    frame, and EVERY rank checks every frame buffer against its own single-launch render."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--rehearse-one-gpu",
           "--steps", "4", "--warmup", "2", "--settle-ms", "0", "--layout", layout, "--inflight", str(inflight)]
    p = subprocess.run(cmd, capture_output=True, text=True, env=env, cwd=ROOT, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([l for l in p.stdout.splitlines() if l.strip()][-1])
    assert line["value"] is None and line["n_gpus"] == world
    d = line["distributed"]
    assert d["backend"] == "gloo" and d["world_size_seen"] == world and d["layout"] == layout
    assert sum(d["rows_per_rank"]) == line["config"]["height"] and len(d["rows_per_rank"]) == world
    k = inflight or 4
    assert d["frames_in_flight"] == k
    assert d["frame_check"] == f"all {k + 1} frame buffers == single-launch render, on every rank"


@pytest.mark.parametrize("world", [2, 8])
def test_rehearsal_animation_ranks_on_one_gpu(world):
    """BASELINE config 5 as the driver runs it (`python bench.py --gpus N --config anim120`: frames
    dealt round-robin, f = rank (mod N), src/raydebugger/gui.rs:78-89) with every rank on the one
    GPU of this box: each rank compiles and uploads its frames, renders them on its own-queue
    streams, and after the timed region checks EVERY owned frame buffer against a single-launch
    render of that frame."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--rehearse-one-gpu",
           "--config", "anim120", "--steps", "2", "--warmup", "1", "--settle-ms", "0", "--streams", "2"]
    p = subprocess.run(cmd, capture_output=True, text=True, env=env, cwd=ROOT, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([l for l in p.stdout.splitlines() if l.strip()][-1])
    assert line["value"] is None and line["n_gpus"] == world
    d = line["distributed"]
    assert d["backend"] == "gloo" and d["world_size_seen"] == world
    assert d["frames_per_rank"] == [len(range(r, 120, world)) for r in range(world)]
    assert d["frames_of_rank"] == [list(range(r, 120, world)) for r in range(world)]
    assert d["frame_check"] == f"all {len(range(0, 120, world))} frame buffers == single-launch render, on every rank"
