"""Multi-rank frame assembly (tinyraytracerinrust_amd/distributed.py) on CPU with gloo,
world_size 2 and 3: every rank renders its row tiles (here with the CPU oracle standing in for
the GPU renderer), one all_gather assembles the frame, which must equal the single-process frame
bit for bit -- contiguous and cyclic layouts, heights not divisible by the world size."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tests.conftest import ROOT, SCENES


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, W, H, layout, band, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from oracle import oracle as O
    from tinyraytracerinrust_amd import distributed as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    O.register_texture_file("worldmap.png", os.path.join(SCENES, "worldmap.png"))
    sc = O.OracleScene(open(os.path.join(SCENES, "globes.scene")).read(), 0.0, W, H)

    def render_rows(y0, y1, out):
        _, u = sc.render(y0, y1, threads=1)
        out.copy_(torch.from_numpy(u))

    frame = D.render_frame_distributed(render_rows, H, W, "cpu", layout=layout, band=band)
    np.save(os.path.join(out_dir, f"frame_{rank}.npy"), frame.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,layout,band", [
    (2, 40, 30, "contiguous", 0), (2, 40, 31, "contiguous", 0), (2, 40, 31, "cyclic", 4),
    (3, 24, 25, "cyclic", 3), (3, 24, 25, "contiguous", 0),
])
def test_gloo_assembly(tmp_path, worldmap, world, W, H, layout, band):
    from oracle import oracle as O
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, W, H, layout, band or 16, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    _, want = O.OracleScene(open(os.path.join(SCENES, "globes.scene")).read(), 0.0, W, H).render()
    for r in range(world):
        got = np.load(tmp_path / f"frame_{r}.npy")
        assert got.shape == (H, W, 4)
        assert np.array_equal(got, want)


def test_row_ownership_partitions_frame():
    from tinyraytracerinrust_amd import distributed as D
    for H in (1, 7, 2160, 2161):
        for world in (1, 2, 3, 8):
            for layout, band in (("contiguous", 0), ("cyclic", 16), ("cyclic", 5)):
                rows = []
                for r in range(world):
                    own = D.owned_rows(H, world, r, layout, band or 16)
                    n = sum(b - a for a, b in own)
                    assert n <= D.rows_per_rank(H, world, layout, band or 16)
                    rows += [y for a, b in own for y in range(a, b)]
                assert sorted(rows) == list(range(H))
