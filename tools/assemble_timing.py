"""Kernel time of the multi-GPU frame assembly (rt_assemble_row_bands_rgb8 / rt_assemble_row_bands)
at the 4K frame's slot sizes, N ranks, 8-row cyclic bands (diagnostic; run it under
`rocprofv3 --kernel-trace --stats` for the per-kernel trace).  Prints the mean of REPS launches
timed with one event pair around them.
usage: python tools/assemble_timing.py [N ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from tinyraytracerinrust_amd import distributed as D  # noqa: E402

W, H, band, reps = 3840, 2160, 8, 50
for world in [int(v) for v in sys.argv[1:]] or [2, 4, 8]:
    slot_rows = D.rows_per_rank(H, world, "cyclic", band)
    for ch in (3, 4):
        g = torch.randint(0, 256, (world * slot_rows, W, ch), dtype=torch.uint8, device="cuda")
        out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
        for _ in range(5):
            D.assemble(g, H, world, "cyclic", band, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            D.assemble(g, H, world, "cyclic", band, out=out)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        moved = g.numel() // world * world + out.numel()
        print(f"N={world} {'RGB8' if ch == 3 else 'RGBA8'} slots -> RGBA8 frame: {us:.1f} us per assembly, "
              f"{moved / (us * 1e-6) / 1e9:.0f} GB/s of {moved / 1e6:.1f} MB moved", flush=True)
