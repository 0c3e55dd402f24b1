"""Calibration of the WRITE_SIZE / FETCH_SIZE counters on the row kernels' own store pattern
(diagnostic, run under rocprofv3 --pmc).  A wave of the row kernels shades one 8x8 tile and stores
eight 32-byte RGBA8 row segments (rt_device.h rows_body / store_pixel), a narrower access than the
16-byte-per-lane streaming stores the guide calibrated.  An empty scene (no objects: every pixel is
the background, nothing but the frame is written) rendered at 4K by the generic kernels isolates
the counter's figure for those stores: 3840 * 2160 * 4 = 33.2 MB of frame per launch.  A torch
fill of a tensor of the same size is the 16-byte-per-lane reference.
usage: rocprofv3 --pmc WRITE_SIZE -- python3 tools/write_calib.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tinyraytracerinrust_amd as T  # noqa: E402

W, H = 3840, 2160
rt = T.RayTracer(W, H)
rt.load_scene("", 0.0)
r = rt.renderer
out = r.render_rows(0, H)                            # calibration launch
for _ in range(10):
    r.render_rows(0, H, out=out)                     # cost-ordered launches
fill = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
for _ in range(10):
    fill.fill_(7)
torch.cuda.synchronize()
print("frame bytes", W * H * 4, "kernel", r.kernel_info(), flush=True)
