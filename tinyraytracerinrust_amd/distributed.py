"""Multi-GPU frame assembly: row tiles rendered per rank, one all-gather (RCCL over xGMI).

The reference renders a frame as one thread-pool job (src/raydebugger/gui.rs:677,
debug_window.rs:229-273) and has no distributed code.  Pixels are independent, so the frame
is split into equal row tiles, one per rank (one process per GPU); each rank renders its tile
with the HIP kernel and a single ``all_gather_into_tensor`` (backend "nccl" = RCCL) assembles
the RGBA8 frame on every rank.  Two tilings:

* ``contiguous``: rank r owns rows [r*T, (r+1)*T), T = ceil(H/G) (last tile padded);
* ``cyclic``: bands of ``band`` rows dealt round-robin (band b -> rank b % G), which evens out
  the sky-vs-floor cost imbalance; the gathered buffer is reordered locally afterwards.

The same functions run on CPU tensors under ``gloo`` (tests/test_distributed_gloo.py), with a
caller-supplied ``render_rows(y0, y1, out)`` instead of the GPU renderer.
"""
from __future__ import annotations

from typing import Callable, List, Tuple

import torch
import torch.distributed as dist


def contiguous_rows(height: int, world: int, rank: int) -> List[Tuple[int, int]]:
    tile = -(-height // world)
    y0 = min(height, rank * tile)
    return [(y0, min(height, y0 + tile))]


def cyclic_rows(height: int, world: int, rank: int, band: int) -> List[Tuple[int, int]]:
    out = []
    nb = -(-height // band)
    for b in range(rank, nb, world):
        out.append((b * band, min(height, (b + 1) * band)))
    return out


def rows_per_rank(height: int, world: int, layout: str, band: int) -> int:
    """Rows in every rank's (padded) slot of the gather buffer; equal for all ranks."""
    if layout == "contiguous":
        return -(-height // world)
    nb = -(-height // band)
    return -(-nb // world) * band


def owned_rows(height: int, world: int, rank: int, layout: str = "contiguous", band: int = 16):
    return contiguous_rows(height, world, rank) if layout == "contiguous" else cyclic_rows(height, world, rank, band)


def band_params(height: int, world: int, rank: int, layout: str, band: int) -> Tuple[int, int, int, int]:
    """(y_first, band_rows, band_pitch, n_bands) of this rank's rows for rt_render_row_bands."""
    own = owned_rows(height, world, rank, layout, band)
    if not own:
        return 0, 0, 0, 0
    if layout == "contiguous":
        return own[0][0], own[0][1] - own[0][0], height, 1
    return own[0][0], band, world * band, len(own)


def chunk_plan(height: int, world: int, band: int, chunks: int, row_cost=None) -> List[Tuple[int, int]]:
    """Split a cyclic-band frame into `chunks` sub-frames that gather independently: slot band s of
    every rank covers frame rows [s * world * band, (s + 1) * world * band), so a run of slot bands
    is a contiguous frame row range with the same cyclic layout inside it (its own render launch per
    rank, its own all-gather of world x its slot rows, its own assembly into frame rows [Y0, Y1)).
    Returns [(Y0, Y1)] in the order to render and gather them: cheapest first when per-row costs are
    given (the costly tail then renders while the cheap chunks' gathers run), else frame order."""
    span = world * band
    nsb = -(-height // span)                       # slot bands per rank (the last may be partial)
    chunks = max(1, min(chunks, nsb))
    cuts = [round(i * nsb / chunks) for i in range(chunks + 1)]
    plan = [(cuts[i] * span, min(height, cuts[i + 1] * span)) for i in range(chunks) if cuts[i + 1] > cuts[i]]
    if row_cost is not None:
        plan.sort(key=lambda c: sum(row_cost[c[0]:c[1]]))
    return plan


def chunk_band_params(y0: int, y1: int, world: int, rank: int, band: int) -> Tuple[int, int, int, int, int]:
    """(y_first, band_rows, band_pitch, n_bands, slot_rows) of this rank's bands in frame rows [y0, y1)
    of a chunk_plan chunk; slot_rows = the chunk's (equal, padded) rows per rank."""
    span = world * band
    nsb = -(-(y1 - y0) // span)
    first = y0 + rank * band
    n = len(range(first, y1, span))
    return first, band, span, n, nsb * band


def render_local(render_rows: Callable[[int, int, torch.Tensor], None], height: int, width: int, world: int,
                 rank: int, layout: str, band: int, device, dtype=torch.uint8) -> torch.Tensor:
    """This rank's slot: its rows packed densely (padding rows left zero)."""
    slot = torch.zeros((rows_per_rank(height, world, layout, band), width, 4), dtype=dtype, device=device)
    r = 0
    for y0, y1 in owned_rows(height, world, rank, layout, band):
        render_rows(y0, y1, slot[r:r + (y1 - y0)])
        r += y1 - y0
    return slot


def assemble(gathered: torch.Tensor, height: int, world: int, layout: str, band: int,
             out: torch.Tensor = None) -> torch.Tensor:
    """gathered: (world * slot_rows, W, 4) RGBA8 or (world * slot_rows, W, 3) packed RGB8 slots in
    rank order -> (H, W, 4) RGBA8 frame (A = 255 for RGB slots).

    On a GPU tensor this is ONE launch of the library's row-placement kernel
    (rt_assemble_row_bands, 16-byte row copies; rt_assemble_row_bands_rgb8 for RGB slots); on CPU
    tensors (gloo) the torch restatement assemble_reference below, which the GPU tests compare it
    with."""
    if not gathered.is_cuda:
        return assemble_reference(gathered, height, world, layout, band, out)
    slot_rows = gathered.shape[0] // world
    band_rows = slot_rows if layout == "contiguous" else band
    if gathered.shape[-1] == 3:
        return _assemble_device_rgb(gathered, height, world, slot_rows, band_rows, out)
    if layout == "contiguous" and out is None:
        return gathered[:height]                                  # already in frame order: a view
    return _assemble_device(gathered, height, world, slot_rows, band_rows, out)


def _assemble_device_rgb(gathered: torch.Tensor, height: int, world: int, slot_rows: int, band_rows: int,
                         out: torch.Tensor = None) -> torch.Tensor:
    import ctypes
    from . import _lib
    W = gathered.shape[1]
    if out is None:
        out = torch.empty((height, W, 4), dtype=torch.uint8, device=gathered.device)
    if tuple(out.shape) != (height, W, 4) or out.dtype != torch.uint8 or out.device != gathered.device:
        raise ValueError(f"frame tensor {tuple(out.shape)} {out.dtype} does not match {(height, W, 4)} uint8")
    if not (gathered[0].is_contiguous() and out[0].is_contiguous()):
        raise ValueError("rows of the gathered buffer and the frame must be contiguous")
    st = torch.cuda.current_stream(gathered.device).cuda_stream
    _lib.check(_lib.lib().rt_assemble_row_bands_rgb8(
        ctypes.c_void_p(gathered.data_ptr()), gathered.stride(0), world, slot_rows, band_rows, height, W,
        ctypes.c_void_p(out.data_ptr()), out.stride(0), ctypes.c_void_p(st)))
    return out


def _assemble_device(gathered: torch.Tensor, height: int, world: int, slot_rows: int, band_rows: int,
                     out: torch.Tensor = None) -> torch.Tensor:
    import ctypes
    from . import _lib
    tail = tuple(gathered.shape[1:])
    if out is None:
        out = torch.empty((height,) + tail, dtype=gathered.dtype, device=gathered.device)
    if tuple(out.shape) != (height,) + tail or out.dtype != gathered.dtype or out.device != gathered.device:
        raise ValueError(f"frame tensor {tuple(out.shape)} {out.dtype} does not match {(height,) + tail} {gathered.dtype}")
    if not (gathered[0].is_contiguous() and out[0].is_contiguous()):
        raise ValueError("rows of the gathered buffer and the frame must be contiguous")
    es = gathered.element_size()
    st = torch.cuda.current_stream(gathered.device).cuda_stream
    _lib.check(_lib.lib().rt_assemble_row_bands(
        ctypes.c_void_p(gathered.data_ptr()), gathered.stride(0) * es, world, slot_rows, band_rows, height,
        gathered[0].numel() * es, ctypes.c_void_p(out.data_ptr()), out.stride(0) * es, ctypes.c_void_p(st)))
    return out


def assemble_reference(gathered: torch.Tensor, height: int, world: int, layout: str, band: int,
                       out: torch.Tensor = None) -> torch.Tensor:
    """The same placement in torch ops.  Contiguous tiles are already in frame order (a view).
    Cyclic slots hold bands g = b * world + rank at slot rows [b * band, (b + 1) * band), so the
    frame is a permutation: view (world, bands_per_rank, band, ...) -> swap the first two axes ->
    first H rows."""
    slot_rows = gathered.shape[0] // world
    if gathered.shape[-1] == 3:                                    # packed RGB slots -> RGBA, A = 255
        rgba = torch.full(gathered.shape[:-1] + (4,), 255, dtype=gathered.dtype, device=gathered.device)
        rgba[..., :3] = gathered
        gathered = rgba
    if layout == "contiguous":
        frame = gathered[:height]
        if out is not None:
            out.copy_(frame)
            return out
        return frame
    nbpr = slot_rows // band
    tail = tuple(gathered.shape[1:])
    perm = gathered.view((world, nbpr, band) + tail).transpose(0, 1).reshape((world * nbpr * band,) + tail)
    if out is None:
        return perm[:height].contiguous()
    out.copy_(perm[:height])
    return out


def render_frame_distributed(render_rows: Callable[[int, int, torch.Tensor], None], height: int, width: int,
                             device, layout: str = "contiguous", band: int = 16, group=None,
                             assemble_frame: bool = True) -> torch.Tensor:
    """Render this rank's rows, all-gather every slot, return the (H, W, 4) RGBA8 frame."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    slot = render_local(render_rows, height, width, world, rank, layout, band, device)
    gathered = torch.empty((world * slot.shape[0], width, 4), dtype=slot.dtype, device=slot.device)
    dist.all_gather_into_tensor(gathered, slot, group=group)
    return assemble(gathered, height, world, layout, band) if assemble_frame else gathered
