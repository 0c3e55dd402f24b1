"""Pixel stores at the edges of the row kernels' tiles (rt_device.h rows_body / deferred_body /
store_pixel), against the CPU oracle (raytracer.rs:132-287 + easy_pixbuf.rs:46-53), bit-identical:
ragged frame widths (tiles cut by the frame edge), destinations whose rows are not aligned (pitched
and offset device buffers, padding left untouched), packed RGB8 band slots of odd widths, and the
split tiles of the deferred kernel (lanes without a pixel).  (A packed variant -- four pixels per
16-byte store -- was measured and dropped: no change in WRITE_SIZE, profiles/r05k_store_pattern.txt.)"""
import numpy as np
import pytest

from tests.conftest import SCENES, scene_text

pytestmark = pytest.mark.gpu


def _rt(text, W, H, depth=10, kernel="auto"):
    import tinyraytracerinrust_amd as T
    rt = T.RayTracer(W, H)
    rt.max_depth = depth
    rt.load_scene(text, 0.0, asset_dir=SCENES)
    rt.renderer.set_kernel(kernel)
    return rt.renderer


def _ref(text, W, H, depth=10):
    from oracle import oracle as O
    return O.OracleScene(text, 0.0, W, H, max_depth=depth).render(0, H)[1]


@pytest.mark.parametrize("W,H", [(101, 67), (98, 35), (3, 9), (1, 1)])
@pytest.mark.parametrize("kernel", ["mega", "deferred"])
def test_ragged_widths(worldmap, W, H, kernel):
    text = scene_text("globes")
    r = _rt(text, W, H, kernel=kernel)
    got = r.render_rows_host(0, H)
    ref = _ref(text, W, H)
    assert np.array_equal(got, ref), f"{W}x{H} {kernel}: {int((got != ref).sum())} channels differ"


@pytest.mark.parametrize("offset,pad", [(0, 4), (4, 0), (8, 12), (12, 3)])
def test_unaligned_destination_rgba8(worldmap, offset, pad):
    """Rows start `offset` bytes into a device buffer with `pad` bytes between rows (no 16-byte
    alignment anywhere); the padding stays untouched."""
    import torch
    W, H = 96, 64
    text = scene_text("globes")
    r = _rt(text, W, H)
    pitch = W * 4 + pad
    buf = torch.full((offset + pitch * H + 16,), 0xA5, dtype=torch.uint8, device="cuda")
    for _ in range(2):                                   # unordered, then (>= 2048 tiles only) ordered
        r.render_rows_into(0, H, buf.data_ptr() + offset, pitch)
    torch.cuda.synchronize()
    host = buf.cpu().numpy()
    rows = np.stack([host[offset + y * pitch: offset + y * pitch + W * 4] for y in range(H)]).reshape(H, W, 4)
    assert np.array_equal(rows, _ref(text, W, H))
    gaps = [host[offset + y * pitch + W * 4: offset + (y + 1) * pitch] for y in range(H - 1)]
    assert all((g == 0xA5).all() for g in gaps) and (host[:offset] == 0xA5).all()


@pytest.mark.parametrize("W", [99, 128, 1922])
def test_rgb8_band_slots(worldmap, W):
    """Packed RGB8 rows (the N > 1 gather slots) at widths whose last tile is partial or whose rows
    start on odd byte offsets (W * 3 not a multiple of 4)."""
    import torch
    from tinyraytracerinrust_amd import distributed as D
    H, world = 120, 4
    text = scene_text("globes")
    r = _rt(text, W, H, depth=6)
    ref = _ref(text, W, H, depth=6)
    for rank in range(world):
        y_first, band_rows, pitch, n_bands = D.band_params(H, world, rank, "cyclic", 8)
        slot = torch.zeros((n_bands * band_rows, W, 3), dtype=torch.uint8, device="cuda")
        r.render_row_bands(y_first, band_rows, pitch, n_bands, slot)
        torch.cuda.synchronize()
        rows = [y for y0, y1 in D.owned_rows(H, world, rank, "cyclic", 8) for y in range(y0, y1)]
        got = slot.cpu().numpy()[:len(rows)]
        assert np.array_equal(got, ref[rows][..., :3]), f"W={W} rank {rank}"


def test_split_tiles_4k_share(worldmap):
    """The N = 8 share of the 4K frame: the deferred kernel's costliest tiles split over 2-8 waves
    (lanes past a part's pixels store nothing), RGBA8 band slot."""
    import torch
    from tinyraytracerinrust_amd import distributed as D
    from oracle import oracle as O
    W, H, world = 3840, 2160, 8
    text = scene_text("globes")
    r = _rt(text, W, H, kernel="deferred")
    y_first, band_rows, pitch, n_bands = D.band_params(H, world, 3, "cyclic", 8)
    sc = O.OracleScene(text, 0.0, W, H, max_depth=10)
    ref = np.concatenate([sc.render(y0, y1)[1] for y0, y1 in D.owned_rows(H, world, 3, "cyclic", 8)])
    for launch in range(2):
        slot = torch.zeros((n_bands * band_rows, W, 4), dtype=torch.uint8, device="cuda")
        r.render_row_bands(y_first, band_rows, pitch, n_bands, slot)
        torch.cuda.synchronize()
        got = slot.cpu().numpy()[:ref.shape[0]]
        assert np.array_equal(got, ref), f"launch {launch}: {int((got != ref).sum())} channels differ ({r.kernel_info()})"


@pytest.mark.parametrize("W,pad,depth", [(512, 0, 0), (512, 128, 0), (512, 4, 0), (520, 0, 0), (512, 0, 10)])
def test_cached_frame_stores_and_xcd_order(worldmap, W, pad, depth):
    """The XCD-aware line order (k_rows.hip xcd_line_order): ordered primary-ray (max_depth 0) RGBA8
    launches whose rows are whole 128-byte lines (tiles_x % 4 == 0, 128-byte pitch and base) put a
    line's four tiles at entries e, e + 8, e + 16, e + 24 of the cost order; other pitches and widths,
    and deeper launches, keep the plain cost order.  >= 2048 tiles, so the calibration launch and two
    ordered launches each give the oracle's bits, and the row padding is left untouched."""
    import torch
    H = 256
    text = scene_text("globes")
    r = _rt(text, W, H, depth=depth)
    pitch = W * 4 + pad
    ref = _ref(text, W, H, depth=depth)
    buf = torch.full((pitch * H + 256,), 0xA5, dtype=torch.uint8, device="cuda")
    for launch in ("calibration", "ordered", "ordered again"):
        r.render_rows_into(0, H, buf.data_ptr(), pitch)
        torch.cuda.synchronize()
        host = buf.cpu().numpy()
        rows = np.stack([host[y * pitch: y * pitch + W * 4] for y in range(H)]).reshape(H, W, 4)
        assert np.array_equal(rows, ref), f"{W} pad {pad} {launch}: {int((rows != ref).sum())} channels differ"
        gaps = [host[y * pitch + W * 4: (y + 1) * pitch] for y in range(H - 1)]
        assert all((g == 0xA5).all() for g in gaps)
