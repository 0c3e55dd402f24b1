"""The tail kernel (rt_device.h tail_body, k_rows.hip render_tail_kernel; RT_OPT_TAIL_TILES): the
costliest calibrated tiles of a tail-bound launch of a reflection-only scene, taken out of the
deferred kernel's launch and traced by groups of G lanes per pixel (nearest_hit_coop / shadow_coop:
each lane tests some leaves, the group reduces the least (distance, object) -- the reference's
draw-order first-wins nearest hit, raytracer.rs:141-150 -- and ORs the shadow hits, :181-197).
Every frame against the CPU oracle, RGBA8 bit-identical, with the tail kernel taking up to an eighth
of the launch's tiles, over scenes whose leaf counts select G = 16, 32 and 64.  Frames are at least
2048 tiles of 8x8 (RT_ORDER_MIN_TILES, k_rows.hip): smaller launches are not calibrated or ordered."""
import numpy as np
import pytest

from tests.conftest import SCENES, scene_text
from tests.test_gpu_parity import assert_close

pytestmark = pytest.mark.gpu


def _tail_frames(text, t, W, H, depth, tiles, launches=2):
    import tinyraytracerinrust_amd as T
    rt = T.RayTracer(W, H)
    rt.max_depth = depth
    rt.load_scene(text, t, asset_dir=SCENES)
    r = rt.renderer
    r.set_kernel("deferred")
    r.set_tail_tiles(tiles)
    out = [r.render_rows_host(0, H) for _ in range(launches)]     # calibration, then ordered (tail + deferred)
    return out, r.kernel_info()


def _leaves(text, t=0.0):
    import tinyraytracerinrust_amd as T
    return T.Scene.compile(text, t, 16, 12, asset_dir=SCENES).info()["leaves"]


@pytest.mark.parametrize("name,t", [("globes", 0.0), ("globes", 0.4), ("three_cubes", 0.0), ("spinning_cube", 0.3),
                                    ("ground_star", 0.2), ("spinning_gimbals", 0.4)])
def test_tail_kernel_reference_scenes(worldmap, name, t):
    from oracle import oracle as O
    W, H, depth = 512, 384, 10
    text = scene_text(name)
    (cal, ordered), info = _tail_frames(text, t, W, H, depth, 4096)
    _, ref = O.OracleScene(text, t, W, H, max_depth=depth).render(0, H)
    assert_close(cal, None, ref, None, f"{name} calibration")
    assert_close(ordered, None, ref, None, f"{name} tail + deferred ({info}, {_leaves(text, t)} leaves)")
    # the tail kernel takes reflection-only scenes; with a transparent object the deferred kernel runs alone
    import tinyraytracerinrust_amd as T
    reflection_only = "any_transparent=0" in T.Scene.compile(text, t, W, H, asset_dir=SCENES).describe()
    assert ("tail + deferred" in info) == reflection_only, info


def _many_spheres(n):
    """n reflective spheres in a ring over a reflective floor: n + 1 leaves (G = 32 / 64; the tables must
    fit the kernel's LDS, RT_TAIL_MAX_TABLE_BYTES = 48 KB: 35 leaves of 864 bytes do, 51 do not)."""
    import math
    lines = []
    for i in range(n):
        a = 2 * math.pi * i / n
        lines.append(f"draw(sphere(<{40 * math.cos(a):.3f}, {4 + (i % 5) * 6}, {40 * math.sin(a):.3f}>, {5 + i % 3}, "
                     f"rgb({0.2 + (i % 4) * 0.2}, 0.5, {0.9 - (i % 3) * 0.3}), {0.3 + (i % 2) * 0.4}))")
    lines.append("draw(plane(<0, 1, 0>, 20, blue, 0.5))")
    return "\n".join(lines) + "\n"


@pytest.mark.parametrize("n", [24, 34])
def test_tail_kernel_many_objects(worldmap, n):
    from oracle import oracle as O
    text = _many_spheres(n)
    W, H, depth = 512, 384, 10
    (_, ordered), info = _tail_frames(text, 0.0, W, H, depth, 4096)
    _, ref = O.OracleScene(text, 0.0, W, H, max_depth=depth).render(0, H)
    assert_close(ordered, None, ref, None, f"{n} spheres tail ({_leaves(text)} leaves, {info})")
    assert "tail + deferred" in info


def test_tail_kernel_fuzz_scenes(worldmap):
    """Reflection-only random scenes of every leaf count class (G = 16 / 32 / 64)."""
    from oracle import oracle as O
    from tests.scene_fuzz import random_scene, random_rod_scene
    W, H, depth = 384, 352, 6
    seen = {}
    cases = [random_scene(s) for s in range(200, 240)] + [random_rod_scene(s) for s in range(3000, 3010)]
    import tinyraytracerinrust_amd as T
    for text in cases:
        sc = T.Scene.compile(text, 0.0, W, H, asset_dir=SCENES)
        if "any_transparent=0" not in sc.describe():
            continue                                 # the tail kernel takes reflection-only scenes
        nl = sc.info()["leaves"]
        g = 16 if nl <= 16 else 32 if nl <= 32 else 64
        if seen.get(g, 0) >= 8:
            continue
        (_, ordered), info = _tail_frames(text, 0.0, W, H, depth, 4096)
        _, ref = O.OracleScene(text, 0.0, W, H, max_depth=depth).render(0, H)
        assert_close(ordered, None, ref, None, f"fuzz tail G={g} ({nl} leaves, {info})")
        seen[g] = seen.get(g, 0) + 1
    print("tail fuzz scenes per G:", seen)
    assert 16 in seen, seen


def test_tail_kernel_rank_share_4k(worldmap):
    """A rank's share of the 4K frame at N = 8 (the tail-bound launch the kernel is for), RGB8 bands,
    at 64 (the default) and 256 tail tiles, against the oracle rows."""
    import torch
    from oracle import oracle as O
    from tinyraytracerinrust_amd import distributed as D
    import tinyraytracerinrust_amd as T
    W, H, world = 3840, 2160, 8
    rt = T.RayTracer(W, H)
    rt.load_scene(scene_text("globes"), 0.0, asset_dir=SCENES)
    r = rt.renderer
    y_first, band_rows, pitch, n_bands = D.band_params(H, world, 0, "cyclic", 8)
    rows = [y for y0, y1 in D.owned_rows(H, world, 0, "cyclic", 8) for y in range(y0, y1)]
    sc = O.OracleScene(scene_text("globes"), 0.0, W, H, max_depth=10)
    ref = np.concatenate([sc.render(y0, y1)[1] for y0, y1 in D.owned_rows(H, world, 0, "cyclic", 8)])
    for tiles in (64, 256):
        r.set_tail_tiles(tiles)
        for launch in range(2):
            slot = torch.zeros((len(rows), W, 3), dtype=torch.uint8, device="cuda")
            r.render_row_bands(y_first, band_rows, pitch, n_bands, slot)
            torch.cuda.synchronize()
            got = slot.cpu().numpy()
            assert np.array_equal(got, ref[..., :3]), \
                f"N=8 share, tail {tiles}, launch {launch}: {int((got != ref[..., :3]).sum())} channels differ ({r.kernel_info()})"
        assert "tail + deferred" in r.kernel_info()
