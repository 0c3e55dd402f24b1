"""CPU checks of the oracle's probes that the GPU edge tests aim with (oracle/rt_oracle.c
orc_hit_signature, orc_texel_probe): they must agree with the oracle's own renders."""
import math

import numpy as np

from tests.test_gpu_cull_edges import CUBES, _edges


def test_hit_signature_matches_render_and_finds_edges():
    from oracle import oracle as O
    W, H = 192, 108
    osc = O.OracleScene(CUBES, 0.0, W, H, max_depth=0)
    f64, _ = osc.render(0, H, f64=True)
    sig = np.array([[osc.hit_signature(x, y) for x in range(W)] for y in range(H)])
    assert (sig == -1).any() and (sig == 1).any()                     # sky and floor (object 0)
    assert np.all((sig == -1) == (f64[..., :3] == 0).all(axis=2))    # a miss is black (raytracer.rs:152-160)
    lit = sig[sig > 0] // 4096                                       # occluded-light masks (3 lights: test light first)
    assert lit.min() >= 0 and lit.max() < 8 and len(np.unique(lit)) >= 3
    # bisected edges end on adjacent doubles with different signatures
    osc2 = O.OracleScene(CUBES, 0.0, 1920, 1080, max_depth=0)
    pairs = _edges(osc2, 1920, 1080, True, n_lines=4, step=4.0, cap=20)
    assert len(pairs) >= 8
    for lo, hi, c in pairs:
        assert math.nextafter(lo, hi) == hi
        assert osc2.hit_signature(lo, c) != osc2.hit_signature(hi, c)
