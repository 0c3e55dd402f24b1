"""The parity-fuzzing scenes (tests/scene_fuzz.py) are valid input for both front ends: the
product's rt_scene_compile and the oracle's parser accept every one, and their camera and light
lists agree (the pixels themselves are compared on the GPU, tests/test_gpu_fuzz.py)."""
import pytest

from tests.scene_fuzz import random_scene


@pytest.mark.parametrize("seed", list(range(160)) + list(range(1000, 1012)))
def test_fuzz_scene_compiles_in_both_front_ends(seed):
    import tinyraytracerinrust_amd as T
    from oracle import oracle as O
    text = random_scene(seed)
    assert random_scene(seed) == text                      # seeded: the same text every time
    sc = T.Scene.compile(text, 0.0, 16, 12)
    assert sc.status == 0, sc.error
    o = O.OracleScene(text, 0.0, 16, 12, max_depth=2)
    _, u8 = o.render(0, 12)
    assert u8.shape == (12, 16, 4)
    assert o.status == 0, o.error
    assert sc.info()["lights"] == o.n_lights and sc.info()["objects"] == o.n_objects
