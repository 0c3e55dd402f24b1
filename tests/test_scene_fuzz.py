"""The parity-fuzzing scenes (tests/scene_fuzz.py) are valid input for both front ends: the
product's rt_scene_compile and the oracle's parser accept every one, and their camera and light
lists agree (the pixels themselves are compared on the GPU, tests/test_gpu_fuzz.py)."""
import pytest

from tests.scene_fuzz import random_rod_scene, random_scene


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


@pytest.mark.parametrize("seed", list(range(3000, 3048)) + list(range(3100, 3106)))
def test_rod_scene_compiles_in_both_front_ends(seed):
    """The thin rotated rod / slab scenes (random_rod_scene) as well, and the host gives their rod
    objects oriented boxes (scene.cpp obb, reported by rt_scene_describe's object lines)."""
    import tinyraytracerinrust_amd as T
    from oracle import oracle as O
    text = random_rod_scene(seed)
    sc = T.Scene.compile(text, 0.0, 16, 12)
    assert sc.status == 0, sc.error
    o = O.OracleScene(text, 0.0, 16, 12, max_depth=2)
    o.render(0, 12)
    assert o.status == 0, o.error
    assert sc.info()["lights"] == o.n_lights and sc.info()["objects"] == o.n_objects
    if seed == 3000:
        d = sc.describe()
        assert sum("obb_leaf=" in l and "obb_leaf=-1" not in l for l in d.splitlines()) >= 2
