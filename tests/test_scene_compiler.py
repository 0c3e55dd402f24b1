"""The product's host scene front end (rt_scene_compile: DSL -> rt_scene) against the oracle's
load_scene restatement: object/light counts, lights, camera, error semantics.  CPU only."""
import numpy as np
import pytest

from tests.conftest import SCENES, scene_text

ALL = ["globes", "spinning_globes", "three_cubes", "spinning_cube", "ground_star", "spinning_gimbals", "fractal"]


@pytest.mark.parametrize("name", ALL)
@pytest.mark.parametrize("time", [0.0, 0.37])
def test_compile_matches_oracle(worldmap, name, time):
    import tinyraytracerinrust_amd as T
    from oracle import oracle as O
    text = scene_text(name)
    s = T.Scene.compile(text, time, 320, 200, asset_dir=SCENES)
    o = O.OracleScene(text, time, 320, 200)
    info = s.info()
    assert info["objects"] == o.n_objects and info["lights"] == o.n_lights
    cam = s.camera()
    oc = o.camera()
    assert cam["center"] == list(oc[0:3]) and cam["direction"] == list(oc[3:6])
    assert cam["right"] == list(oc[6:9]) and cam["aspect"] == oc[9]
    for i in range(info["lights"]):
        p, c = s.light(i)
        ol = o.light(i)
        assert p == list(ol[0:3]) and c == list(ol[3:7])


def test_camera_transformed_twice():
    """SetCamera transforms the position, then set_camera_from_vector transforms it again
    (ast_node.rs:257-262, raytracer.rs:291-294)."""
    import tinyraytracerinrust_amd as T
    s = T.Scene.compile("translate(0, 5, 0) set camera(<0, 0, -100>)", 0.0, 64, 48)
    assert s.camera()["center"] == [0.0, 10.0, -100.0]


def test_parse_error_gives_default_scene():
    import tinyraytracerinrust_amd as T
    with pytest.raises(T.RtError) as e:
        T.Scene.compile("draw(sphere(\t1))", 0.0, 8, 8)
    assert e.value.status == -2
    s = T.Scene.compile("draw(sphere(\t1))", 0.0, 8, 8, strict=False)
    assert s.status == -2 and s.info()["objects"] == 0 and s.info()["lights"] == 1
    assert s.camera()["center"] == [0.0, 0.0, -100.0]


@pytest.mark.parametrize("text,status", [
    ("x = 3 % 2", -3), ("draw(y)", -3), ("display(sphere(1))", -3),
    ("draw(csg(sphere(1), 'intersection'))", -3), ("if 1 then draw(sphere(1)) end", -2),
    ("draw(sphere(texture('nope.png')))", -4), ("call f()", -3),
])
def test_error_status(text, status):
    import tinyraytracerinrust_amd as T
    with pytest.raises(T.RtError) as e:
        T.Scene.compile(text, 0.0, 8, 8, asset_dir=SCENES)
    assert e.value.status == status


def test_builder_vs_dsl_structure():
    """The Rust host's builder path and the DSL path yield the same scene content."""
    import tinyraytracerinrust_amd as T
    rt = T.RayTracer(64, 48)
    rt.add_test_objects()
    rt.add_light((0, 0, -35), (0.5, 0.5, 0.5, 0.5), 100)
    rt.transformation_stack.push_transformation(T.MatrixTransformation.create_translation_matrix(0, 2, 0))
    rt.set_camera_from_vector((0, 10, -85))
    dsl = T.Scene.compile("append light(<0, 0, -35>, white * 0.5, 100) translate(0, 2, 0) do "
                          "set camera(<0, 8, -85>) end", 0.0, 64, 48)
    assert rt.scene.camera() == dsl.camera()
    assert rt.scene.light(1) == dsl.light(1)


def test_scene_info_leaves(worldmap):
    import tinyraytracerinrust_amd as T
    info = T.Scene.compile(scene_text("globes"), 0.0, 64, 48, asset_dir=SCENES).info()
    assert info == {"objects": 6, "lights": 2, "leaves": 11, "width": 64, "height": 48}


def _check_traversal(nodes, n_objects):
    """Pre-order hierarchy invariants: object nodes in draw order, each object once, every
    group's skip closes its subtree (nodes i+1 .. skip-1 are its descendants)."""
    objs = [o for o, _ in nodes if o >= 0]
    assert objs == list(range(n_objects))
    stack = []
    for i, (o, skip) in enumerate(nodes):
        while stack and stack[-1] <= i:
            stack.pop()
        assert skip > i and skip <= len(nodes)
        assert all(skip <= s for s in stack), "subtree escapes its parent group"
        if o < 0:
            assert skip > i + 1, "empty group"
            stack.append(skip)
        else:
            assert skip == i + 1


@pytest.mark.parametrize("name", ALL)
def test_traversal_hierarchy(worldmap, name):
    import tinyraytracerinrust_amd as T
    s = T.Scene.compile(scene_text(name), 0.0, 64, 48, asset_dir=SCENES)
    _check_traversal(s.traversal(), s.info()["objects"])


def test_traversal_globes_groups(worldmap):
    """globes.scene: the unbounded floor plane is visited alone; the five bounded objects sit
    under one group (a ray that misses the whole assembly tests one box instead of five)."""
    import tinyraytracerinrust_amd as T
    nodes = T.Scene.compile(scene_text("globes"), 0.0, 64, 48, asset_dir=SCENES).traversal()
    assert nodes[0] == (0, 1)
    assert nodes[1] == (-1, len(nodes))


def test_traversal_huge_coordinates_not_grouped():
    """Boxes beyond the proven culling range (1e6) are never culled, hence never grouped."""
    import tinyraytracerinrust_amd as T
    s = T.Scene.compile("draw(sphere(<0, 0, 2000000>, 1500000, red))\ndraw(sphere(<0, 0, 0>, 5, red))\n"
                        "draw(sphere(<10, 0, 0>, 5, red))", 0.0, 64, 48)
    nodes = s.traversal()
    assert nodes[0] == (0, 1)
    _check_traversal(nodes, 3)
