"""Host-side culling facts the kernels rely on (tinyraytracerinrust_amd/csrc/scene.cpp), read from
the flattener's report (rt_scene_describe): oriented object boxes (obb), the order of hit-filter
literals (order_literals) and constant hit filters (const_filters).  Each is exact by construction
(DESIGN.md §2); the pixels are compared with the oracle on the GPU (tests/test_gpu_*.py)."""
import os
import re

from tests.conftest import ROOT

SCENES = os.path.join(ROOT, "tests", "golden", "scenes")


def _dump(scene_text: str, time: float = 0.0) -> str:
    import tinyraytracerinrust_amd as T
    s = T.Scene.compile(scene_text, time, 64, 48, asset_dir=SCENES)
    assert s.status == 0, s.error
    return s.describe()


def _objects(dump: str):
    objs = []
    for line in dump.splitlines():
        m = re.match(r"object (\d+) .* obb_leaf=(-?\d+)", line)
        if m:
            objs.append({"obb": int(m.group(2)), "leaves": []})
        m = re.match(r"\s+leaf (\d+) kind=(\d+) .* lits (-?\d+) \((-?\d+) (-?\d+) (-?\d+)\) const (\d)", line)
        if m:
            n = int(m.group(3))
            objs[-1]["leaves"].append({"leaf": int(m.group(1)), "kind": int(m.group(2)),
                                       "lits": [int(m.group(4 + k)) for k in range(max(0, min(n, 3)))],
                                       "const": int(m.group(7))})
    return objs


def test_globes_oriented_boxes_and_literal_order():
    objs = _objects(_dump(open(os.path.join(SCENES, "globes.scene")).read()))
    assert len(objs) == 6
    # plane, base, support, globe: the world box is tight enough; claw and axis rod: a leaf's frame
    assert [o["obb"] >= 0 for o in objs] == [False, False, False, True, False, True]
    claw = objs[3]["leaves"]
    s20, s18, cube = (l["leaf"] for l in claw)
    assert objs[3]["obb"] == cube                               # the thin slab, not the 40-wide sphere
    # a hit on either shell: the slab test (usually failing) before the shell test (never failing)
    assert claw[0]["lits"] == [2 * cube + 1, 2 * s18 + 0]
    assert claw[1]["lits"] == [2 * cube + 1, 2 * s20 + 1]
    # a hit on the slab face: "not inside the inner sphere" fails more often than "inside the outer"
    assert claw[2]["lits"] == [2 * s18 + 0, 2 * s20 + 1]
    # the claw's filters also test the slab: not constant
    assert not any(l["const"] for o in objs for l in o["leaves"])


def test_spinning_globes_shell_filters_are_constant():
    objs = _objects(_dump(open(os.path.join(SCENES, "spinning_globes.scene")).read(), 0.3))
    shells = [o for o in objs if len(o["leaves"]) == 2]
    assert len(shells) == 3
    for o in shells:
        assert [l["const"] for l in o["leaves"]] == [1, 1]


def test_constant_filter_needs_a_radius_gap_and_one_transform():
    # a shell 0.5 thick at radius 10: above the margin (~0.02 for origins within 1e6) -> constant
    thick = "draw(csg(sphere(<0, 0, 0>, 10), sphere(<0, 0, 0>, 9.5), 'difference', red, 0, 0.5))\n"
    assert [l["const"] for l in _objects(_dump(thick))[0]["leaves"]] == [1, 1]
    # 1e-3 thick: inside the margin -> evaluated
    thin = "draw(csg(sphere(<0, 0, 0>, 10), sphere(<0, 0, 0>, 9.999), 'difference', red, 0, 0.5))\n"
    assert [l["const"] for l in _objects(_dump(thin))[0]["leaves"]] == [0, 0]
    # the same radii: no gap -> evaluated
    same = "draw(csg(sphere(<0, 0, 0>, 10), sphere(<0, 0, 0>, 10), 'difference', red, 0, 0.5))\n"
    assert [l["const"] for l in _objects(_dump(same))[0]["leaves"]] == [0, 0]
    # different centres -> evaluated
    off = "draw(csg(sphere(<0, 0, 0>, 10), sphere(<1, 0, 0>, 5), 'difference', red, 0, 0.5))\n"
    assert [l["const"] for l in _objects(_dump(off))[0]["leaves"]] == [0, 0]
    # the inner sphere under a further transform -> evaluated
    xf = ("a = sphere(<0, 0, 0>, 10)\nscale(1, 2, 1) do\n  b = sphere(<0, 0, 0>, 5)\nend\n"
          "draw(csg(a, b, 'difference', red, 0, 0.5))\n")
    assert [l["const"] for l in _objects(_dump(xf))[0]["leaves"]] == [0, 0]


def test_shadow_walk_visits_likeliest_occluders_first():
    """globes.scene has no transparent object: shadow rays only ask whether any object occludes,
    so their walk (strav) takes the largest regions first -- the globe, the claw slab, the base,
    the axis rod, the support rod -- and the unbounded floor plane last.  spinning_globes.scene
    (glass shells) keeps the draw order: its shadow product's order is the reference's."""
    def strav(dump):
        return [int(m.group(1)) for m in re.finditer(r"^strav \d+ obj=(-?\d+)", dump, re.M) if int(m.group(1)) >= 0]
    assert strav(_dump(open(os.path.join(SCENES, "globes.scene")).read())) == [4, 3, 1, 5, 2, 0]
    assert strav(_dump(open(os.path.join(SCENES, "spinning_globes.scene")).read(), 0.3)) == [0, 1, 2, 3]


def _flags(dump: str) -> dict:
    m = re.search(r"scene any_transparent=(\d) ray_chains=(\d) colour_fast=(\d) shadow_early_out=(\d)", dump)
    assert m, dump[-2000:]
    return dict(zip(("any_transparent", "ray_chains", "colour_fast", "shadow_early_out"), map(int, m.groups())))


def test_ray_chain_flag():
    """ray_chains (scene.cpp flatten): no object both transparent and reflective, so every hit spawns
    at most one ray (raytracer.rs:242-267) and the refraction kernels may take the chain form."""
    sg = _flags(_dump(open(os.path.join(SCENES, "spinning_globes.scene")).read(), 0.3))
    assert sg["any_transparent"] == 1 and sg["ray_chains"] == 1          # glass refl 0, floor transp 0
    fr = _flags(_dump(open(os.path.join(SCENES, "fractal.scene")).read()))
    assert fr["any_transparent"] == 1 and fr["ray_chains"] == 0          # spheres refl 0.4, transp 0.6
    gl = _flags(_dump(open(os.path.join(SCENES, "globes.scene")).read()))
    assert gl["any_transparent"] == 0 and gl["ray_chains"] == 1
    # -0 counts as zero, NaN as nonzero (IEEE comparisons, as the kernels test them)
    assert _flags(_dump("draw(sphere(<0, 0, 0>, 30, red, 0 * (0 - 1), 0.5))"))["ray_chains"] == 1
    assert _flags(_dump("draw(sphere(<0, 0, 0>, 30, red, 0.1, 0.5))"))["ray_chains"] == 0


def test_shadow_pow_flag():
    """shadow_pow (scene.cpp flatten): every transparency outside {+-0, 1} is one finite value, so a
    shadow ray's product (raytracer.rs:181-197) is 0 or T^count whatever the order its hits are
    found in -- the wavefront pair path's condition."""
    def pw(text, t=0.0):
        m = re.search(r"shadow_pow=(\d)", _dump(text, t))
        assert m
        return int(m.group(1))
    assert pw(open(os.path.join(SCENES, "fractal.scene")).read()) == 1           # glass 0.6, the rest 0
    assert pw(open(os.path.join(SCENES, "globes.scene")).read()) == 1            # all opaque
    assert pw(open(os.path.join(SCENES, "spinning_globes.scene")).read(), 0.3) == 1
    assert pw("draw(sphere(<0, 0, 0>, 30, red, 0, 0.5))\ndraw(sphere(<0, 9, 0>, 3, red, 0, 1))") == 1
    assert pw("draw(sphere(<0, 0, 0>, 30, red, 0, 0.5))\ndraw(sphere(<0, 9, 0>, 3, red, 0, 0.25))") == 0
    # -0 is a zero factor (the product is 0 at it, whatever the order); 1 is skipped
    assert pw("draw(sphere(<0, 0, 0>, 30, red, 0, 0.5))\ndraw(sphere(<0, 9, 0>, 3, red, 0, 0 * (0 - 1)))") == 1
    assert pw("draw(sphere(<0, 0, 0>, 30, red, 0, 0.5))\ndraw(sphere(<0, 9, 0>, 3, red, 0, 0.5))\n"
              "draw(sphere(<9, 0, 0>, 3, red, 0, 1))") == 1
    # |T| > 1 with an opaque object: T^k may overflow to inf and inf * 0 is NaN, so the draw-order
    # product depends on where the zero factor comes -- not order-free
    assert pw("draw(sphere(<0, 0, 0>, 30, red, 0, 2))\ndraw(sphere(<0, 9, 0>, 3, red, 0, 0))") == 0
    assert pw("draw(sphere(<0, 0, 0>, 30, red, 0, 0 - 2))\ndraw(sphere(<0, 9, 0>, 3, red, 0, 0))") == 0
    # |T| > 1 without one: every factor is T, the product is T^k in any order
    assert pw("draw(sphere(<0, 0, 0>, 30, red, 0, 2))\ndraw(sphere(<0, 9, 0>, 3, red, 0, 2))") == 1
    # |T| <= 1: T^k only underflows, to a zero that stays zero
    assert pw("draw(sphere(<0, 0, 0>, 30, red, 0, 0 - 1))\ndraw(sphere(<0, 9, 0>, 3, red, 0, 0))") == 1
