"""Seeded random scenes in the reference's DSL (sceneparser grammar: sphere / cube / plane, csg,
translate / rotate / scale blocks, materials with reflectivity and transparency, appended lights,
camera), for parity fuzzing of the product path against the oracle (tests/test_gpu_fuzz.py).

The generator leans on the cases the kernels special-case, so each exact shortcut meets scenes it
must not change: concentric sphere pairs under one transform (RtLeaf::share_prev and the dropped
leaf box tests), axis-aligned and tilted planes (RtLeaf::plane_axis), transparent objects (the
refraction kernel), nested CSG (literal and postfix hit filters), colours outside [0, 1] and
reflectivities above 1 (the compare/select clamps), diagonal and full transforms."""
import random

_COLOURS = ["red", "blue", "white"]


def _num(r, lo, hi, nd=2):
    return round(r.uniform(lo, hi), nd)


def _vec(r, lo, hi):
    return f"<{_num(r, lo, hi)}, {_num(r, lo, hi)}, {_num(r, lo, hi)}>"


def _colour(r, odd):
    k = r.random()
    if odd and k < 0.1:
        return f"{r.choice(_COLOURS)} * (0 - {_num(r, 0.1, 0.9)})"          # negative channel
    if odd and k < 0.2:
        return f"rgb({_num(r, 0, 1.6)}, {_num(r, 0, 1.6)}, {_num(r, 0, 1.6)})"
    if k < 0.5:
        return f"{r.choice(_COLOURS)} * {_num(r, 0.2, 1.0)}"
    return f"rgb({_num(r, 0, 1)}, {_num(r, 0, 1)}, {_num(r, 0, 1)})"


_CHAINS = [False]      # random_scene(chains=True): no object both transparent and reflective


def _material(r, odd, allow_transp=True):
    refl = r.choice([0, 0, 0.2, 0.5, 0.8] + ([1.3] if odd else []))
    transp = r.choice([0, 0, 0, 0.5, 0.9]) if allow_transp else 0
    if _CHAINS[0] and transp != 0:
        refl = 0                  # every hit spawns at most one ray (scene.cpp ray_chains)
    return f"{_colour(r, odd)}, {refl}, {transp}"


def _transform(r):
    k = r.random()
    if k < 0.3:
        return f"translate({_num(r, -20, 20)}, {_num(r, -10, 10)}, {_num(r, -10, 20)})"
    if k < 0.6:
        return f"rotate({_num(r, -3.1, 3.1)}, {_num(r, -3.1, 3.1)}, {_num(r, -3.1, 3.1)})"
    if k < 0.8:
        return f"scale({_num(r, 0.3, 2)}, {_num(r, 0.3, 2)}, {_num(r, 0.3, 2)})"
    return None


def _primitive(r, name):
    k = r.random()
    if k < 0.55:
        return f"{name} = sphere({_vec(r, -15, 15)}, {_num(r, 3, 14)})"
    return f"{name} = cube({_vec(r, -15, 15)}, {_num(r, 4, 20)})"


def random_scene(seed: int, chains: bool = False) -> str:
    """chains=True: transparent objects get reflectivity 0, so the scene's rays form chains (the
    refraction chain kernels: rt_device.h trace, RT_MODE_CHAIN and the deferred REFR path)."""
    _CHAINS[0] = chains
    try:
        return _random_scene(seed)
    finally:
        _CHAINS[0] = False


def _random_scene(seed: int) -> str:
    r = random.Random(seed)
    odd = r.random() < 0.3
    lines = []
    n = r.randint(2, 5)
    for i in range(n):
        t = _transform(r)
        body = []
        kind = r.random()
        if kind < 0.3:                                   # concentric sphere shells (shared terms)
            c = _vec(r, -12, 12)
            rad = _num(r, 6, 15)
            body.append(f"a{i} = sphere({c}, {rad})")
            body.append(f"b{i} = sphere({c}, {round(rad * r.uniform(0.5, 0.9), 2)})")
            if r.random() < 0.4:
                body.append(f"c{i} = sphere({c}, {round(rad * r.uniform(0.2, 0.45), 2)})")
                body.append(f"s{i} = csg(csg(a{i}, b{i}, 'difference'), c{i}, 'union', {_material(r, odd)})")
            else:
                body.append(f"s{i} = csg(a{i}, b{i}, '{r.choice(['difference', 'intersection', 'union'])}', {_material(r, odd)})")
        elif kind < 0.55:                                # CSG of two unrelated primitives
            body.append(_primitive(r, f"a{i}"))
            body.append(_primitive(r, f"b{i}"))
            body.append(f"s{i} = csg(a{i}, b{i}, '{r.choice(['difference', 'intersection', 'union'])}', {_material(r, odd)})")
        elif kind < 0.8:
            if r.random() < 0.5:
                body.append(f"s{i} = sphere({_vec(r, -15, 15)}, {_num(r, 3, 14)}, {_material(r, odd)})")
            else:
                body.append(f"s{i} = cube({_vec(r, -15, 15)}, {_num(r, 4, 20)}, {_material(r, odd)})")
        else:                                            # a plane: axis-aligned or tilted
            nrm = r.choice(["<0, 1, 0>", "<1, 0, 0>", "<0, 0, -1>", f"<{_num(r, -1, 1)}, 1, {_num(r, -1, 1)}>"])
            body.append(f"s{i} = plane({nrm}, {_num(r, 20, 60)}, {_material(r, odd, allow_transp=False)})")
        if t:
            lines.append(f"{t} do")
            lines += ["  " + b for b in body]
            lines.append("end")
        else:
            lines += body
        lines.append(f"draw(s{i})")
    for _ in range(r.randint(0, 2)):
        lines.append(f"append light({_vec(r, -40, 40)}, {r.choice(_COLOURS)} * {_num(r, 0.3, 1)}, 100)")
    lines.append(f"set camera(<{_num(r, -20, 20)}, {_num(r, 0, 25)}, {_num(r, -110, -70)}>)")
    return "\n".join(lines) + "\n"


def random_rod_scene(seed: int) -> str:
    """Scenes built like globes.scene's axis rod and claw: a primitive scaled into a thin rod or
    slab, intersected with (or cut from) another primitive, under nested rotate / translate blocks.
    Their world boxes are loose, so the kernels' oriented object boxes (scene.cpp obb) cull these
    objects in the leaf's own frame; the margins of that test meet grazing rays, rods seen end-on
    and shadow rays along the rod here.  Opaque materials only (the reflection-only kernels take
    the oriented boxes), reflective floors so secondary rays cross the rods too."""
    r = random.Random(seed)
    lines = [f"draw(plane(<0, 1, 0>, {_num(r, 20, 30)}, {_colour(r, False)}, {r.choice([0.2, 0.5])}))"]
    for i in range(r.randint(2, 4)):
        thin = [round(r.uniform(0.03, 0.15), 3), round(r.uniform(5, 100), 1), 1]
        r.shuffle(thin)
        lines.append(f"translate({_num(r, -15, 15)}, {_num(r, -8, 12)}, {_num(r, -10, 20)}) do")
        lines.append(f"  rotate({_num(r, -3.1, 3.1)}, {_num(r, -3.1, 3.1)}, {_num(r, -3.1, 3.1)}) do")
        lines.append(f"    scale({thin[0]}, {thin[1]}, {thin[2]}) do")
        rod = f"sphere({_num(r, 0.5, 3)})" if r.random() < 0.5 else f"cube({_num(r, 1, 6)})"
        lines.append(f"      a{i} = {rod}")
        lines.append("    end")
        other = f"cube({_num(r, 10, 40)})" if r.random() < 0.6 else f"sphere({_num(r, 8, 20)})"
        op = r.choice(["intersection", "intersection", "difference"])
        if op == "difference":                          # the rod is a: every hit lies inside it
            lines.append(f"    s{i} = csg(a{i}, {other}, 'difference', {_material(r, False, allow_transp=False)})")
        else:
            lines.append(f"    s{i} = csg({other}, a{i}, 'intersection', {_material(r, False, allow_transp=False)})")
        lines.append("  end")
        lines.append("end")
        lines.append(f"draw(s{i})")
    if r.random() < 0.5:
        lines.append(f"draw(sphere(<{_num(r, -10, 10)}, {_num(r, -5, 10)}, {_num(r, 0, 20)}>, {_num(r, 5, 12)}, "
                     f"{_material(r, False, allow_transp=False)}))")
    for _ in range(r.randint(0, 2)):
        lines.append(f"append light({_vec(r, -40, 40)}, {r.choice(_COLOURS)} * {_num(r, 0.3, 1)}, 100)")
    lines.append(f"set camera(<{_num(r, -20, 20)}, {_num(r, 0, 25)}, {_num(r, -110, -70)}>)")
    return "\n".join(lines) + "\n"
