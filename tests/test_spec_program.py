"""The scene-specialised program (tinyraytracerinrust_amd/csrc/spec.hip, RT_OPT_SPECIALIZE) on the CPU:
its text carries the flattened scene's records bit for bit, and hipRTC compiles it without a device
(rt_scene_precompile).  The pixels it renders are checked on the GPU (tests/test_gpu_spec.py)."""
import re
import struct

from tests.conftest import SCENES, scene_text


def _scene(text, t=0.0, w=64, h=48):
    import tinyraytracerinrust_amd as T
    s = T.Scene.compile(text, t, w, h, asset_dir=SCENES)
    assert s.status == 0, s.error
    return s


def test_program_holds_the_flattened_tables():
    s = _scene(scene_text("globes"))
    prog = s.spec_program()
    m = re.search(r"N_OBJECTS = (\d+), N_LIGHTS = (\d+), N_TRAV = (\d+), N_STRAV = (\d+)", prog)
    assert m and int(m.group(1)) == 6 and int(m.group(2)) == 2
    trav = [(o, k) for o, k in s.traversal()]
    assert int(m.group(3)) == len(trav)
    # every RtTrav record's obj / skip words (bytes 48..55) equal the traversal the kernels walk
    rows = re.search(r"constexpr RtTrav TRAV\[\] = \{(.*?)\};", prog, re.S).group(1)
    words = [[int(w, 16) for w in re.findall(r"0x([0-9a-f]+)ull", r)] for r in rows.strip().splitlines()]
    assert len(words) == len(trav)
    for (o, k), w in zip(trav, words):
        obj, skip = struct.unpack("<ii", struct.pack("<Q", w[6]))
        assert (obj, skip) == (o, k)
    # reflection-only scene: megakernel and deferred kernels, f64 and calibration forms
    for k in ("rt_spec_rows_00", "rt_spec_rows_11", "rt_spec_def_00", "rt_spec_def_11"):
        assert f"void {k}(" in prog
    # a refraction-chain scene has no deferred kernels in its program
    assert "rt_spec_def_" not in _scene(scene_text("spinning_globes"), 0.3).spec_program()


def test_precompile_without_a_device_and_cache():
    s = _scene("draw(sphere(<0, 0, 0>, 30, red))")
    ms = s.precompile()
    assert ms > 0.0
    assert s.precompile() == 0.0                      # the process cache has every program now


def test_scene_family_programs():
    """rt_spec_family_register: the frames of spinning_globes.scene fall into families of the same
    hierarchy; every member's program is its family's (one text, so one compile), the varying words
    are masked (VARY_*) and zeroed, the shared ones carried bit for bit; other scenes keep their own."""
    import tinyraytracerinrust_amd as T
    text = scene_text("spinning_globes")
    frames = [_scene(text, f / 12) for f in range(12)]
    T.Scene.clear_families()
    try:
        assert T.Scene.register_family(frames + [_scene(scene_text("globes"))]) >= 0.0
        progs = [s.spec_program() for s in frames]
        assert all("#define RT_SPEC_FAMILY 1" in p for p in progs)
        assert 1 <= len(set(progs)) <= 3, len(set(progs))
        vary = re.search(r"VARY_OBJECTS\[\] = \{([^}]*)\}", progs[0]).group(1).split(",")
        assert len(vary) == 4 * 192 // 4 and 0 < vary.count("1") < len(vary)
        assert "RT_SPEC_FAMILY" in _scene(scene_text("globes")).spec_program()    # a family of one
        # the exact program of a frame carries its own values where the family's has zeros
        T.Scene.clear_families()
        assert "RT_SPEC_FAMILY" not in frames[3].spec_program()
    finally:
        T.Scene.clear_families()
