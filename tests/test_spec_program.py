"""The scene-specialised program (tinyraytracerinrust_amd/csrc/spec.hip, RT_OPT_SPECIALIZE) on the CPU:
its text carries the flattened scene's records bit for bit, and hipRTC compiles it without a device
(rt_scene_precompile).  The pixels it renders are checked on the GPU (tests/test_gpu_spec.py)."""
import os
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
    for k in ("rt_spec_rows_00", "rt_spec_rows_11", "rt_spec_def_00", "rt_spec_def_11", "rt_spec_prim_00", "rt_spec_prim_11"):
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
        assert len(vary) % 4 == 0 and len(vary) // 4 >= 48 and 0 < vary.count("1") < len(vary)   # 4 objects, one mask word per 4 bytes
        # a scene of a structure of its own ("a family of one") keeps its own, exact program -- compiled
        # by the registration (every word a constant: globes.scene's family form spilled 1 392 B/lane)
        g = _scene(scene_text("globes"))
        assert "RT_SPEC_FAMILY" not in g.spec_program() and g.precompile() == 0.0
        # the exact program of a frame carries its own values where the family's has zeros
        T.Scene.clear_families()
        assert "RT_SPEC_FAMILY" not in frames[3].spec_program()
    finally:
        T.Scene.clear_families()


def _report(text):
    """rt_scene_spec_report lines as {kernel: {field: value}} plus the compiler line."""
    out, comp = {}, None
    for line in _scene(text).spec_report().splitlines():
        if line.startswith("compiler: "):
            comp = line
            continue
        name, rest = line.split(": ", 1)
        f = rest.split()
        out[name] = {f[i]: f[i + 1] for i in range(0, len(f) - 1, 2)}
    return comp, out


def test_compiler_origin_and_resources_after_torch():
    """The programs compile with the ROCm installation's hipRTC even when PyTorch -- which bundles
    an older hipRTC / comgr (LLVM 20) under the same sonames -- was imported first (round 4: the family
    program built by torch's copy ran 19x slower, profiles/r05v_family_compilers.txt), and the code
    objects stay inside the resource guard's bounds.  A fresh interpreter, torch imported first."""
    import json
    import subprocess
    import sys
    from tests.conftest import ROOT
    code = ("import torch, json, sys; sys.path.insert(0, %r)\n"
            "import tinyraytracerinrust_amd as T\n"
            "ident, rocm = T.spec_compiler_info()\n"
            "s = T.Scene.compile('draw(sphere(<0, 0, 0>, 30, red))', 0.0, 64, 48)\n"
            "print(json.dumps({'ident': ident, 'rocm': rocm, 'report': s.spec_report()}))\n" % ROOT)
    env = dict(os.environ, RT_SPEC_CACHE_DIR="")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    rocm_root = os.environ.get("ROCM_PATH") or "/opt/rocm"
    assert d["rocm"] and d["ident"].startswith(rocm_root + "/lib/libhiprtc.so.7"), d["ident"]
    rows = [l for l in d["report"].splitlines() if l.startswith("rt_spec_rows_00:")]
    assert rows, d["report"]
    f = rows[0].split()
    v = {f[i]: f[i + 1] for i in range(1, len(f) - 1, 2)}
    assert int(v["vgprs"]) <= 128 and int(v["scratch"]) <= 1024 and v["source"] == "hiprtc", rows[0]


def test_guard_bounds_hold_for_the_benchmark_programs():
    """The resource guard (spec.hip RT_SPEC_MAX_*) accepts the programs the benchmark configs run --
    globes.scene's megakernel and deferred kernel -- and reports what hipRTC built."""
    comp, ks = _report(scene_text("globes"))
    assert "ROCm installation" in comp, comp
    assert set(ks) == {"rt_spec_rows_00", "rt_spec_def_00", "rt_spec_prim_00"}, ks
    assert int(ks["rt_spec_prim_00"]["scratch"]) == 0         # no frame stack in the primary-ray kernel
    assert int(ks["rt_spec_rows_00"]["vgprs"]) <= 128 and int(ks["rt_spec_rows_00"]["scratch"]) <= 1024
    assert int(ks["rt_spec_def_00"]["scratch"]) <= 2048


def test_disk_cache_keyed_and_checked_by_text(tmp_path):
    """rt_spec_cache_dir: a program compiled in one process is read back by another (no hipRTC run), and
    an entry whose stored program text does not match is ignored (recompiled), never trusted on its
    file name (a hash)."""
    import subprocess
    import sys
    from tests.conftest import ROOT
    text = "draw(sphere(<1, 2, 3>, 29.5, blue))"          # a program no other test compiles
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import tinyraytracerinrust_amd as T\n"
            "s = T.Scene.compile(%r, 0.0, 64, 48)\n"
            "print(s.spec_report())\n" % (ROOT, text))
    env = dict(os.environ, RT_SPEC_CACHE_DIR=str(tmp_path))

    def run():
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        return [l for l in r.stdout.splitlines() if l.startswith("rt_spec_rows_00:")][0]
    assert "source hiprtc" in run()
    files = list(tmp_path.glob("spec_*.rtco"))
    assert len(files) == 3                                 # a reflection-only scene: megakernel, deferred, primary-ray
    assert "source disk" in run()                          # another process: from the disk cache
    rows = [f for f in files if b"void rt_spec_rows_00(" in f.read_bytes()][0]
    blob = bytearray(rows.read_bytes())
    i = blob.find(b"constexpr RtObject OBJECTS")
    assert i > 0
    blob[i + 40] ^= 1                                      # the stored text no longer matches
    rows.write_bytes(bytes(blob))
    assert "source hiprtc" in run()                        # recompiled (and rewritten)
    assert "source disk" in run()


def test_family_count_is_bounded():
    """rt_spec_family_register compiles one program per family: scenes of more distinct structures than
    RT_SPEC_MAX_FAMILIES (16) are refused before anything compiles."""
    import tinyraytracerinrust_amd as T
    scenes = [_scene(" ".join(f"draw(sphere(<{3 * i}, 0, 0>, 1, red))" for i in range(n))) for n in range(1, 19)]
    try:
        T.Scene.register_family(scenes)
        raise AssertionError("17+ families accepted")
    except T.RtError as e:
        assert e.status == -6 and "families" in e.message, e.message


def _fnv1a(b):
    h = 1469598103934665603
    for ch in b:
        h = ((h ^ ch) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def test_disk_cache_identity_covers_headers_and_options(tmp_path):
    """the program text only #includes rt_device.h / rt_blob.h / rt_math.h, which the
    library embeds, so the disk-cache identity must cover them (and the compile options): it ends in
    "build H" with H = FNV-1a over the three embedded headers and the options, here recomputed from the
    sources, and an entry written under another build's identity is recompiled, not read."""
    import subprocess
    import sys
    import tinyraytracerinrust_amd as T
    from tests.conftest import ROOT
    ident, rocm = T.spec_compiler_info()
    m = re.search(r" build ([0-9a-f]{16})$", ident)
    assert m, ident
    key = b""
    for h in ("rt_device", "rt_blob", "rt_math"):
        with open(os.path.join(ROOT, "tinyraytracerinrust_amd", "csrc", h + ".h"), "rb") as f:
            key += f.read() + b"\0"
    for o in ("--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-mllvm",
              "-disable-machine-licm"):
        key += o.encode() + b"\0"
    assert int(m.group(1), 16) == _fnv1a(key), "the embedded headers differ from csrc/ (rebuild the library)"

    text = "draw(sphere(<1, 2, 4>, 28.5, green))"          # a program no other test compiles
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import tinyraytracerinrust_amd as T\n"
            "s = T.Scene.compile(%r, 0.0, 64, 48)\n"
            "print(s.spec_report())\n" % (ROOT, text))
    env = dict(os.environ, RT_SPEC_CACHE_DIR=str(tmp_path))

    def run():
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        return [l for l in r.stdout.splitlines() if l.startswith("rt_spec_rows_00:")][0]
    assert "source hiprtc" in run()
    rows = [f for f in tmp_path.glob("spec_*.rtco") if b"void rt_spec_rows_00(" in f.read_bytes()][0]
    blob = bytearray(rows.read_bytes())
    assert blob[:9] == b"RTSPEC03\n"
    i = blob.find((" build " + m.group(1)).encode())
    assert i > 0                                           # the entry carries the build identity
    blob[i + 7] = ord("0") if blob[i + 7] != ord("0") else ord("1")   # another build's headers
    rows.write_bytes(bytes(blob))
    assert "source hiprtc" in run()                        # not read: recompiled (and rewritten)
    assert "source disk" in run()
