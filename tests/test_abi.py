"""The C-ABI library: it loads, exports exactly what include/rt_abi.h declares, and its
host-side (no-GPU) entry points behave.  CPU only -- no compute launches here."""
import ctypes
import os
import re

import numpy as np
import pytest

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "rt_abi.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    import tinyraytracerinrust_amd as T
    lib = T.lib()
    names = declared()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"declared but not exported: {missing}"


def test_python_binding_covers_header():
    from tinyraytracerinrust_amd import _lib
    assert sorted(_lib.SIGNATURES) == declared()


def test_exports_are_extern_c():
    """No C++-mangled rt_ symbols: the Rust host links these names verbatim."""
    import subprocess
    so = os.path.join(ROOT, "tinyraytracerinrust_amd", "librt_mi355x.so")
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if l.split()[-1].startswith("rt_")}
    assert set(declared()) <= exported


def test_version_and_errors():
    import tinyraytracerinrust_amd as T
    lib = T.lib()
    assert lib.rt_abi_version() == 1
    h = ctypes.c_void_p()
    assert lib.rt_scene_new(0, 10, ctypes.byref(h)) == -1          # RT_ERR_INVALID
    assert b"frame size" in lib.rt_last_error()
    assert lib.rt_scene_add_test_objects(None) == -1
    assert lib.rt_render_rows(None, 0, 1, -1, None, 0, None) == -1
    with pytest.raises(T.RtError) as e:
        T.Scene.compile("draw(sphere(1, 2, 3, 4))", 0.0, 8, 8)
    assert e.value.status == -3


def test_transformations_match_reference_math():
    """rt_xform_* against the Python restatement's matrices, bit for bit."""
    import tinyraytracerinrust_amd as T
    from oracle import pyref as P
    MT = T.MatrixTransformation
    cases = [(MT.create_rotation_matrix(0.3, 1.1, -0.7), P.MatrixTransformation.rotation(0.3, 1.1, -0.7)),
             (MT.create_translation_matrix(1.5, -2, 3), P.MatrixTransformation.translation(1.5, -2.0, 3.0)),
             (MT.create_scaling_matrix(0.05, 1, 3), P.MatrixTransformation.scaling(0.05, 1.0, 3.0))]
    a = MT.create_rotation_matrix(0.3, 0, 0).compose_with(MT.create_translation_matrix(0, 5, 0))
    b = P.MatrixTransformation.rotation(0.3, 0.0, 0.0).compose_with(P.MatrixTransformation.translation(0.0, 5.0, 0.0))
    cases.append((a, b))
    for t, r in cases:
        assert np.array_equal(t.matrix, np.array(r.m))
        assert np.array_equal(t.inverse_matrix, np.array(r.inv))


def test_stack_mirror():
    import tinyraytracerinrust_amd as T
    st = T.TransformationStack()
    st.push_transformation(T.MatrixTransformation.create_translation_matrix(0, 5, 0))
    st.push_transformation(T.MatrixTransformation.create_scaling_matrix(2, 2, 2))
    assert np.allclose(st.get_transformation().transform_vector([1, 1, 1]), [2, 7, 2])
    st.pop_transformation()
    st.pop_transformation()
    assert np.array_equal(st.get_transformation().matrix, np.eye(4))


def test_no_gpu_fails_loudly():
    """Without a HIP device the render path raises: there is no CPU fallback."""
    import torch
    import tinyraytracerinrust_amd as T
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(T.RtError) as e:
        T.Renderer(0)
    assert e.value.status == -5
    with pytest.raises(T.RtError):                  # own-queue streams need a device too
        T.HwStream(0)


def _header_arity():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(rt_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", src, flags=re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_integration_rust_block_matches_header():
    """INTEGRATION.md's Rust `extern "C"` block declares every header export with the same
    number of parameters (the binding a Rust maintainer would paste)."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r'extern "C" \{(.*?)\n\}', doc, flags=re.S)
    assert blocks, "no extern block"
    rust = {}
    for m in re.finditer(r"pub fn (rt_[a-z0-9_]+)\s*\((.*?)\)\s*(->[^;]*)?;", blocks[0], flags=re.S):
        args = re.sub(r"//[^\n]*", "", m.group(2)).strip()
        rust[m.group(1)] = 0 if not args else args.rstrip(",").count(",") + 1
    hdr = _header_arity()
    assert sorted(hdr) == declared()
    assert rust == hdr


def test_one_hip_runtime_per_process():
    """Loading the library before torch must not start a second HIP runtime: torch wheels bundle
    their own libamdhip64 / libhsa-runtime64, and with /opt/rocm's copies loaded first torch finds
    no device.  _lib.lib() imports torch first, so exactly one libamdhip64 is mapped."""
    import subprocess
    import sys
    code = ("import re, tinyraytracerinrust_amd as T; T.lib(); import torch; "
            "m = open('/proc/self/maps').read(); "
            "print(len(set(re.findall(r'(\\S*libamdhip64\\S*)', m))), len(set(re.findall(r'(\\S*libhsa-runtime64\\S*)', m))))")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    assert p.stdout.split() == ["1", "1"], p.stdout
