"""Host-side mirror of the reference's render-path interface, over the C ABI.

Mirrors the names and argument meaning of the reference (andreivasiliu/TinyRaytracerInRust):

* ``MatrixTransformation`` / ``TransformationStack``  -- src/raytracer/transformation.rs:7-205
* ``RayTracer``  -- src/raytracer/raytracer.rs:21-364 (new_default, add_test_objects, add_object,
  add_light, set_camera_from_vector, get_pixel, max_depth) plus the DebugWindow row loop
  ``render_lines`` (src/raydebugger/debug_window.rs:74-87) and ``load_scene``
  (src/sceneparser/scene_loader.rs:24-47, as reached from debug_window.rs:53-62).

Everything renders on the GPU through librt_mi355x.so; there is no CPU path.  Device buffers are
torch tensors (``torch`` is plumbing for HBM allocations and streams), host results are numpy.
"""
from __future__ import annotations

import ctypes
import os
import sys as _sys
from typing import Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import check, d3, d4, lib

MAX_FRAMES = 300   # src/raydebugger/gui.rs:20 -- the GUI's time = frame / MAX_FRAMES


class MatrixTransformation:
    """transformation.rs:47-205: a 4x4 matrix and its separately built inverse."""

    def __init__(self, xf: Optional[_lib.rt_transformation] = None):
        self.xf = xf if xf is not None else _lib.rt_transformation()
        if xf is None:
            check(lib().rt_xform_identity(ctypes.byref(self.xf)))

    @classmethod
    def create_identity_matrix(cls) -> "MatrixTransformation":
        return cls()

    @classmethod
    def _make(cls, fn, x, y, z) -> "MatrixTransformation":
        t = _lib.rt_transformation()
        check(fn(float(x), float(y), float(z), ctypes.byref(t)))
        return cls(t)

    @classmethod
    def create_translation_matrix(cls, x, y, z):
        return cls._make(lib().rt_xform_translation, x, y, z)

    @classmethod
    def create_rotation_matrix(cls, x, y, z):
        return cls._make(lib().rt_xform_rotation, x, y, z)

    @classmethod
    def create_scaling_matrix(cls, x, y, z):
        return cls._make(lib().rt_xform_scaling, x, y, z)

    def compose_with(self, other: "MatrixTransformation") -> "MatrixTransformation":
        out = _lib.rt_transformation()
        check(lib().rt_xform_compose(ctypes.byref(self.xf), ctypes.byref(other.xf), ctypes.byref(out)))
        return MatrixTransformation(out)

    @property
    def matrix(self) -> np.ndarray:
        return np.array(self.xf.matrix[:]).reshape(4, 4)

    @property
    def inverse_matrix(self) -> np.ndarray:
        return np.array(self.xf.inverse[:]).reshape(4, 4)

    def transform_vector(self, v: Sequence[float]) -> np.ndarray:
        """transformation.rs:53-59, left-to-right sums."""
        m = self.xf.matrix
        x, y, z = (float(c) for c in v)
        return np.array([m[4 * r] * x + m[4 * r + 1] * y + m[4 * r + 2] * z + m[4 * r + 3] for r in range(3)])


class TransformationStack:
    """transformation.rs:7-37."""

    def __init__(self):
        self.stack = [MatrixTransformation.create_identity_matrix()]

    def push_transformation(self, t: MatrixTransformation) -> None:
        self.stack.append(t.compose_with(self.stack[-1]) if self.stack else t)

    def pop_transformation(self) -> MatrixTransformation:
        if not self.stack:
            raise IndexError("Trying to pop from an empty TransformationStack!")
        return self.stack.pop()

    def get_transformation(self) -> MatrixTransformation:
        return self.stack[-1]


def solid_material(color=(0.0, 0.0, 0.0, 1.0), reflectivity=0.0, transparency=0.0) -> _lib.rt_material:
    """SolidColorMaterial::new (material.rs:41-49); RTObject::new's default is BLACK (rt_object.rs:13-20)."""
    c = list(color) + [1.0] * (4 - len(color))
    return _lib.rt_material(d4(c), -1, float(reflectivity), float(transparency))


def textured_material(texture_id: int, reflectivity=0.0, transparency=0.0) -> _lib.rt_material:
    """TexturedMaterial::new (material.rs:76-84)."""
    return _lib.rt_material(d4((0, 0, 0, 1)), int(texture_id), float(reflectivity), float(transparency))


class Scene:
    """Owner of an ``rt_scene*`` (the RayTracer's scene content)."""

    def __init__(self, handle: int, width: int, height: int, status: int = 0, error: str = ""):
        self.h = ctypes.c_void_p(handle)
        self.width, self.height = width, height
        self.status, self.error = status, error

    @classmethod
    def new_default(cls, width: int, height: int) -> "Scene":
        h = ctypes.c_void_p()
        check(lib().rt_scene_new(width, height, ctypes.byref(h)))
        return cls(h.value, width, height)

    @classmethod
    def compile(cls, text: str, time: float, width: int, height: int,
                asset_dir: Optional[str] = None, strict: bool = True) -> "Scene":
        """load_scene on a fresh new_default()+add_test_objects() RayTracer.

        A parse error raises when ``strict``; otherwise the default scene is returned with
        ``status``/``error`` set, as the reference prints the error and renders on
        (debug_window.rs:58-60)."""
        h = ctypes.c_void_p()
        rc = lib().rt_scene_compile(text.encode(), asset_dir.encode() if asset_dir else None,
                                    float(time), width, height, ctypes.byref(h))
        if rc == -2 and not strict and h.value:
            return cls(h.value, width, height, rc, lib().rt_last_error().decode())
        check(rc)
        return cls(h.value, width, height)

    def info(self) -> dict:
        no, nl, nlf = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        w, h = ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().rt_scene_info(self.h, ctypes.byref(no), ctypes.byref(nl), ctypes.byref(nlf),
                                  ctypes.byref(w), ctypes.byref(h)))
        return {"objects": no.value, "lights": nl.value, "leaves": nlf.value,
                "width": w.value, "height": h.value}

    def trace_pixel(self, x: float, y: float, max_depth: int = -1, device: int = 0) -> np.ndarray:
        """rt_trace_pixel_f64: RayTracer::get_pixel(x, y) of this scene, traced on GPU ``device``
        (no context of the caller's; one upload per call).  Returns 4 doubles (r, g, b, a)."""
        out = np.empty(4, np.float64)
        check(lib().rt_trace_pixel_f64(self.h, float(x), float(y), int(max_depth), int(device),
                                       ctypes.c_void_p(out.ctypes.data)))
        return out

    def traversal(self) -> List[Tuple[int, int]]:
        """The kernels' object hierarchy: pre-order (obj, skip) nodes, obj = -1 for a group."""
        n = ctypes.c_int32()
        check(lib().rt_scene_traversal(self.h, None, None, 0, ctypes.byref(n)))
        obj, skip = (ctypes.c_int32 * max(1, n.value))(), (ctypes.c_int32 * max(1, n.value))()
        check(lib().rt_scene_traversal(self.h, obj, skip, n.value, ctypes.byref(n)))
        return [(obj[i], skip[i]) for i in range(n.value)]

    def describe(self) -> str:
        """rt_scene_describe: the flattened scene (flags, hierarchies, culling records) as text."""
        n = ctypes.c_size_t()
        check(lib().rt_scene_describe(self.h, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value + 1)
        check(lib().rt_scene_describe(self.h, buf, n.value + 1, ctypes.byref(n)))
        return buf.value.decode()

    def spec_program(self) -> str:
        """rt_scene_spec_program: the scene-specialised program's text (RT_OPT_SPECIALIZE)."""
        n = ctypes.c_size_t()
        check(lib().rt_scene_spec_program(self.h, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value + 1)
        check(lib().rt_scene_spec_program(self.h, buf, n.value + 1, ctypes.byref(n)))
        return buf.value.decode()

    def precompile(self) -> float:
        """rt_scene_precompile: compile the specialised program into the process cache (no device);
        returns the hipRTC milliseconds (0 when cached)."""
        ms = ctypes.c_double()
        check(lib().rt_scene_precompile(self.h, ctypes.byref(ms)))
        return ms.value

    def spec_report(self) -> str:
        """rt_scene_spec_report: compile (or find) the scene's specialised programs and describe them --
        the compiler, and per kernel its VGPRs, spills, scratch, occupancy and where it came from."""
        n = ctypes.c_size_t()
        check(lib().rt_scene_spec_report(self.h, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value + 1)
        check(lib().rt_scene_spec_report(self.h, buf, n.value + 1, ctypes.byref(n)))
        return buf.value.decode()

    @staticmethod
    def register_family(scenes) -> float:
        """rt_spec_family_register: one specialised program for scenes of the same structure (the
        frames of an animation); renderers whose scene belongs to it load that program when
        specialisation is on.  Returns the hipRTC milliseconds (0 when cached)."""
        arr = (ctypes.c_void_p * len(scenes))(*[s.h.value for s in scenes])
        ms = ctypes.c_double()
        check(lib().rt_spec_family_register(arr, len(scenes), ctypes.byref(ms)))
        return ms.value

    @staticmethod
    def clear_families() -> None:
        """rt_spec_family_clear: forget every registered scene family."""
        check(lib().rt_spec_family_clear())

    def camera(self) -> dict:
        out = (ctypes.c_double * 13)()
        check(lib().rt_scene_get_camera(self.h, out))
        v = list(out)
        return {"center": v[0:3], "direction": v[3:6], "right": v[6:9], "up": v[9:12], "aspect": v[12]}

    def light(self, i: int) -> Tuple[list, list]:
        p, c = (ctypes.c_double * 3)(), (ctypes.c_double * 4)()
        check(lib().rt_scene_get_light(self.h, i, p, c))
        return list(p), list(c)

    def free(self) -> None:
        if self.h and self.h.value:
            lib().rt_scene_free(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Renderer:
    """Owner of an ``rt_ctx*``: one device, its stream, the uploaded scene."""

    # RT_OPT_SPECIALIZE for new renderers: None keeps the library's default (1: the scene's kernels
    # compiled in the background after each upload, taken once ready).  tests/conftest.py sets 0 so
    # that tests which pin a kernel choice see a deterministic one; the specialised paths have tests of
    # their own (tests/test_gpu_spec*.py, test_gpu_spec_async.py).
    LIBRARY_DEFAULT = -1            # specialize=LIBRARY_DEFAULT: leave the option as the library sets it
    default_specialize: Optional[int] = None

    def __init__(self, device: int = 0, specialize: Optional[int] = None):
        h = ctypes.c_void_p()
        check(lib().rt_ctx_create(int(device), ctypes.byref(h)))
        self.h = h
        Renderer._register(self)
        self.device = device
        self.width = self.height = 0
        level = specialize if specialize is not None else Renderer.default_specialize
        if level is not None and level != Renderer.LIBRARY_DEFAULT:
            self.set_specialize(level, wait=False)

    def upload(self, scene: Scene) -> None:
        check(lib().rt_ctx_upload(self.h, scene.h))
        self.width, self.height = scene.width, scene.height

    def render_rows_into(self, y0: int, y1: int, out_ptr: int, row_stride: int, max_depth: int = -1,
                         stream: Optional[int] = None, f64: bool = False) -> None:
        fn = lib().rt_render_rows_f64 if f64 else lib().rt_render_rows
        check(fn(self.h, y0, y1, max_depth, ctypes.c_void_p(out_ptr), row_stride, ctypes.c_void_p(stream or 0)))

    def render_rows(self, y0: int, y1: int, max_depth: int = -1, f64: bool = False, out=None,
                    stream=None):
        """Render rows [y0, y1) into a device tensor (torch, on this device) and return it.

        uint8 RGBA (rows, W, 4) by default, float64 RGBA with ``f64``.  Runs on ``stream``
        (a torch.cuda.Stream) or torch's current stream, asynchronously."""
        import torch
        dev = torch.device("cuda", self.device)
        if out is None:
            out = torch.empty((y1 - y0, self.width, 4), dtype=torch.float64 if f64 else torch.uint8, device=dev)
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        self.render_rows_into(y0, y1, out.data_ptr(), out.stride(0) * out.element_size(), max_depth,
                              st.cuda_stream, f64)
        return out

    def rows_launcher(self, y0: int, y1: int, out, max_depth: int = -1, stream=None):
        """A zero-argument callable that launches rt_render_rows(y0, y1) into the device tensor ``out``
        on ``stream`` (torch's current stream by default) each time it is called: the arguments are
        converted once, so a host loop pays one ctypes call per frame -- what a native host's FFI call
        costs -- instead of this wrapper's per-call argument handling (a 1080p single-sphere frame takes
        ~19 us on the GPU, the same order as that handling)."""
        import torch
        st = stream if stream is not None else torch.cuda.current_stream(torch.device("cuda", self.device))
        fn = lib().rt_render_rows
        args = (self.h, ctypes.c_uint32(y0), ctypes.c_uint32(y1), ctypes.c_int32(max_depth), ctypes.c_void_p(out.data_ptr()),
                ctypes.c_size_t(out.stride(0) * out.element_size()), ctypes.c_void_p(st.cuda_stream))
        keep = out

        def launch():
            rc = fn(*args)
            if rc < 0:
                check(rc)
            return keep
        return launch

    def render_row_bands(self, y_first: int, band_rows: int, band_pitch: int, n_bands: int, out,
                         max_depth: int = -1, stream=None) -> None:
        """rt_render_row_bands into a device uint8 tensor ``out`` of >= n_bands*band_rows rows: RGBA8
        (rows, W, 4), or packed RGB8 (rows, W, 3) through rt_render_row_bands_rgb8."""
        import torch
        st = stream if stream is not None else torch.cuda.current_stream(torch.device("cuda", self.device))
        fn = lib().rt_render_row_bands_rgb8 if out.shape[-1] == 3 else lib().rt_render_row_bands
        check(fn(self.h, y_first, band_rows, band_pitch, n_bands, max_depth, ctypes.c_void_p(out.data_ptr()),
                 out.stride(0) * out.element_size(), ctypes.c_void_p(st.cuda_stream)))

    def render_rows_host(self, y0: int, y1: int, max_depth: int = -1, f64: bool = False) -> np.ndarray:
        """Synchronous render into a host numpy array (the library stages through HBM)."""
        out = np.empty((y1 - y0, self.width, 4), np.float64 if f64 else np.uint8)
        self.render_rows_into(y0, y1, out.ctypes.data, out.strides[0], max_depth, None, f64)
        return out

    def render_points(self, xy: np.ndarray, max_depth: int = -1) -> np.ndarray:
        xy = np.ascontiguousarray(xy, dtype=np.float64).reshape(-1, 2)
        out = np.empty((xy.shape[0], 4), np.float64)
        check(lib().rt_render_points_f64(self.h, ctypes.c_void_p(xy.ctypes.data), xy.shape[0], max_depth,
                                         ctypes.c_void_p(out.ctypes.data), None))
        return out

    def antialias(self, frame, threshold: float = 0.01, level: int = 3, max_depth: int = -1, f64: bool = False,
                  out=None, stream=None):
        """rt_antialias over a whole quantised frame.  ``frame`` is an (H, W, 4) uint8 torch tensor
        on this device (returns a device tensor; asynchronous up to the edge count) or a numpy
        array (returns numpy).  Returns (anti-aliased frame, sub-pixel rays traced); the frame is
        float64 RGBA with ``f64``."""
        rays = ctypes.c_uint64(0)
        if isinstance(frame, np.ndarray):
            src = np.ascontiguousarray(frame, dtype=np.uint8)
            res = out if out is not None else np.empty(src.shape, np.float64 if f64 else np.uint8)
            sp, ss, rp, rs = src.ctypes.data, src.strides[0], res.ctypes.data, res.strides[0]
            st = 0
        else:
            import torch
            src = frame
            res = out if out is not None else torch.empty(tuple(frame.shape), dtype=torch.float64 if f64 else torch.uint8,
                                                          device=frame.device)
            sp, ss = src.data_ptr(), src.stride(0) * src.element_size()
            rp, rs = res.data_ptr(), res.stride(0) * res.element_size()
            st = (stream if stream is not None else torch.cuda.current_stream(frame.device)).cuda_stream
        u8p, u8s, fp, fs = (None, 0, rp, rs) if f64 else (rp, rs, None, 0)
        check(lib().rt_antialias(self.h, ctypes.c_void_p(sp), ss, float(threshold), int(level), int(max_depth),
                                 ctypes.c_void_p(u8p), u8s, ctypes.c_void_p(fp), fs, ctypes.byref(rays),
                                 ctypes.c_void_p(st)))
        return res, rays.value

    def record_rays(self, x: float, y: float, max_depth: int = -1, cap: int = 1 << 17):
        """rt_record_rays: (records as a RAY_RECORD_DTYPE array in callback order, pixel colour)."""
        buf = np.zeros(cap, RAY_RECORD_DTYPE)
        n = ctypes.c_int32(0)
        rgba = (ctypes.c_double * 4)()
        check(lib().rt_record_rays(self.h, float(x), float(y), int(max_depth), ctypes.c_void_p(buf.ctypes.data),
                                   cap, ctypes.byref(n), rgba))
        return buf[:min(n.value, cap)].copy(), np.array(rgba[:])

    def render_ortho(self, axes: "OrthoAxes", y0: int = 0, y1: Optional[int] = None, f64: bool = False) -> np.ndarray:
        """rt_render_ortho rows [y0, y1) into a host array (uint8 RGBA, or float64 with ``f64``)."""
        y1 = self.height if y1 is None else y1
        out = np.empty((y1 - y0, self.width, 4), np.float64 if f64 else np.uint8)
        p8, s8, pf, sf = (None, 0, out.ctypes.data, out.strides[0]) if f64 else (out.ctypes.data, out.strides[0], None, 0)
        check(lib().rt_render_ortho(self.h, axes.axis1, axes.axis2, float(axes.dir1), float(axes.dir2),
                                    float(axes.scale), y0, y1, ctypes.c_void_p(p8), s8, ctypes.c_void_p(pf), sf,
                                    None))
        return out

    def set_kernel(self, kernel: str = "auto") -> None:
        """rt_ctx_set_option(RT_OPT_KERNEL): "auto", "mega", "deferred" or "wavefront" (same pixels;
        see rt_abi.h)."""
        v = {"auto": _lib.RT_KERNEL_AUTO, "mega": _lib.RT_KERNEL_MEGA, "deferred": _lib.RT_KERNEL_DEFERRED,
             "wavefront": _lib.RT_KERNEL_WAVEFRONT}[kernel]
        check(lib().rt_ctx_set_option(self.h, _lib.RT_OPT_KERNEL, v))

    def set_timing(self, on: bool) -> None:
        """rt_ctx_set_option(RT_OPT_TIMING): record (default) or skip the HIP event pair around every
        render launch that last_kernel_ms() reads (each timed event costs the stream ~5 us)."""
        check(lib().rt_ctx_set_option(self.h, _lib.RT_OPT_TIMING, 1 if on else 0))

    def set_tile_order(self, on: bool) -> None:
        """rt_ctx_set_option(RT_OPT_TILE_ORDER): longest-first tile dispatch after a calibration launch
        (default) or row-major tiles (same pixels)."""
        check(lib().rt_ctx_set_option(self.h, _lib.RT_OPT_TILE_ORDER, 1 if on else 0))

    def set_fast_clamp(self, on: bool) -> None:
        """rt_ctx_set_option(RT_OPT_FAST_CLAMP): min/max colour clamps where the host proved them exact
        (default) or the reference's compare/select clamps everywhere (same pixels)."""
        check(lib().rt_ctx_set_option(self.h, _lib.RT_OPT_FAST_CLAMP, 1 if on else 0))

    def set_wavefront_cap(self, percent: int) -> None:
        """rt_ctx_set_option(RT_OPT_WAVEFRONT_CAP): rays per recursion level of the wavefront path, in
        percent of the launch's pixel slots (pixels whose tree overflows are re-rendered, same bits)."""
        check(lib().rt_ctx_set_option(self.h, _lib.RT_OPT_WAVEFRONT_CAP, int(percent)))

    def set_wavefront_pairs(self, mode: int) -> None:
        """rt_ctx_set_option(RT_OPT_WAVEFRONT_PAIRS): the wavefront path's per-level tracing: 0 one wave
        walks the hierarchy for 64 rays, 1 (default) levels >= 1 as (ray, object) pairs sorted by
        object, 2 every level (same pixels)."""
        check(lib().rt_ctx_set_option(self.h, _lib.RT_OPT_WAVEFRONT_PAIRS, int(mode)))

    def set_specialize(self, level: int = 1, wait: bool = True) -> None:
        """rt_ctx_set_option(RT_OPT_SPECIALIZE): 0 the precompiled kernels; 1 (the library default) the
        uploaded scene's RGBA8 / RGB8 row kernels compiled with the scene as constants (hipRTC in the
        library's background pool; same pixels); 2 its f64 and calibration kernels too.  ``wait``: block
        until the program is loaded (spec_wait), raising if it failed."""
        check(lib().rt_ctx_set_option(self.h, _lib.RT_OPT_SPECIALIZE, int(level)))
        if wait and level:
            self.spec_wait()

    def spec_wait(self, timeout_ms: int = -1) -> bool:
        """rt_ctx_spec_wait: block until the scene-specialised program is loaded (True), or until
        ``timeout_ms`` passed (False); raises RtError when the compile failed or the guard refused it."""
        rc = check(lib().rt_ctx_spec_wait(self.h, int(timeout_ms)))
        return rc != _lib.RT_PENDING

    def kernel_info(self) -> str:
        """rt_ctx_kernel_info: generic or scene-specialised kernels, and what the last row launch ran."""
        buf = ctypes.create_string_buffer(4096)
        check(lib().rt_ctx_kernel_info(self.h, buf, 4096))
        return buf.value.decode()

    def kernel_variant(self) -> str:
        """"spec" when the context holds scene-specialised kernels, else "generic"."""
        return "spec" if self.kernel_info().startswith("scene-specialised") else "generic"

    def last_kernel_ms(self) -> float:
        ms = ctypes.c_float()
        check(lib().rt_ctx_last_kernel_ms(self.h, ctypes.byref(ms)))
        return ms.value

    def synchronize(self) -> None:
        check(lib().rt_ctx_synchronize(self.h))

    def free(self) -> None:
        if self.h and self.h.value:
            lib().rt_ctx_free(self.h)
            self.h = ctypes.c_void_p()

    # Contexts still alive at interpreter exit are freed by an atexit hook, registered after torch's
    # (atexit runs last-registered first) and so while the HIP runtime is still up: a context freed
    # during module teardown unloaded its specialised modules / freed its buffers after torch had
    # shut its side of the runtime down (round 4: SIGSEGV / std::bad_variant_access at exit).
    # The hook is moved to the END of the atexit list whenever a renderer is made (atexit runs the
    # last-registered first), so it still runs before hooks that torch registers once its CUDA side
    # starts; it also stops the library's compile pool (rt_spec_shutdown) so that no hipRTC compile
    # runs while the process tears the runtime down.
    @classmethod
    def _register(cls, r: "Renderer") -> None:
        import atexit
        if "_live" not in cls.__dict__:
            import weakref
            cls._live = weakref.WeakSet()
        atexit.unregister(cls.free_all)
        atexit.register(cls.free_all)
        cls._live.add(r)

    @classmethod
    def free_all(cls) -> None:
        for r in list(cls.__dict__.get("_live", ())):
            r.free()
        lib().rt_spec_shutdown()

    def __del__(self):
        if _sys.is_finalizing():
            return
        try:
            self.free()
        except Exception:
            pass


class RayTracer:
    """raytracer.rs:21-364 over the GPU path.

    Build the scene with the same calls the reference's scene parser makes, or ``load_scene``
    a DSL text; then ``get_pixel`` / ``render_lines`` as the GUI worker does."""

    def __init__(self, width: int, height: int, device: int = 0):
        self.width, self.height = width, height
        self.scene = Scene.new_default(width, height)       # RayTracer::new_default (:38-44)
        self.transformation_stack = TransformationStack()
        self.device = device
        self._renderer: Optional[Renderer] = None
        self._dirty = True
        self._max_depth = 10

    new_default = classmethod(lambda cls, width, height, device=0: cls(width, height, device))

    # -- scene construction (raytracer.rs:72-130, 289-330) --------------------------------
    def add_test_objects(self) -> None:
        check(lib().rt_scene_add_test_objects(self.scene.h))
        self._dirty = True

    def add_texture(self, rgba8: np.ndarray) -> int:
        rgba8 = np.ascontiguousarray(rgba8, dtype=np.uint8)
        h, w = rgba8.shape[:2]
        self._dirty = True
        return check(lib().rt_scene_add_texture(self.scene.h, w, h, ctypes.c_void_p(rgba8.ctypes.data)))

    def _xf(self, t: Optional[MatrixTransformation]) -> _lib.rt_transformation:
        return (t or self.transformation_stack.get_transformation()).xf

    def sphere(self, center=(0, 0, 0), radius=1.0, t: Optional[MatrixTransformation] = None) -> int:
        return check(lib().rt_shape_sphere(self.scene.h, ctypes.byref(self._xf(t)), d3(center), float(radius)))

    def cube(self, center=(0, 0, 0), length=1.0, t: Optional[MatrixTransformation] = None) -> int:
        return check(lib().rt_shape_cube(self.scene.h, ctypes.byref(self._xf(t)), d3(center), float(length)))

    def plane(self, normal=(0, 1, 0), distance=1.0, t: Optional[MatrixTransformation] = None) -> int:
        return check(lib().rt_shape_plane(self.scene.h, ctypes.byref(self._xf(t)), d3(normal), float(distance)))

    def csg(self, a: int, b: int, operator: str = "union") -> int:
        op = {"union": 0, "intersection": 1, "difference": 2}[operator]
        return check(lib().rt_shape_csg(self.scene.h, op, a, b))

    def add_object(self, shape: int, material: Optional[_lib.rt_material] = None) -> None:
        check(lib().rt_scene_add_object(self.scene.h, shape, ctypes.byref(material or solid_material())))
        self._dirty = True

    def add_light(self, point, color=(0.5, 0.5, 0.5, 1.0), fade_distance=100.0) -> None:
        check(lib().rt_scene_add_light(self.scene.h, d3(point), d4(list(color) + [1.0] * (4 - len(color))),
                                       float(fade_distance)))
        self._dirty = True

    def set_camera_from_vector(self, center) -> None:
        """raytracer.rs:289-299: the centre is transformed by the stack top first."""
        c = self.transformation_stack.get_transformation().transform_vector(center)
        check(lib().rt_scene_set_camera(self.scene.h, d3(c)))
        self._dirty = True

    @property
    def max_depth(self) -> int:
        return self._max_depth

    @max_depth.setter
    def max_depth(self, d: int) -> None:
        check(lib().rt_scene_set_max_depth(self.scene.h, int(d)))
        self._max_depth = int(d)
        self._dirty = True

    def load_scene(self, text: str, time: float = 0.0, asset_dir: Optional[str] = None,
                   strict: bool = True) -> None:
        """DebugWindow::load_ray_tracer (debug_window.rs:53-62): a fresh new_default RayTracer
        with the test light, then load_scene(text, time).  Replaces this tracer's scene."""
        self.scene = Scene.compile(text, time, self.width, self.height, asset_dir, strict)
        self.transformation_stack = TransformationStack()
        if self._max_depth != 10:
            check(lib().rt_scene_set_max_depth(self.scene.h, self._max_depth))
        self._dirty = True

    # -- rendering ------------------------------------------------------------------------
    @property
    def renderer(self) -> Renderer:
        if self._renderer is None:
            self._renderer = Renderer(self.device)
        if self._dirty:
            self._renderer.upload(self.scene)
            self._dirty = False
        return self._renderer

    def get_pixel(self, x: float, y: float) -> np.ndarray:
        """raytracer.rs:359-363: colour (r, g, b, a) of the camera ray through (x, y)."""
        return self.renderer.render_points(np.array([[x, y]], np.float64))[0]

    def render_lines(self, line_range: Iterable[int]) -> Iterator[Tuple[int, np.ndarray]]:
        """debug_window.rs:74-87: yields (y, row of W colours as (W, 4) f64)."""
        r = self.renderer
        for y in line_range:
            yield y, r.render_rows_host(y, y + 1, f64=True)[0]

    def render_frame(self) -> np.ndarray:
        """The whole frame as RGBA8 (H, W, 4), quantised as easy_pixbuf.rs:46-53."""
        return self.renderer.render_rows_host(0, self.height)

    def render_orthogonal_view_line(self, y: int, ortho_axes: "OrthoAxes") -> np.ndarray:
        """DebugWindow::render_orthogonal_view_line (debug_window.rs:166-227): (W, 4) f64 colours."""
        return _ortho_line(self, y, ortho_axes)

    def render_orthogonal_view(self, area: str = "top") -> np.ndarray:
        """A whole orthogonal preview ("top", "front", "side") as RGBA8 (H, W, 4)."""
        return self.renderer.render_ortho(OrthoAxes.from_area(area))


ORTHO_SCALE = 2.0   # ray_debugger.rs:11

# rt_ray_record (include/rt_abi.h) as a numpy dtype
RAY_RECORD_DTYPE = np.dtype([
    ("depth", "<i4"), ("ray_type", "<i4"), ("object", "<i4"), ("intersected", "<i4"), ("has_normal", "<i4"),
    ("pad", "<i4"), ("point", "<f8", 3), ("direction", "<f8", 3), ("distance", "<f8"),
    ("intersection", "<f8", 3), ("normal", "<f8", 3), ("color", "<f8", 4)])
RAY_TYPES = ("NormalRay", "ReflectionRay", "TransmissionRay")


class RayDebugger:
    """ray_debugger.rs:71-137: records every ray of one pixel (RayInfo list in callback order)."""

    def __init__(self, width: int, height: int):
        self.rays = np.zeros(0, RAY_RECORD_DTYPE)
        self.debugged_position = None
        self.width, self.height = width, height
        self.show_normals = True

    def record_rays(self, ray_tracer: "RayTracer", x: float, y: float) -> None:
        if self.debugged_position == (x, y):          # already showing these rays (:93-97)
            return
        self.debugged_position = (x, y)
        self.rays = ray_tracer.renderer.record_rays(x, y, ray_tracer.max_depth)[0]

    def reset_debugger(self) -> None:
        self.debugged_position = None


class OrthoAxes:
    """ray_debugger.rs:24-68: the axes of an orthogonal preview view."""

    def __init__(self, axis1: int, axis2: int, dir1: float, dir2: float, scale: float = ORTHO_SCALE):
        self.axis1, self.axis2, self.dir1, self.dir2, self.scale = int(axis1), int(axis2), dir1, dir2, scale

    @staticmethod
    def from_area(area: str) -> "OrthoAxes":
        """impl From<DrawingArea> for OrthoAxes: "top", "front" or "side"."""
        if area == "top":
            return OrthoAxes(0, 2, 1.0, -1.0)
        if area == "front":
            return OrthoAxes(0, 1, 1.0, -1.0)
        if area == "side":
            return OrthoAxes(2, 1, -1.0, -1.0)
        raise ValueError("Main view is not an orthogonal view!" if area == "main" else f"unknown area {area!r}")


class AntiAliaser:
    """antialiaser.rs:7-192: adaptive anti-aliasing of a rendered (quantised) frame.

    ``AntiAliaser(ray_tracer, threshold=None, level=None)`` takes the reference's defaults
    (0.1 and 3, antialiaser.rs:18-19); the GUI passes ANTIALIAS_THRESHOLD = 0.01 and
    ANTIALIAS_LEVEL = 3 (debug_window.rs:26-27).  The whole frame is one GPU pass (rt_antialias);
    ``ray_counter`` accumulates the sub-pixel rays traced like the reference's counter."""

    def __init__(self, ray_tracer: "RayTracer", threshold: Optional[float] = None, level: Optional[int] = None):
        self.ray_tracer = ray_tracer
        self.threshold = 0.1 if threshold is None else float(threshold)
        self.level = 3 if level is None else int(level)
        self.size = (1 << self.level) + 1
        self.ray_counter = 0

    def set_threshold(self, threshold: float) -> None:
        self.threshold = float(threshold)

    def anti_alias_frame(self, frame, f64: bool = False):
        """Every line of ``anti_alias_line_vec`` (antialiaser.rs:53-71) for y in 0..H-1, as the
        AA worker does (debug_window.rs:298-318); the last row is passed through."""
        out, rays = self.ray_tracer.renderer.antialias(frame, self.threshold, self.level, self.ray_tracer.max_depth,
                                                       f64=f64)
        self.ray_counter += rays
        return out


def _ortho_line(rt: "RayTracer", y: int, ortho_axes: OrthoAxes) -> np.ndarray:
    return rt.renderer.render_ortho(ortho_axes, y, y + 1, f64=True)[0]


def write_png(path: str, rgba8: np.ndarray, channels: int = 3) -> None:
    rgba8 = np.ascontiguousarray(rgba8, dtype=np.uint8)
    h, w = rgba8.shape[:2]
    check(lib().rt_write_png(path.encode(), ctypes.c_void_p(rgba8.ctypes.data), w, h, rgba8.strides[0], channels))


def read_png_rgba8(path: str) -> np.ndarray:
    p = ctypes.c_void_p()
    w, h = ctypes.c_uint32(), ctypes.c_uint32()
    check(lib().rt_read_png_rgba8(path.encode(), ctypes.byref(p), ctypes.byref(w), ctypes.byref(h)))
    try:
        buf = (ctypes.c_uint8 * (w.value * h.value * 4)).from_address(p.value)
        return np.frombuffer(buf, np.uint8).reshape(h.value, w.value, 4).copy()
    finally:
        lib().rt_free_buffer(p)


def device_count() -> int:
    n = ctypes.c_int()
    check(lib().rt_device_count(ctypes.byref(n)))
    return n.value


def spec_compiler_info() -> Tuple[str, bool]:
    """rt_spec_compiler_info: (identity of the hipRTC the specialised programs compile with, True when
    it is the ROCm installation's own -- the only one the library lets compile them)."""
    buf = ctypes.create_string_buffer(1024)
    rocm = ctypes.c_int32()
    check(lib().rt_spec_compiler_info(buf, 1024, ctypes.byref(rocm)))
    return buf.value.decode(), bool(rocm.value)


def spec_cache_dir(path: Optional[str]) -> None:
    """rt_spec_cache_dir: the on-disk code-object cache of the specialised programs (None: none)."""
    check(lib().rt_spec_cache_dir(path.encode() if path else None))


class HwStream:
    """A HIP stream on a hardware queue of its own (rt_stream_create), usable as a torch stream
    (``.torch``, a torch.cuda.ExternalStream).  Renders meant to overlap go on such streams: plain
    torch / HIP streams share the process's few hardware queues, and two renders on one queue run
    one after the other (include/rt_abi.h rt_stream_create).

    Lifetime: close() (or ``with HwStream() as s``) synchronises and destroys the stream.  Streams
    still open when the interpreter exits are closed by an atexit hook, while the HIP runtime is
    still up: a stream left for the runtime's own teardown (__cxa_finalize) was destroyed after a
    profiler's intercept tables were gone, and rocprofv3 runs died there with SIGSEGV
    (gpurun_out/r03j_kt.err, round-3 VERDICT).  __del__ never destroys a stream during interpreter
    finalisation."""

    _live: "weakref.WeakSet[HwStream]"

    def __init__(self, device: int = 0):
        import torch
        h = ctypes.c_void_p()
        check(lib().rt_stream_create(device, ctypes.byref(h)))
        self.handle = h.value
        self.torch = torch.cuda.ExternalStream(self.handle, device=torch.device("cuda", device))
        HwStream._register(self)

    @classmethod
    def _register(cls, s: "HwStream") -> None:
        if "_live" not in cls.__dict__:
            import atexit
            import weakref
            cls._live = weakref.WeakSet()
            atexit.register(cls.close_all)
        cls._live.add(s)

    @classmethod
    def close_all(cls) -> None:
        for s in list(getattr(cls, "_live", ())):
            s.close()

    def close(self) -> None:
        if getattr(self, "handle", None):
            self.torch.synchronize()
            lib().rt_stream_destroy(ctypes.c_void_p(self.handle))
            self.handle = None

    def __enter__(self) -> "HwStream":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def __del__(self):
        if _sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass
