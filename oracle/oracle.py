"""ctypes front-end for the CPU oracle (oracle/rt_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package.  Textures are decoded here with PIL
(an independent PNG decoder from the product's own) and registered by file name, the
way the reference's `texture("worldmap.png")` resolves a path relative to the CWD
(sceneparser/texture.rs:20-40).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "build")

COUNTER_NAMES = [
    "ray_primary", "ray_shadow", "ray_reflect", "ray_refract",
    "xform_ray",
    "sphere_isect_miss", "sphere_isect_hit",
    "plane_isect", "cube_isect_axis", "cube_isect_zero_axis",
    "csg_point",
    "inside_sphere", "inside_cube", "inside_plane",
    "onsurf_sphere", "onsurf_cube", "onsurf_plane",
    "normal_sphere", "normal_cube_planechk", "normal_plane",
    "uv_sphere", "texture_fetch",
    "shade", "light", "light_lit", "shadow_hit", "inside_test",
    "refract_dir", "reflect_dir", "combine",
    "flop", "transcendental",
]

_libs: dict = {}


def usable_cores() -> int:
    """Cores this process may run on: the affinity mask, capped by the cgroup CPU quota (a GPU
    box's os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                n = min(n, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def default_threads() -> int:
    """Host threads for oracle renders (tests, smoke): every usable core, at most 64, or
    $ORACLE_THREADS."""
    env = os.environ.get("ORACLE_THREADS")
    return int(env) if env else min(64, usable_cores())
_registered: dict = {}


def build() -> None:
    """Compile the oracle with its own Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _lib(counting: bool = False):
    key = bool(counting)
    if key in _libs:
        return _libs[key]
    name = "librt_oracle_count.so" if counting else "librt_oracle.so"
    path = os.path.join(BUILD, name)
    if not os.path.exists(path):
        build()
    lib = ctypes.CDLL(path)
    lib.orc_load_scene.restype = ctypes.c_void_p
    lib.orc_load_scene.argtypes = [ctypes.c_char_p, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
    lib.orc_free_scene.argtypes = [ctypes.c_void_p]
    lib.orc_set_max_depth.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.orc_num_objects.argtypes = [ctypes.c_void_p]
    lib.orc_num_lights.argtypes = [ctypes.c_void_p]
    lib.orc_camera.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
    lib.orc_light.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    lib.orc_texel_probe.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double, ctypes.POINTER(ctypes.c_double)]
    lib.orc_texel_probe.restype = ctypes.c_int
    lib.orc_hit_signature.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double, ctypes.POINTER(ctypes.c_double)]
    lib.orc_hit_signature.restype = ctypes.c_longlong
    lib.orc_get_pixel.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double,
                                  ctypes.POINTER(ctypes.c_double)]
    lib.orc_render_rows.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    lib.orc_render_ortho.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                     ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    lib.orc_record_rays.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double, ctypes.c_void_p, ctypes.c_int,
                                    ctypes.c_void_p]
    lib.orc_antialias.restype = ctypes.c_longlong
    lib.orc_antialias.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_double,
                                  ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    lib.orc_register_texture.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    _libs[key] = lib
    return lib


def decode_png_rgba8(path: str) -> np.ndarray:
    """RGBA8 pixels as lodepng::decode32_file returns them (A=255 for RGB files)."""
    from PIL import Image
    with Image.open(path) as im:
        return np.ascontiguousarray(np.asarray(im.convert("RGBA"), dtype=np.uint8))


def register_texture(name: str, rgba8: np.ndarray) -> None:
    rgba8 = np.ascontiguousarray(rgba8, dtype=np.uint8)
    h, w = rgba8.shape[:2]
    for counting in (False, True):
        key = (counting, name)
        if _registered.get(key) is rgba8:
            continue
        lib = _lib(counting)
        rc = lib.orc_register_texture(name.encode(), w, h, rgba8.ctypes.data)
        if rc != 0:
            raise RuntimeError("orc_register_texture failed")
        _registered[key] = rgba8


def register_texture_file(name: str, path: str) -> np.ndarray:
    pix = decode_png_rgba8(path)
    register_texture(name, pix)
    return pix


class OracleScene:
    """A compiled scene in the oracle (RayTracer after load_scene)."""

    def __init__(self, text: str, time: float, width: int, height: int, max_depth: int = 10,
                 counting: bool = False):
        self.lib = _lib(counting)
        self.width, self.height = width, height
        status = ctypes.c_int(0)
        err = ctypes.create_string_buffer(512)
        h = self.lib.orc_load_scene(text.encode(), float(time), width, height,
                                    ctypes.byref(status), err, 512)
        self.status = status.value
        self.error = err.value.decode(errors="replace")
        if not h:
            raise RuntimeError(f"oracle scene load failed: {self.error}")
        self.h = ctypes.c_void_p(h)
        self.lib.orc_set_max_depth(self.h, max_depth)
        self.counting = counting

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            self.lib.orc_free_scene(h)
            self.h = None

    @property
    def n_objects(self) -> int:
        return self.lib.orc_num_objects(self.h)

    @property
    def n_lights(self) -> int:
        return self.lib.orc_num_lights(self.h)

    def camera(self) -> np.ndarray:
        out = (ctypes.c_double * 10)()
        self.lib.orc_camera(self.h, out)
        return np.array(out[:])

    def light(self, i: int) -> np.ndarray:
        out = (ctypes.c_double * 7)()
        self.lib.orc_light(self.h, i, out)
        return np.array(out[:])

    def get_pixel(self, x: float, y: float) -> np.ndarray:
        out = (ctypes.c_double * 4)()
        self.lib.orc_get_pixel(self.h, float(x), float(y), out)
        return np.array(out[:])

    def texel_probe(self, x: float, y: float):
        """(object, (x_tex, y_tex, u, v)) of get_pixel(x, y)'s primary hit when its object is textured
        (texture.rs:27-34's coordinates before truncation), else (-1, None)."""
        out = (ctypes.c_double * 4)()
        o = self.lib.orc_texel_probe(self.h, float(x), float(y), out)
        return (o, tuple(out[:])) if o >= 0 else (-1, None)

    def hit_signature(self, x: float, y: float) -> int:
        """-1 for a miss, else object + 1 + 4096 * (bit i: light i's shadow ray occluded) of get_pixel(x, y)'s
        primary hit: its changes along a line are silhouettes and shadow edges."""
        t = ctypes.c_double(0.0)
        return int(self.lib.orc_hit_signature(self.h, float(x), float(y), ctypes.byref(t)))

    def render(self, y0: int = 0, y1: int | None = None, row_step: int = 1, threads: int = 0,
               f64: bool = False, u8: bool = True):
        """Render rows y0, y0+row_step, ... < y1. Returns (f64 or None, u8 or None[, counters])."""
        if y1 is None:
            y1 = self.height
        if threads <= 0:
            threads = default_threads()
        nrows = len(range(y0, y1, row_step))
        of = np.zeros((nrows, self.width, 4), np.float64) if f64 else None
        ou = np.zeros((nrows, self.width, 4), np.uint8) if u8 else None
        cnt = np.zeros(len(COUNTER_NAMES), np.uint64)
        self.lib.orc_render_rows(self.h, y0, y1, row_step,
                                 of.ctypes.data if of is not None else None,
                                 ou.ctypes.data if ou is not None else None,
                                 threads, cnt.ctypes.data)
        if self.counting:
            return of, ou, dict(zip(COUNTER_NAMES, (int(c) for c in cnt)))
        return of, ou

    def antialias(self, frame_u8: np.ndarray, threshold: float = 0.01, level: int = 3, threads: int = 0,
                  f64: bool = True):
        """Adaptive anti-aliasing of a quantised (H, W, 4) RGBA8 frame (antialiaser.rs:87-191).
        Returns (f64 or None, u8, sub-pixel rays traced)."""
        fr = np.ascontiguousarray(frame_u8, dtype=np.uint8)
        assert fr.shape == (self.height, self.width, 4)
        if threads <= 0:
            threads = default_threads()
        of = np.zeros((self.height, self.width, 4), np.float64) if f64 else None
        ou = np.zeros((self.height, self.width, 4), np.uint8)
        rays = self.lib.orc_antialias(self.h, fr.ctypes.data, self.width * 4, float(threshold), int(level),
                                      of.ctypes.data if of is not None else None, ou.ctypes.data, threads)
        if rays < 0:
            raise ValueError("unsupported anti-aliasing level")
        return of, ou, int(rays)

    def render_ortho(self, axis1: int, axis2: int, dir1: float, dir2: float, scale: float = 2.0,
                     y0: int = 0, y1: int | None = None):
        """Orthogonal preview rows (debug_window.rs:166-227). Returns (f64, u8)."""
        y1 = self.height if y1 is None else y1
        of = np.zeros((y1 - y0, self.width, 4), np.float64)
        ou = np.zeros((y1 - y0, self.width, 4), np.uint8)
        if self.lib.orc_render_ortho(self.h, axis1, axis2, dir1, dir2, scale, y0, y1, of.ctypes.data, ou.ctypes.data):
            raise ValueError("Invalid axes")
        return of, ou

    def record_rays(self, x: float, y: float, cap: int = 1 << 17):
        """Ray-debugger records of one pixel (callback order) as raw bytes of the C struct; the
        caller views them with the product's RAY_RECORD_DTYPE (identical layout)."""
        size = self.lib.orc_ray_record_size()
        buf = np.zeros(cap * size, np.uint8)
        rgba = (ctypes.c_double * 4)()
        n = self.lib.orc_record_rays(self.h, float(x), float(y), buf.ctypes.data, cap, rgba)
        return buf[:min(n, cap) * size], np.array(rgba[:])
