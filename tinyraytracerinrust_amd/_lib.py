"""ctypes binding of librt_mi355x.so (include/rt_abi.h).

The shared library is built in-tree (``make -C tinyraytracerinrust_amd``, or
``__graft_entry__.build()``) and loaded from this directory.  There is deliberately no
fallback: if the library is missing or no HIP device is present, the calls fail loudly.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# RT_LIB_PATH: load an alternative build (kernel-variant experiments, tools/); default in-tree.
LIB_PATH = os.environ.get("RT_LIB_PATH") or os.path.join(HERE, "librt_mi355x.so")

RT_OK = 0
RT_PENDING = 1          # rt_ctx_spec_wait: the time limit passed before the compile finished (not an error)
STATUS_NAMES = {
    0: "RT_OK", -1: "RT_ERR_INVALID", -2: "RT_ERR_PARSE", -3: "RT_ERR_EVAL", -4: "RT_ERR_IO",
    -5: "RT_ERR_DEVICE", -6: "RT_ERR_UNSUPPORTED", -7: "RT_ERR_NOMEM",
}
RT_CSG_UNION, RT_CSG_INTERSECTION, RT_CSG_DIFFERENCE = 0, 1, 2
RT_OPT_KERNEL = 0
RT_OPT_TIMING = 1
RT_OPT_TILE_ORDER = 2
RT_OPT_FAST_CLAMP = 3
RT_OPT_WAVEFRONT_CAP = 4
RT_OPT_WAVEFRONT_PAIRS = 5
RT_OPT_SPECIALIZE = 6
RT_KERNEL_AUTO, RT_KERNEL_MEGA, RT_KERNEL_DEFERRED, RT_KERNEL_WAVEFRONT = 0, 1, 2, 3


class RtError(RuntimeError):
    """A negative rt_status from the library, with rt_last_error()'s message."""

    def __init__(self, status: int, message: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")
        self.status = status
        self.message = message


class rt_transformation(ctypes.Structure):
    _fields_ = [("matrix", ctypes.c_double * 16), ("inverse", ctypes.c_double * 16)]


class rt_material(ctypes.Structure):
    _fields_ = [("color", ctypes.c_double * 4), ("texture", ctypes.c_int32),
                ("reflectivity", ctypes.c_double), ("transparency", ctypes.c_double)]


_P = ctypes.c_void_p
_D3 = ctypes.POINTER(ctypes.c_double)
_XF = ctypes.POINTER(rt_transformation)
_I = ctypes.c_int
_U32 = ctypes.c_uint32

# name -> (restype, argtypes); mirrors include/rt_abi.h one to one
SIGNATURES = {
    "rt_abi_version": (_I, []),
    "rt_last_error": (ctypes.c_char_p, []),
    "rt_xform_identity": (_I, [_XF]),
    "rt_xform_translation": (_I, [ctypes.c_double] * 3 + [_XF]),
    "rt_xform_rotation": (_I, [ctypes.c_double] * 3 + [_XF]),
    "rt_xform_scaling": (_I, [ctypes.c_double] * 3 + [_XF]),
    "rt_xform_compose": (_I, [_XF, _XF, _XF]),
    "rt_scene_new": (_I, [_U32, _U32, ctypes.POINTER(_P)]),
    "rt_scene_add_test_objects": (_I, [_P]),
    "rt_scene_add_texture": (_I, [_P, _U32, _U32, _P]),
    "rt_shape_sphere": (_I, [_P, _XF, _D3, ctypes.c_double]),
    "rt_shape_cube": (_I, [_P, _XF, _D3, ctypes.c_double]),
    "rt_shape_plane": (_I, [_P, _XF, _D3, ctypes.c_double]),
    "rt_shape_csg": (_I, [_P, _I, ctypes.c_int32, ctypes.c_int32]),
    "rt_scene_add_object": (_I, [_P, ctypes.c_int32, ctypes.POINTER(rt_material)]),
    "rt_scene_add_light": (_I, [_P, _D3, _D3, ctypes.c_double]),
    "rt_scene_set_camera": (_I, [_P, _D3]),
    "rt_scene_set_max_depth": (_I, [_P, ctypes.c_int32]),
    "rt_scene_compile": (_I, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_double, _U32, _U32,
                              ctypes.POINTER(_P)]),
    "rt_scene_traversal": (_I, [_P, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32), ctypes.c_int32,
                                ctypes.POINTER(ctypes.c_int32)]),
    "rt_scene_describe": (_I, [_P, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    "rt_scene_spec_program": (_I, [_P, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    "rt_scene_precompile": (_I, [_P, ctypes.POINTER(ctypes.c_double)]),
    "rt_spec_family_register": (_I, [ctypes.POINTER(_P), ctypes.c_int32, ctypes.POINTER(ctypes.c_double)]),
    "rt_spec_family_clear": (_I, []),
    "rt_ctx_kernel_info": (_I, [_P, ctypes.c_char_p, ctypes.c_size_t]),
    "rt_ctx_spec_wait": (_I, [_P, ctypes.c_int32]),
    "rt_scene_spec_report": (_I, [_P, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    "rt_spec_compiler_info": (_I, [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int32)]),
    "rt_spec_cache_dir": (_I, [ctypes.c_char_p]),
    "rt_spec_shutdown": (None, []),
    "rt_scene_info": (_I, [_P, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                           ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(_U32),
                           ctypes.POINTER(_U32)]),
    "rt_scene_get_camera": (_I, [_P, _D3]),
    "rt_scene_get_light": (_I, [_P, ctypes.c_int32, _D3, _D3]),
    "rt_scene_free": (None, [_P]),
    "rt_device_count": (_I, [ctypes.POINTER(_I)]),
    "rt_ctx_create": (_I, [_I, ctypes.POINTER(_P)]),
    "rt_ctx_upload": (_I, [_P, _P]),
    "rt_render_rows": (_I, [_P, _U32, _U32, ctypes.c_int32, _P, ctypes.c_size_t, _P]),
    "rt_render_row_bands": (_I, [_P, _U32, _U32, _U32, _U32, ctypes.c_int32, _P, ctypes.c_size_t, _P]),
    "rt_assemble_row_bands": (_I, [_P, ctypes.c_size_t, _U32, _U32, _U32, _U32, ctypes.c_size_t, _P,
                                   ctypes.c_size_t, _P]),
    "rt_render_row_bands_rgb8": (_I, [_P, _U32, _U32, _U32, _U32, ctypes.c_int32, _P, ctypes.c_size_t, _P]),
    "rt_assemble_row_bands_rgb8": (_I, [_P, ctypes.c_size_t, _U32, _U32, _U32, _U32, _U32, _P, ctypes.c_size_t, _P]),
    "rt_render_rows_f64": (_I, [_P, _U32, _U32, ctypes.c_int32, _P, ctypes.c_size_t, _P]),
    "rt_render_points_f64": (_I, [_P, _P, ctypes.c_size_t, ctypes.c_int32, _P, _P]),
    "rt_trace_pixel_f64": (_I, [_P, ctypes.c_double, ctypes.c_double, ctypes.c_int32, ctypes.c_int, _P]),
    "rt_record_rays": (_I, [_P, ctypes.c_double, ctypes.c_double, ctypes.c_int32, _P, ctypes.c_int32,
                            ctypes.POINTER(ctypes.c_int32), _P]),
    "rt_render_ortho": (_I, [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                             ctypes.c_uint32, ctypes.c_uint32, _P, ctypes.c_size_t, _P, ctypes.c_size_t, _P]),
    "rt_antialias": (_I, [_P, _P, ctypes.c_size_t, ctypes.c_double, ctypes.c_int32, ctypes.c_int32, _P,
                          ctypes.c_size_t, _P, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64), _P]),
    "rt_ctx_last_kernel_ms": (_I, [_P, ctypes.POINTER(ctypes.c_float)]),
    "rt_ctx_synchronize": (_I, [_P]),
    "rt_ctx_set_option": (_I, [_P, ctypes.c_int32, ctypes.c_int32]),
    "rt_stream_create": (_I, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "rt_stream_destroy": (_I, [_P]),
    "rt_ctx_free": (None, [_P]),
    "rt_write_png": (_I, [ctypes.c_char_p, _P, _U32, _U32, ctypes.c_size_t, _I]),
    "rt_read_png_rgba8": (_I, [ctypes.c_char_p, ctypes.POINTER(_P), ctypes.POINTER(_U32),
                               ctypes.POINTER(_U32)]),
    "rt_free_buffer": (None, [_P]),
}

_lib = None


def lib() -> ctypes.CDLL:
    """Load librt_mi355x.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C {HERE}` or __graft_entry__.build(); "
            "there is no CPU fallback for the render path")
    # One HIP runtime per process: torch wheels bundle their own libamdhip64 / libhsa-runtime64
    # (same SONAMEs as /opt/rocm's).  Loaded after torch, this library binds to torch's copies;
    # loaded first, it would pull in /opt/rocm's, and torch's runtime, started later on top of an
    # HSA runtime of another release, finds no device (torch.cuda.is_available() -> False).
    # RT_NO_TORCH_PRELOAD=1 skips this (a host that never uses torch binds /opt/rocm's runtime).
    if not os.environ.get("RT_NO_TORCH_PRELOAD"):
        try:
            import torch  # noqa: F401
        except Exception:                             # no (working) torch: /opt/rocm's runtime
            pass
    handle = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    _lib = handle
    # The on-disk cache of scene-specialised code objects (rt_spec_cache_dir; keyed and checked by
    # program text and compiler): ~/.cache/tinyraytracerinrust_amd/spec, or RT_SPEC_CACHE_DIR
    # ("" turns it off).  The C library itself keeps none unless its host asks.
    cache = os.environ.get("RT_SPEC_CACHE_DIR")
    if cache is None:
        cache = os.path.join(os.path.expanduser("~"), ".cache", "tinyraytracerinrust_amd", "spec")
    handle.rt_spec_cache_dir(cache.encode())
    return handle


def check(status: int) -> int:
    """Raise RtError for a negative status; return non-negative values (ids) unchanged."""
    if status is not None and status < 0:
        msg = lib().rt_last_error()
        raise RtError(status, msg.decode(errors="replace") if msg else "")
    return status


def d3(v) -> ctypes.Array:
    return (ctypes.c_double * 3)(*[float(x) for x in v])


def d4(v) -> ctypes.Array:
    return (ctypes.c_double * 4)(*[float(x) for x in v])
