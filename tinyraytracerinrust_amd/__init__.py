"""tinyraytracerinrust_amd -- MI355X-native per-pixel render path for the TinyRaytracer scene DSL.

The reference (andreivasiliu/TinyRaytracerInRust) renders with a recursive f64 CPU loop
(src/raytracer/raytracer.rs:132-287) driven row by row from its GUI.  This package replaces that
loop with hand-written gfx950 HIP kernels behind a C ABI (include/rt_abi.h, librt_mi355x.so);
this Python layer mirrors the reference's RayTracer interface over that ABI.
"""
from ._lib import RtError, lib  # noqa: F401
from .raytracer import (  # noqa: F401
    MAX_FRAMES,
    ORTHO_SCALE,
    AntiAliaser,
    HwStream,
    OrthoAxes,
    RAY_RECORD_DTYPE,
    RayDebugger,
    MatrixTransformation,
    RayTracer,
    Renderer,
    Scene,
    TransformationStack,
    device_count,
    read_png_rgba8,
    spec_cache_dir,
    spec_compiler_info,
    solid_material,
    textured_material,
    write_png,
)

__all__ = [
    "RtError", "lib", "MAX_FRAMES", "ORTHO_SCALE", "AntiAliaser", "HwStream", "OrthoAxes", "RAY_RECORD_DTYPE", "RayDebugger", "MatrixTransformation", "RayTracer", "Renderer", "Scene",
    "TransformationStack", "device_count", "read_png_rgba8", "spec_cache_dir", "spec_compiler_info", "solid_material", "textured_material",
    "write_png",
]
