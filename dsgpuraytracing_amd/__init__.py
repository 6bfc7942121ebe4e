"""MI355X-native path-tracing hot path for Khrylx/DSGPURayTracing.

The per-pixel radiance loop of PathTracer::raytrace_tile (src/pathtracer.cpp)
runs in hand-written gfx950 HIP kernels behind the C ABI of include/ptgpu.h
(libptgpu.so, built in-tree by dsgpuraytracing_amd.build).  This package is
the host-side mirror of the reference interface over that library.
"""
from .native import NativeLibraryError, PtError  # noqa: F401

__all__ = ["NativeLibraryError", "PtError"]
