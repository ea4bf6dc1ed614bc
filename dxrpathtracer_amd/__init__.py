"""dxrpathtracer_amd — MI355X-native (gfx950) drop-in for the DXR path tracer of
WANG-Ruipeng/DXRPathTracer (RayTrace.hlsl + BRDF/Sampling includes).

The product is the HIP library lib/libdxrpt.so behind the C ABI in include/dxrpt.h; this package is
the thin host driver (ctypes) over it plus the host-side scene/camera/sky inputs (lib/libdxrpt_host.so).
"""
from . import _abi
from .scene import Scene, Sky, make_constants, make_lights, make_sky, nominal_rays

__all__ = ["_abi", "Scene", "Sky", "make_constants", "make_lights", "make_sky", "nominal_rays"]
