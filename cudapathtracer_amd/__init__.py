"""cudapathtracer_amd -- MI355X-native (gfx950) re-authoring of CulDeVu/CUDAPathTracer's
per-pixel path-integration loop behind a C-ABI (include/pt/pt.h, libptamd.so).

Host surface (OBJ ingest, BVH build, camera, PPM) is C++ in csrc/host; the render path is
hand-written HIP in csrc/hip.  Python here is only orchestration over ctypes.
"""
from ._lib import (PT_FLAG_COUNT, PT_FLAG_NO_DEAD_PATH_SKIP, PT_FLAG_NO_PRIMARY_CACHE,  # noqa: F401
                   PT_FLAG_REFERENCE_TRAVERSAL, PT_FLAG_REFERENCE_BVH, PT_FLAG_TRI_COUNTS, PT_INTEGRATOR_HEAD, PT_INTEGRATOR_UNIDIR, PtError, LIB_PATH, PT_E_INVALID,
                   PT_LIGHT_SPHERE, PT_ORDER_SCANLINE, PT_ORDER_MORTON)
from . import api  # noqa: F401
from .api import (Group, Renderer, Scene, camera_ray, make_camera, morton_i_to_pxl, morton_pxl_to_i,  # noqa: F401
                  tonemap_u8, write_ppm, write_ppm_codes, write_pfm, read_pfm)

__all__ = ["Scene", "Renderer", "Group", "make_camera", "camera_ray", "morton_pxl_to_i", "morton_i_to_pxl", "write_ppm", "write_ppm_codes", "write_pfm", "read_pfm",
           "tonemap_u8", "PtError"]
