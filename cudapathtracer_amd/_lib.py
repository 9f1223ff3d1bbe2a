"""ctypes declarations for libptamd.so (include/pt/pt.h).  No compute happens in Python.

The library is built in-tree (``python __graft_entry__.py build`` or
``make -C cudapathtracer_amd/csrc``).  If it is missing this module raises immediately: there
is no Python or CPU fallback for the render path.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PT_LIB selects an experiment build (tools/build_variants.sh); the default is the in-tree library
LIB_PATH = os.environ.get("PT_LIB") or os.path.join(_HERE, "libptamd.so")

PT_OK = 0
PT_E_INVALID, PT_E_IO, PT_E_SCENE, PT_E_BVH_DEPTH, PT_E_HIP, PT_E_NODEV, PT_E_OOM = -1, -2, -3, -4, -5, -6, -7
PT_INTEGRATOR_UNIDIR, PT_INTEGRATOR_HEAD = 0, 1
PT_FLAG_REFERENCE_TRAVERSAL = 0x1
PT_FLAG_NO_DEAD_PATH_SKIP = 0x2
PT_FLAG_NO_PRIMARY_CACHE = 0x4
PT_FLAG_COUNT = 0x8
PT_FLAG_REFERENCE_BVH = 0x10
PT_FLAG_TRI_COUNTS = 0x20
PT_ORDER_SCANLINE, PT_ORDER_MORTON = 0, 1
PT_LIGHT_SPHERE = 0x80000000     # lights[] entry of an emissive sphere
ABI_VERSION = 6                 # PT_ABI_VERSION of include/pt/pt.h these bindings mirror
PT_BVH_LEAF_FLAG = 0x80000000


class Vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class Triangle(C.Structure):
    _fields_ = [("v0", C.c_int32), ("v1", C.c_int32), ("v2", C.c_int32), ("norm", Vec3), ("mat", C.c_int32)]


class Material(C.Structure):
    _fields_ = [("albedo", C.c_double * 3), ("emission", C.c_double * 3)]


class BvhNode(C.Structure):
    _fields_ = [("lo", Vec3), ("hi", Vec3), ("left", C.c_uint32), ("right", C.c_uint32)]


class Camera(C.Structure):
    _fields_ = [("pos", Vec3), ("dist_from_film", C.c_float), ("focal_length", C.c_float), ("radius", C.c_float),
                ("pxl_width", C.c_int32), ("pxl_height", C.c_int32)]


class Sphere(C.Structure):   # sphere.h:7-12 (pt_sphere)
    _fields_ = [("pos", Vec3), ("rad", C.c_float), ("diffuse", C.c_double * 3), ("emission", C.c_double * 3)]


class SceneView(C.Structure):
    _fields_ = [("num_verts", C.c_uint32), ("num_tris", C.c_uint32), ("num_mats", C.c_uint32),
                ("num_lights", C.c_uint32), ("verts", C.POINTER(Vec3)), ("tris", C.POINTER(Triangle)),
                ("mats", C.POINTER(Material)), ("lights", C.POINTER(C.c_uint32)), ("total_light_area", C.c_float),
                ("bvh", C.POINTER(BvhNode)), ("bvh_size", C.c_uint32), ("bvh_depth", C.c_int32),
                ("spheres", C.POINTER(Sphere)), ("num_spheres", C.c_uint32)]


class Params(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("spp", C.c_int32), ("bounces", C.c_int32),
                ("integrator", C.c_int32), ("flags", C.c_uint32), ("seed", C.c_uint64),
                ("shard_index", C.c_int32), ("shard_count", C.c_int32), ("pixel_order", C.c_int32),
                ("tile_w", C.c_int32), ("tile_h", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [("seconds", C.c_double), ("kernel_ms", C.c_double), ("samples", C.c_uint64),
                ("rays_traced", C.c_uint64), ("rays_reference", C.c_uint64), ("rays_nominal", C.c_uint64),
                ("node_tests", C.c_uint64), ("tri_tests", C.c_uint64), ("walk_lane_slots", C.c_uint64),
                ("leaf_steps", C.c_uint64), ("shade_lane_slots", C.c_uint64), ("accel_fallbacks", C.c_uint64),
                ("walk_cycles", C.c_uint64), ("shade_cycles", C.c_uint64), ("spill_entries", C.c_uint64),
                ("lds_node_tests", C.c_uint64), ("work_units", C.c_uint64), ("split_pixels", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


assert C.sizeof(Vec3) == 12 and C.sizeof(Triangle) == 28 and C.sizeof(Material) == 48
assert C.sizeof(BvhNode) == 32 and C.sizeof(Camera) == 32

# symbol -> (restype, argtypes); the list IS the exported surface of include/pt/pt.h
SIGNATURES = {
    "pt_abi_version": (C.c_int, []),
    "pt_last_error": (C.c_char_p, []),
    "pt_scene_new": (C.c_void_p, []),
    "pt_scene_free": (None, [C.c_void_p]),
    "pt_scene_load_obj": (C.c_int, [C.c_void_p, C.c_char_p, C.c_char_p, Vec3, C.c_float, C.c_int]),
    "pt_scene_last_warning": (C.c_char_p, [C.c_void_p]),
    "pt_scene_build_bvh": (C.c_int, [C.c_void_p]),
    "pt_scene_add_sphere": (C.c_int, [C.c_void_p, C.POINTER(Sphere)]),
    "pt_scene_view": (C.c_int, [C.c_void_p, C.POINTER(SceneView)]),
    "pt_morton_pxl_to_i": (C.c_uint32, [C.c_uint32, C.c_uint32]),
    "pt_morton_i_to_pxl": (None, [C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "pt_camera_ray": (None, [C.POINTER(Camera), C.c_uint32, C.c_int, C.c_float, C.c_float,
                             C.POINTER(Vec3), C.POINTER(Vec3)]),
    "pt_write_ppm": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int, C.c_int]),
    "pt_write_ppm_f64": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int, C.c_int]),
    "pt_write_ppm_order": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int, C.c_int, C.c_int]),
    "pt_tonemap_u8": (C.c_int, [C.c_double]),
    "pt_accel_digest": (C.c_int, [C.POINTER(SceneView), C.POINTER(C.c_uint64), C.POINTER(C.c_uint32),
                                  C.POINTER(C.c_int32)]),
    "pt_create": (C.c_void_p, [C.POINTER(SceneView), C.c_int, C.POINTER(C.c_int)]),
    "pt_render": (C.c_int, [C.c_void_p, C.POINTER(Params), C.POINTER(Camera), C.c_void_p, C.POINTER(Stats)]),
    "pt_render_device": (C.c_int, [C.c_void_p, C.POINTER(Params), C.POINTER(Camera), C.c_void_p, C.c_void_p,
                                   C.POINTER(Stats)]),
    "pt_render_device_async": (C.c_int, [C.c_void_p, C.POINTER(Params), C.POINTER(Camera), C.c_void_p, C.c_void_p]),
    "pt_render_wait": (C.c_int, [C.c_void_p, C.POINTER(Stats)]),
    "pt_trace": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]),
    "pt_trace_counts": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                  C.c_void_p, C.POINTER(C.c_uint64)]),
    "pt_tri_counts": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    "pt_tonemap_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p]),
    "pt_tonemap": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "pt_write_ppm_codes": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int, C.c_int]),
    "pt_write_pfm": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int, C.c_int]),
    "pt_shard_pixels": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_uint32,
                                  C.POINTER(C.c_uint32)]),
    "pt_group_create": (C.c_void_p, [C.POINTER(C.c_void_p), C.c_int, C.POINTER(C.c_int)]),
    "pt_group_size": (C.c_int, [C.c_void_p]),
    "pt_render_group": (C.c_int, [C.c_void_p, C.POINTER(Params), C.POINTER(Camera), C.c_void_p, C.POINTER(Stats)]),
    "pt_group_destroy": (None, [C.c_void_p]),
    "pt_render_multi": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.POINTER(Params), C.POINTER(Camera), C.c_void_p,
                                  C.POINTER(Stats)]),
    "pt_destroy": (None, [C.c_void_p]),
}

_lib = None


def _torch_runtime_first():
    """One process, two HIP runtimes: PyTorch's ROCm wheel bundles its own (torch/lib/libamdhip64.so, loaded by path),
    libptamd.so links the system's (libamdhip64.so.7).  With this library's runtime up first, PyTorch then finds no
    device ("no ROCm-capable device is detected", profiles/r06_async_dbg); with PyTorch's first, both work (every suite
    and bench run).  So when PyTorch is importable and sees a GPU, its runtime is initialised before the library is
    loaded (PT_NO_TORCH_FIRST=1 skips this; the C-ABI itself never needs PyTorch)."""
    if os.environ.get("PT_NO_TORCH_FIRST"):
        return
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.is_available():
        torch.cuda.init()


def lib():
    """Load libptamd.so once; raise loudly if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                "libptamd.so not found at %s: build it with `python __graft_entry__.py build` "
                "(there is no fallback render path)" % LIB_PATH)
        _torch_runtime_first()
        handle = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        if handle.pt_abi_version() != ABI_VERSION:
            raise RuntimeError("libptamd.so ABI %d, bindings expect %d: rebuild it" % (handle.pt_abi_version(), ABI_VERSION))
        _lib = handle
    return _lib


class PtError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("pt error %d: %s" % (code, msg))
        self.code = code


def check(rc):
    if rc != PT_OK:
        raise PtError(rc, (lib().pt_last_error() or b"").decode(errors="replace"))
    return rc
