"""ctypes binding of the CPU oracle (liboracle.so) and the reference-source golden tool.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- never by the product (cudapathtracer_amd).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REFGEN = os.path.join(HERE, "_ref", "refgen")


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


class OVec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class OTri(C.Structure):
    _fields_ = [("v0", C.c_int32), ("v1", C.c_int32), ("v2", C.c_int32), ("norm", OVec3), ("mat", C.c_int32)]


class OCamera(C.Structure):
    _fields_ = [("pos", OVec3), ("dist", C.c_float), ("focal", C.c_float), ("radius", C.c_float),
                ("w", C.c_int32), ("h", C.c_int32)]


class OXorwow(C.Structure):
    _fields_ = [("d", C.c_uint32), ("v", C.c_uint32 * 5)]


class OSphere(C.Structure):
    _fields_ = [("pos", OVec3), ("rad", C.c_float), ("diffuse", C.c_double * 3), ("emission", C.c_double * 3)]


class OScene(C.Structure):
    _fields_ = [("num_verts", C.c_uint32), ("num_tris", C.c_uint32), ("num_mats", C.c_uint32),
                ("num_lights", C.c_uint32), ("verts", C.c_void_p), ("tris", C.c_void_p), ("mats", C.c_void_p),
                ("lights", C.c_void_p), ("total_light_area", C.c_float), ("bvh", C.c_void_p),
                ("bvh_size", C.c_uint32),
                ("spheres", C.c_void_p), ("num_spheres", C.c_uint32)]


class OCounters(C.Structure):
    _fields_ = [("traces", C.c_uint64), ("node_tests", C.c_uint64), ("tri_tests", C.c_uint64),
                ("tri_counts", C.c_void_p)]


_libs = {}
# sensitivity variants of the restatement (oracle/Makefile VARIANTS; tools/parity/ref_gap.py)
VARIANTS = ("fma", "fma_notri", "libm", "ulp1", "ulp2", "unfused", "nvcc", "fma_tri", "fmal_tri", "fmar_tri")


def lib(variant=None):
    """The oracle library; variant = one of VARIANTS loads that sensitivity build instead (same ABI)."""
    h = _libs.get(variant)
    if h is None:
        path = LIB if variant is None else os.path.join(HERE, "variants", "liboracle_%s.so" % variant)
        if variant is not None and variant not in VARIANTS:
            raise ValueError("unknown oracle variant %r" % (variant,))
        if not os.path.exists(path):
            build()
        h = C.CDLL(path)
        h.or_xorwow_step_images.argtypes = [C.c_void_p]
        h.or_xorwow_jump_images.argtypes = [C.c_int, C.c_void_p]
        h.or_xorwow_init.argtypes = [C.c_uint64, C.c_uint64, C.POINTER(OXorwow)]
        h.or_xorwow_next.argtypes = [C.POINTER(OXorwow)]
        h.or_xorwow_next.restype = C.c_uint32
        h.or_uniform.argtypes = [C.POINTER(OXorwow)]
        h.or_uniform.restype = C.c_float
        h.or_sincos.argtypes = [C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        h.or_trace_batch.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
        h.or_trace_batch.restype = C.c_int
        h.or_trace_batch_counts.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        h.or_trace_batch_counts.restype = C.c_int
        h.or_tri_intersect.argtypes = [OVec3, OVec3, C.c_void_p, C.c_void_p]
        h.or_get_tangent.argtypes = [OVec3, C.POINTER(OVec3)]
        h.or_brdf.argtypes = [C.c_void_p, C.c_void_p]
        h.or_tri_intersect.restype = C.c_float
        h.or_ray_aabb.argtypes = [OVec3, OVec3, OVec3, OVec3]
        h.or_ray_aabb.restype = C.c_int
        h.or_morton_pxl_to_i.argtypes = [C.c_uint32, C.c_uint32]
        h.or_morton_pxl_to_i.restype = C.c_uint32
        h.or_camera_ray.argtypes = [C.POINTER(OCamera), C.c_uint32, C.c_float, C.c_float, C.POINTER(OVec3),
                                    C.POINTER(OVec3)]
        h.or_trace.argtypes = [C.POINTER(OScene), OVec3, OVec3, C.POINTER(C.c_int32), C.POINTER(C.c_float),
                               C.POINTER(OCounters)]
        h.or_trace.restype = C.c_int
        h.or_render.argtypes = [C.POINTER(OScene), C.POINTER(OCamera), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                C.c_uint64, C.c_void_p, C.c_uint32, C.c_int, C.c_void_p, C.POINTER(OCounters)]
        h.or_render.restype = C.c_int
        h.or_write_ppm_imgbuf.argtypes = [C.c_char_p, C.c_void_p, C.c_int, C.c_int]
        h.or_write_ppm_imgbuf.restype = C.c_int
        _libs[variant] = h
    return h


class OracleScene:
    """Holds numpy copies of the scene arrays (reference layouts) and the OScene view."""

    def __init__(self, arrays):
        self.verts = np.ascontiguousarray(arrays["verts"])
        self.tris = np.ascontiguousarray(arrays["tris"])
        self.mats = np.ascontiguousarray(arrays["mats"])
        self.lights = np.ascontiguousarray(arrays["lights"], dtype=np.uint32)
        self.bvh = np.ascontiguousarray(arrays["bvh"])
        s = OScene()
        s.num_verts, s.num_tris, s.num_mats, s.num_lights = len(self.verts), len(self.tris), len(self.mats), len(
            self.lights)
        s.verts, s.tris, s.mats = self.verts.ctypes.data, self.tris.ctypes.data, self.mats.ctypes.data
        s.lights = self.lights.ctypes.data if len(self.lights) else None
        s.total_light_area = float(arrays["total_light_area"])
        s.bvh = self.bvh.ctypes.data if len(self.bvh) else None
        s.bvh_size = len(self.bvh)
        sph = arrays.get("spheres")
        self.spheres = np.ascontiguousarray(sph) if sph is not None and len(sph) else None
        s.spheres = self.spheres.ctypes.data if self.spheres is not None else None
        s.num_spheres = 0 if self.spheres is None else len(self.spheres)
        self.c = s


def camera(pos, dist_from_film, focal_length, radius, width, height):
    c = OCamera()
    c.pos = OVec3(*pos)
    c.dist, c.focal, c.radius, c.w, c.h = dist_from_film, focal_length, radius, width, height
    return c


def render(scene: OracleScene, cam: OCamera, width, height, spp, bounces=3, integrator=0, seed=1234, pixels=None,
           threads=0, tri_counts=None, variant=None):
    """f64 mean image (H, W, 3); pixels = iterable of y*W+x (default: all).  Returns (img, counters).
    tri_counts: optional uint32[num_tris] array the per-triangle test counts are added to
    (kernel.cu:133 test[k] += 1).  variant: a sensitivity build (VARIANTS) instead of the oracle."""
    if pixels is None:
        pixels = np.arange(width * height, dtype=np.uint32)
    pixels = np.ascontiguousarray(pixels, dtype=np.uint32)
    out = np.zeros((height, width, 3), dtype=np.float64)
    cnt = OCounters()
    if tri_counts is not None:
        assert tri_counts.dtype == np.uint32 and tri_counts.flags.c_contiguous and len(tri_counts) == scene.c.num_tris
        cnt.tri_counts = tri_counts.ctypes.data
    rc = lib(variant).or_render(C.byref(scene.c), C.byref(cam), width, height, spp, bounces, integrator, seed,
                         pixels.ctypes.data, len(pixels), threads, out.ctypes.data, C.byref(cnt))
    if rc != 0:
        raise RuntimeError("or_render failed: %d" % rc)
    return out, dict(traces=cnt.traces, node_tests=cnt.node_tests, tri_tests=cnt.tri_tests)


def trace(scene: OracleScene, o, d):
    tri, t = C.c_int32(), C.c_float()
    cnt = OCounters()
    rc = lib().or_trace(C.byref(scene.c), OVec3(*o), OVec3(*d), C.byref(tri), C.byref(t), C.byref(cnt))
    if rc != 0:
        raise RuntimeError("stack overflow")
    return tri.value, t.value


def trace_batch(scene: OracleScene, origins, directions, tri_counts=None):
    """or_trace over many rays (OpenMP): returns (tri int32[n], t float32[n]); tri_counts (optional
    uint32[num_tris]) accumulates the per-triangle test counts of kernel.cu:133."""
    o = np.ascontiguousarray(origins, dtype=np.float32).reshape(-1, 3)
    d = np.ascontiguousarray(directions, dtype=np.float32).reshape(-1, 3)
    rays = np.ascontiguousarray(np.concatenate([o, d], axis=1))
    n = len(rays)
    tri = np.empty(n, dtype=np.int32)
    t = np.empty(n, dtype=np.float32)
    if tri_counts is not None:
        assert tri_counts.dtype == np.uint32 and tri_counts.flags.c_contiguous and len(tri_counts) == scene.c.num_tris
    cp = tri_counts.ctypes.data if tri_counts is not None else None
    if lib().or_trace_batch_counts(C.byref(scene.c), n, rays.ctypes.data, tri.ctypes.data, t.ctypes.data, cp) != 0:
        raise RuntimeError("stack overflow")
    return tri, t


def xorwow_stream(seed, subsequence, n):
    st = OXorwow()
    lib().or_xorwow_init(seed, subsequence, C.byref(st))
    return np.array([lib().or_xorwow_next(C.byref(st)) for _ in range(n)], dtype=np.uint32)


def uniform_stream(seed, subsequence, n):
    st = OXorwow()
    lib().or_xorwow_init(seed, subsequence, C.byref(st))
    return np.array([lib().or_uniform(C.byref(st)) for _ in range(n)], dtype=np.float32)


def jump_images(log2_steps):
    img = np.zeros(800, dtype=np.uint32)
    lib().or_xorwow_jump_images(log2_steps, img.ctypes.data)
    return img


def helpers(normals, albedos, variant=None):
    """kernel.cu:44-54 getTangent of each normal (f32 (n, 3)) and :101-104 BRDF of each albedo (f64 (n, 3)),
    as the restatement computes them."""
    L = lib(variant)
    nrm = np.ascontiguousarray(normals, dtype=np.float32).reshape(-1, 3)
    alb = np.ascontiguousarray(albedos, dtype=np.float64).reshape(-1, 3)
    tan = np.empty_like(nrm)
    brdf = np.empty_like(alb)
    t = OVec3()
    out = np.empty(3, dtype=np.float64)
    for i in range(len(nrm)):
        L.or_get_tangent(OVec3(*nrm[i]), C.byref(t))
        tan[i] = (t.x, t.y, t.z)
    for i in range(len(alb)):
        L.or_brdf(alb[i].ctypes.data, out.ctypes.data)
        brdf[i] = out
    return tan, brdf


def refgen_available():
    return os.path.exists(REFGEN)


def write_ppm_imgbuf(path, imgbuf, width, height):
    """kernel.cu:763-778 restated: the reference's PPM loop over a Morton-indexed (W*H, 3) buffer
    (its imgBuffer_host, f64; an fp32 buffer is widened exactly)."""
    buf = np.ascontiguousarray(imgbuf, dtype=np.float64).reshape(-1)
    assert buf.size == width * height * 3
    if lib().or_write_ppm_imgbuf(str(path).encode(), buf.ctypes.data, int(width), int(height)) != 0:
        raise OSError("or_write_ppm_imgbuf: cannot write %s" % path)


def ref_ppm_imgbuf(imgbuf, width, height, workdir):
    """The reference's OWN loop (refgen ppm: kernel.cu:763-778 compiled verbatim) on the same buffer;
    returns the PPM bytes.  Build container only (needs oracle/_ref/refgen)."""
    buf = np.ascontiguousarray(imgbuf, dtype=np.float64).reshape(-1)
    inp = os.path.join(workdir, "imgbuf.bin")
    buf.tofile(inp)
    subprocess.check_call([REFGEN, "ppm", inp, str(width), str(height)], cwd=workdir)
    with open(os.path.join(workdir, "image.ppm"), "rb") as fh:
        return fh.read()
