"""Host-side mirror of the reference's render flow (kernel.cu:565-790) over the C-ABI.

    scene = Scene()
    scene.load_obj("models/CornellBox-Original.obj", (0, 0, 0), 1)      # loadOBJ, modelLoader.h:125
    scene.load_obj("models/teapot.obj", (0.35, 0.6, 0.3), 0.75)         # kernel.cu:591-592
    scene.build_bvh()                                                   # buildBVH, BVH.h:443 + guard :627
    cam = make_camera(pos=(0, 1, 3), dist_from_film=1, focal_length=3, radius=0,
                      width=512, height=512)                            # kernel.cu:642-648
    with Renderer(scene) as r:                                          # uploads, kernel.cu:664-700
        img, stats = r.render(cam, 512, 512, spp=99, bounces=3)         # NUM_SAMPLES-1 samples, :709
    write_ppm("image.ppm", img)                                         # kernel.cu:763-778

Every call goes through libptamd.so; arrays returned to Python are copies of the C++ host
scene (numpy structured views for tests) or the float32 image the gfx950 kernel wrote.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L

VEC3 = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4")])
TRI = np.dtype([("v0", "<i4"), ("v1", "<i4"), ("v2", "<i4"), ("nx", "<f4"), ("ny", "<f4"), ("nz", "<f4"),
                ("mat", "<i4")])
MAT = np.dtype([("albedo", "<f8", (3,)), ("emission", "<f8", (3,))])
NODE = np.dtype([("lo", "<f4", (3,)), ("hi", "<f4", (3,)), ("left", "<u4"), ("right", "<u4")])
SPHERE = np.dtype([("pos", "<f4", (3,)), ("rad", "<f4"), ("diffuse", "<f8", (3,)), ("emission", "<f8", (3,))])


def _arr(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    buf = C.string_at(ptr, n * dtype.itemsize)
    return np.frombuffer(buf, dtype=dtype).copy()


class Scene:
    """The reference's scene globals (modelLoader.h:43-47) as an object owned by libptamd."""

    def __init__(self):
        self._h = L.lib().pt_scene_new()
        if not self._h:
            raise MemoryError("pt_scene_new failed")

    def close(self):
        if self._h:
            L.lib().pt_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_obj(self, path, origin=(0.0, 0.0, 0.0), scale=1.0, flip_normals=False, mtl_basepath=None):
        """loadOBJ (modelLoader.h:125-210).  mtl_basepath=None is the reference's "models/"."""
        o = L.Vec3(*[float(v) for v in origin])
        L.check(L.lib().pt_scene_load_obj(self._h, str(path).encode(),
                                          None if mtl_basepath is None else str(mtl_basepath).encode(),
                                          o, float(scale), int(bool(flip_normals))))
        return self

    loadOBJ = load_obj

    @property
    def warning(self) -> str:
        return (L.lib().pt_scene_last_warning(self._h) or b"").decode(errors="replace")

    def build_bvh(self):
        """buildBVH (BVH.h:443-474) + the depth guard of kernel.cu:627-631."""
        L.check(L.lib().pt_scene_build_bvh(self._h))
        return self

    buildBVH = build_bvh

    def view(self) -> L.SceneView:
        v = L.SceneView()
        L.check(L.lib().pt_scene_view(self._h, C.byref(v)))
        return v

    def accel_digest(self):
        """(digest, BVH4 node count, BVH4 depth) of the render path's acceleration structure
        as pt_create would build it (host-only diagnostic)."""
        v = self.view()
        dg, n4, d4 = C.c_uint64(), C.c_uint32(), C.c_int32()
        L.check(L.lib().pt_accel_digest(C.byref(v), C.byref(dg), C.byref(n4), C.byref(d4)))
        return int(dg.value), int(n4.value), int(d4.value)

    def arrays(self):
        """Copies of verts/tris/mats/lights/bvh as numpy structured arrays (test surface)."""
        v = self.view()
        return dict(
            verts=_arr(v.verts, v.num_verts, VEC3),
            tris=_arr(v.tris, v.num_tris, TRI),
            mats=_arr(v.mats, v.num_mats, MAT),
            lights=_arr(v.lights, v.num_lights, np.dtype("<u4")),
            total_light_area=np.float32(v.total_light_area),
            bvh=_arr(v.bvh, v.bvh_size, NODE),
            bvh_depth=int(v.bvh_depth),
            spheres=_arr(v.spheres, v.num_spheres, SPHERE),
        )

    def add_sphere(self, pos, rad, diffuse, emission=(0.0, 0.0, 0.0)):
        """sphere.h primitive (this build's semantics); returns self."""
        sp = L.Sphere()
        sp.pos = L.Vec3(*[float(v) for v in pos])
        sp.rad = float(rad)
        for k in range(3):
            sp.diffuse[k] = float(diffuse[k])
            sp.emission[k] = float(emission[k])
        L.check(L.lib().pt_scene_add_sphere(self._h, C.byref(sp)))
        return self


def make_camera(pos=(0.0, 1.0, 3.0), dist_from_film=1.0, focal_length=3.0, radius=0.0, width=512, height=512):
    """camera.h:26-34 (defaults = kernel.cu:642-648)."""
    c = L.Camera()
    c.pos = L.Vec3(*[float(v) for v in pos])
    c.dist_from_film = float(dist_from_film)
    c.focal_length = float(focal_length)
    c.radius = float(radius)
    c.pxl_width = int(width)
    c.pxl_height = int(height)
    return c


def camera_ray(cam, idx, lens=False, u1=0.0, u2=0.0):
    o, d = L.Vec3(), L.Vec3()
    L.lib().pt_camera_ray(C.byref(cam), int(idx), int(bool(lens)), float(u1), float(u2), C.byref(o), C.byref(d))
    return (o.x, o.y, o.z), (d.x, d.y, d.z)


def morton_pxl_to_i(x, y):
    return int(L.lib().pt_morton_pxl_to_i(int(x), int(y)))


def morton_i_to_pxl(i):
    x, y = C.c_uint32(), C.c_uint32()
    L.lib().pt_morton_i_to_pxl(int(i), C.byref(x), C.byref(y))
    return x.value, y.value


def write_ppm(path, img, pixel_order=0, width=None, height=None):
    """kernel.cu:763-778 on a (H, W, 3) float32 or float64 mean image, or on a Morton-ordered
    (W*H, 3) float32 buffer (pixel_order=PT_ORDER_MORTON, width/height given)."""
    img = np.ascontiguousarray(img)
    if pixel_order == L.PT_ORDER_MORTON:
        if width is None or height is None:
            raise ValueError("write_ppm: a Morton-ordered buffer needs width and height")
        width, height = int(width), int(height)
        if width <= 0 or height <= 0 or img.size != width * height * 3:
            raise ValueError("write_ppm: Morton buffer holds %d values, width*height*3 = %d"
                             % (img.size, max(width, 0) * max(height, 0) * 3))
        img = np.ascontiguousarray(img, dtype=np.float32)
        L.check(L.lib().pt_write_ppm_order(str(path).encode(), img.ctypes.data, width, height, 1))
        return
    if pixel_order != L.PT_ORDER_SCANLINE:
        raise ValueError("write_ppm: unknown pixel_order %r" % (pixel_order,))
    h, w = img.shape[:2]
    if img.dtype == np.float64:
        L.check(L.lib().pt_write_ppm_f64(str(path).encode(), img.ctypes.data, w, h))
    else:
        img = np.ascontiguousarray(img, dtype=np.float32)
        L.check(L.lib().pt_write_ppm(str(path).encode(), img.ctypes.data, w, h))


def tonemap_u8(c):
    return int(L.lib().pt_tonemap_u8(float(c)))


def write_ppm_codes(path, codes):
    """The reference PPM text from (H, W, 3) int32 tone-map codes (e.g. Renderer.tonemap)."""
    codes = np.ascontiguousarray(codes, dtype=np.int32)
    h, w = codes.shape[:2]
    L.check(L.lib().pt_write_ppm_codes(str(path).encode(), codes.ctypes.data, w, h))


def write_pfm(path, img):
    """Lossless float dump (PFM, little-endian, rows bottom-up) of an (H, W, 3) mean image."""
    img = np.ascontiguousarray(img, dtype=np.float32)
    h, w = img.shape[:2]
    L.check(L.lib().pt_write_pfm(str(path).encode(), img.ctypes.data, w, h))


def read_pfm(path):
    """Inverse of write_pfm: (H, W, 3) float32."""
    with open(path, "rb") as fh:
        assert fh.readline().strip() == b"PF"
        w, h = (int(v) for v in fh.readline().split())
        scale = float(fh.readline())
        data = np.frombuffer(fh.read(), dtype="<f4" if scale < 0 else ">f4")
    return data.reshape(h, w, 3)[::-1].astype(np.float32)


class Renderer:
    """Device-resident scene on one GPU (pt_create) and the render call (pt_render)."""

    def __init__(self, scene: Scene, device: int = 0):
        err = C.c_int(0)
        self._scene_view = scene.view()
        self._h = L.lib().pt_create(C.byref(self._scene_view), int(device), C.byref(err))
        if not self._h:
            L.check(err.value if err.value != 0 else L.PT_E_HIP)
        self.device = device

    def close(self):
        if self._h:
            L.lib().pt_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def params(width, height, spp, bounces=3, integrator=0, seed=1234, flags=0, shard_index=0, shard_count=1,
               pixel_order=0, tile_w=0, tile_h=0):
        p = L.Params()
        p.width, p.height, p.spp, p.bounces = int(width), int(height), int(spp), int(bounces)
        p.integrator, p.flags, p.seed = int(integrator), int(flags), int(seed)
        p.shard_index, p.shard_count = int(shard_index), int(shard_count)
        p.pixel_order, p.tile_w, p.tile_h = int(pixel_order), int(tile_w), int(tile_h)
        return p

    def render(self, cam, width, height, spp, bounces=3, integrator=0, seed=1234, flags=0,
               shard_index=0, shard_count=1, pixel_order=0, tile_w=0, tile_h=0, out=None):
        """Returns (image float32, stats dict).  The image is (H, W, 3) in scanline order, or the
        reference's Morton-indexed imgBuff (W*H, 3) with pixel_order=PT_ORDER_MORTON.  `out`: a
        C-contiguous float32 array of W*H*3 values to render into (reused across frames)."""
        p = self.params(width, height, spp, bounces, integrator, seed, flags, shard_index, shard_count,
                        pixel_order, tile_w, tile_h)
        shape = (height * width, 3) if pixel_order == L.PT_ORDER_MORTON else (height, width, 3)
        if out is None:
            out = np.zeros(shape, dtype=np.float32)
        elif out.dtype != np.float32 or out.size != width * height * 3 or not out.flags.c_contiguous:
            raise ValueError("out must be a C-contiguous float32 array of W*H*3 values")
        st = L.Stats()
        L.check(L.lib().pt_render(self._h, C.byref(p), C.byref(cam), out.ctypes.data, C.byref(st)))
        return out, st.as_dict()

    def render_device(self, cam, d_out_ptr, width, height, spp, bounces=3, integrator=0, seed=1234, flags=0,
                      shard_index=0, shard_count=1, stream_ptr=None, pixel_order=0, tile_w=0, tile_h=0):
        """Render this shard into a caller-owned, zero-filled device buffer (e.g. a torch tensor)."""
        p = self.params(width, height, spp, bounces, integrator, seed, flags, shard_index, shard_count,
                        pixel_order, tile_w, tile_h)
        st = L.Stats()
        L.check(L.lib().pt_render_device(self._h, C.byref(p), C.byref(cam), C.c_void_p(int(d_out_ptr)),
                                         None if stream_ptr is None else C.c_void_p(int(stream_ptr)), C.byref(st)))
        return st.as_dict()

    def render_device_async(self, cam, d_out_ptr, width, height, spp, bounces=3, integrator=0, seed=1234, flags=0,
                            shard_index=0, shard_count=1, stream_ptr=None, pixel_order=0, tile_w=0, tile_h=0):
        """Enqueue render_device's work on the stream and return at once (at most 2 in flight); collect
        the stats of the oldest with wait()."""
        p = self.params(width, height, spp, bounces, integrator, seed, flags, shard_index, shard_count,
                        pixel_order, tile_w, tile_h)
        L.check(L.lib().pt_render_device_async(self._h, C.byref(p), C.byref(cam), C.c_void_p(int(d_out_ptr)),
                                               None if stream_ptr is None else C.c_void_p(int(stream_ptr))))

    def wait(self):
        """Stats dict of the oldest render in flight (render_device_async), once it has finished."""
        st = L.Stats()
        L.check(L.lib().pt_render_wait(self._h, C.byref(st)))
        return st.as_dict()

    def tonemap(self, img):
        """Output step on the GPU: (H, W, 3) float32 mean image -> int32 codes equal to
        pt_tonemap_u8 (kernel.cu:763-778) per channel."""
        img = np.ascontiguousarray(img, dtype=np.float32)
        h, w = img.shape[:2]
        codes = np.empty(img.shape, dtype=np.int32)
        L.check(L.lib().pt_tonemap(self._h, img.ctypes.data, w, h, codes.ctypes.data))
        return codes

    def tri_counts(self):
        """Per-triangle test counts (uint32[num_tris], original ids) of the last render with
        PT_FLAG_COUNT -- the reference's test[] buffer (kernel.cu:133, :694-697)."""
        n = int(self._scene_view.num_tris)
        out = np.zeros(n, dtype=np.uint32)
        L.check(L.lib().pt_tri_counts(self._h, out.ctypes.data, n))
        return out

    def trace_counts(self, origins, directions, reference_bvh=False):
        """trace() plus diagnostics: returns (tri, t, tri_counts uint32[num_tris], spill_entries)."""
        rays, n = self._rays(origins, directions)
        tri = np.empty(n, dtype=np.int32)
        t = np.empty(n, dtype=np.float32)
        counts = np.zeros(int(self._scene_view.num_tris), dtype=np.uint32)
        spills = C.c_uint64(0)
        L.check(L.lib().pt_trace_counts(self._h, n, rays.ctypes.data, tri.ctypes.data, t.ctypes.data,
                                        L.PT_FLAG_REFERENCE_BVH if reference_bvh else 0, counts.ctypes.data,
                                        C.byref(spills)))
        return tri, t, counts, int(spills.value)

    @staticmethod
    def _rays(origins, directions):
        o = np.ascontiguousarray(origins, dtype=np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(directions, dtype=np.float32).reshape(-1, 3)
        if o.shape != d.shape:
            raise ValueError("origins and directions differ in shape")
        return np.ascontiguousarray(np.concatenate([o, d], axis=1)), len(o)

    def trace(self, origins, directions, reference_bvh=False):
        """The reference's trace() (kernel.cu:112-161) for a batch of rays: returns
        (tri int32[n] original triangle index or -1, t float32[n] closestT, 1e5 on a miss)."""
        rays, n = self._rays(origins, directions)
        tri = np.empty(n, dtype=np.int32)
        t = np.empty(n, dtype=np.float32)
        L.check(L.lib().pt_trace(self._h, n, rays.ctypes.data, tri.ctypes.data, t.ctypes.data,
                                 L.PT_FLAG_REFERENCE_BVH if reference_bvh else 0))
        return tri, t


class Group:
    """One process, N GPUs (pt_group_*): renderer i renders image-tile shard i of N, and one RCCL
    reduce over xGMI sums the shards into the first renderer's device (bit-identical to one GPU).
    The renderers must live on distinct devices and outlive the group."""

    def __init__(self, renderers):
        self._renderers = list(renderers)
        arr = (C.c_void_p * len(self._renderers))(*[r._h for r in self._renderers])
        err = C.c_int(0)
        self._h = L.lib().pt_group_create(arr, len(self._renderers), C.byref(err))
        if not self._h:
            L.check(err.value if err.value != 0 else L.PT_E_HIP)

    def close(self):
        if self._h:
            L.lib().pt_group_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def render(self, cam, width, height, spp, bounces=3, integrator=0, seed=1234, flags=0, pixel_order=0,
               tile_w=0, tile_h=0, out=None):
        """Returns (image float32 (H, W, 3) -- (W*H, 3) in Morton order --, summed stats dict)."""
        p = Renderer.params(width, height, spp, bounces, integrator, seed, flags, 0, 1, pixel_order, tile_w, tile_h)
        shape = (height * width, 3) if pixel_order == L.PT_ORDER_MORTON else (height, width, 3)
        if out is None:
            out = np.zeros(shape, dtype=np.float32)
        elif out.dtype != np.float32 or out.size != width * height * 3 or not out.flags.c_contiguous:
            raise ValueError("out must be a C-contiguous float32 array of W*H*3 values")
        st = L.Stats()
        L.check(L.lib().pt_render_group(self._h, C.byref(p), C.byref(cam), out.ctypes.data, C.byref(st)))
        return out, st.as_dict()
