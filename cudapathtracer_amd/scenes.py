"""Scene authoring: deterministic OBJ/MTL writers for the parity fixtures and the bench.

The reference ships no models (`/root/reference/.gitignore:1` ignores `models/`), so every
scene used here is authored by this module and written as OBJ/MTL text that goes through the
same ingest path a real model would (tinyobj semantics, `modelLoader.h:125-210`):

* ``write_cornell``   -- a Cornell box (walls, two boxes, a ceiling light whose normal is -y,
                         the emitter orientation `kernel.cu:503` hard-codes).
* ``write_blob``      -- a displaced icosphere, the stand-in for `teapot.obj` (`kernel.cu:592`).
* ``write_quirks``    -- an OBJ exercising the tinyobj 0.9.13 corners (fan triangulation,
                         negative / v/vt/vn indices, ``usemtl``/``g``/``o`` splits, unknown
                         material, unparseable ``.5`` floats, CRLF, tabs).
* ``write_sponza_standin`` -- a procedural ~262K-triangle architectural atrium (columns,
                         arcades, galleries, drapes, vases) with a -y-facing roof light.  It is
                         a STAND-IN for Sponza (absent from this container) and every result
                         measured on it is labelled so.  ``PT_SPONZA_OBJ`` selects a real file.

Cameras follow `camera.h:26-34`; the Cornell one is `kernel.cu:642-648` verbatim.
"""
from __future__ import annotations

import math
import os

import numpy as np

# camera.h:26-34 fields: pos, distFromFilm, focalLength, radius, pxlWidth, pxlHeight
CORNELL_CAMERA = dict(pos=(0.0, 1.0, 3.0), dist_from_film=1.0, focal_length=3.0, radius=0.0)  # kernel.cu:642-648
SPONZA_STANDIN_CAMERA = dict(pos=(0.0, 2.6, 13.2), dist_from_film=1.0, focal_length=3.0, radius=0.0)

# ----------------------------------------------------------------------------- writers


class _ObjWriter:
    """Accumulates vertices/faces and writes OBJ text with explicit usemtl/o/g groups."""

    def __init__(self):
        self.lines: list[str] = []
        self.nv = 0

    def raw(self, s: str):
        self.lines.append(s)

    def verts(self, v: np.ndarray) -> int:
        """Append vertices (N,3); return the 1-based index of the first."""
        base = self.nv + 1
        v = np.asarray(v, dtype=np.float64).reshape(-1, 3)
        self.lines.append("\n".join("v %.6f %.6f %.6f" % (a, b, c) for a, b, c in v))
        self.nv += len(v)
        return base

    def faces(self, f: np.ndarray, base: int):
        f = np.asarray(f, dtype=np.int64).reshape(len(f), -1) + base
        self.lines.append("\n".join("f " + " ".join(str(int(i)) for i in row) for row in f))

    def text(self) -> str:
        return "\n".join(s for s in self.lines if s) + "\n"


def _oriented_quad(p, want_normal):
    """Order 4 coplanar corners so the fan's face normal (v1-v0)x(v2-v0) agrees with want_normal."""
    p = [np.asarray(x, dtype=np.float64) for x in p]
    n = np.cross(p[1] - p[0], p[2] - p[0])
    if np.dot(n, want_normal) < 0:
        p = [p[0], p[3], p[2], p[1]]
    return np.array(p)


def _grid(nu, nv, fn):
    """Grid mesh: fn(u,v) -> (N,3) for u,v in [0,1]; returns verts and triangle faces (0-based)."""
    u = np.linspace(0.0, 1.0, nu + 1)
    v = np.linspace(0.0, 1.0, nv + 1)
    uu, vv = np.meshgrid(u, v, indexing="ij")
    pts = fn(uu.ravel(), vv.ravel())
    idx = np.arange((nu + 1) * (nv + 1)).reshape(nu + 1, nv + 1)
    a = idx[:-1, :-1].ravel()
    b = idx[1:, :-1].ravel()
    c = idx[1:, 1:].ravel()
    d = idx[:-1, 1:].ravel()
    tris = np.concatenate([np.stack([a, b, c], 1), np.stack([a, c, d], 1)])
    return pts, tris


def _orient_tris(pts, tris, outward_fn):
    """Flip triangles whose geometric normal disagrees with outward_fn(centroid)."""
    v0, v1, v2 = pts[tris[:, 0]], pts[tris[:, 1]], pts[tris[:, 2]]
    n = np.cross(v1 - v0, v2 - v0)
    want = outward_fn((v0 + v1 + v2) / 3.0)
    flip = np.einsum("ij,ij->i", n, want) < 0
    tris = tris.copy()
    tris[flip] = tris[flip][:, [0, 2, 1]]
    return tris


def _icosphere(level):
    t = (1.0 + 5 ** 0.5) / 2.0
    v = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    f = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2),
         (10, 7, 6), (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11),
         (6, 2, 10), (8, 6, 7), (9, 8, 1)]
    verts = [np.array(p, dtype=np.float64) / np.linalg.norm(p) for p in v]
    faces = list(f)
    for _ in range(level):
        cache = {}

        def mid(a, b):
            key = (min(a, b), max(a, b))
            if key not in cache:
                m = verts[a] + verts[b]
                verts.append(m / np.linalg.norm(m))
                cache[key] = len(verts) - 1
            return cache[key]

        nf = []
        for a, b, c in faces:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        faces = nf
    return np.array(verts), np.array(faces, dtype=np.int64)


def _blob_points(level, seed, amp=0.18):
    v, f = _icosphere(level)
    rng = np.random.default_rng(seed)
    k = rng.normal(size=(6, 3))
    ph = rng.uniform(0, 2 * math.pi, size=6)
    disp = 1.0 + amp * np.mean(np.sin(v @ k.T * 2.5 + ph), axis=1)
    return v * disp[:, None], f


def _write_atomic(path, text):
    tmp = "%s.tmp%d" % (path, os.getpid())
    with open(tmp, "w", newline="") as fh:
        fh.write(text)
    os.replace(tmp, path)


def _write(dirpath, name, obj_text, mtl_text=None):
    """MTL first, then the OBJ, each written to a private temp file and renamed into place: a
    process that sees the OBJ (e.g. another rank of a multi-GPU bench sharing the scene cache)
    sees both files complete."""
    models = os.path.join(dirpath, "models")
    os.makedirs(models, exist_ok=True)
    p = os.path.join(models, name + ".obj")
    if mtl_text is not None:
        _write_atomic(os.path.join(models, name + ".mtl"), mtl_text)
    _write_atomic(p, obj_text)
    return p


# ----------------------------------------------------------------------------- Cornell

CORNELL_MTL = """# Cornell box materials (authored for this repo)
newmtl white
Kd 0.725 0.71 0.68
newmtl red
Kd 0.63 0.065 0.05
newmtl green
Kd 0.14 0.45 0.091
newmtl light
Kd 0.78 0.78 0.78
Ke 17 12 4
"""


def _box(cx, cz, hx, hz, h, ang):
    c, s = math.cos(ang), math.sin(ang)
    loc = [(-hx, -hz), (hx, -hz), (hx, hz), (-hx, hz)]
    ring = [(cx + x * c - z * s, cz + x * s + z * c) for x, z in loc]
    quads = []
    ctr = np.array([cx, h / 2, cz])
    for i in range(4):
        (x0, z0), (x1, z1) = ring[i], ring[(i + 1) % 4]
        q = [(x0, 0, z0), (x1, 0, z1), (x1, h, z1), (x0, h, z0)]
        fc = np.mean(np.array(q), axis=0)
        quads.append(_oriented_quad(q, fc - ctr))
    quads.append(_oriented_quad([(x, h, z) for x, z in ring], (0, 1, 0)))
    return quads


def cornell_quads():
    W = []
    W.append(("white", _oriented_quad([(-1, 0, -1), (-1, 0, 1), (1, 0, 1), (1, 0, -1)], (0, 1, 0))))     # floor
    W.append(("white", _oriented_quad([(-1, 2, -1), (1, 2, -1), (1, 2, 1), (-1, 2, 1)], (0, -1, 0))))     # ceiling
    W.append(("white", _oriented_quad([(-1, 0, -1), (1, 0, -1), (1, 2, -1), (-1, 2, -1)], (0, 0, 1))))    # back
    W.append(("red", _oriented_quad([(-1, 0, -1), (-1, 2, -1), (-1, 2, 1), (-1, 0, 1)], (1, 0, 0))))      # left
    W.append(("green", _oriented_quad([(1, 0, -1), (1, 0, 1), (1, 2, 1), (1, 2, -1)], (-1, 0, 0))))       # right
    for q in _box(-0.33, -0.3, 0.3, 0.3, 1.2, 0.29):                                                       # tall box
        W.append(("white", q))
    for q in _box(0.35, 0.35, 0.29, 0.29, 0.6, -0.3):                                                      # short box
        W.append(("white", q))
    W.append(("light", _oriented_quad([(-0.24, 1.98, -0.22), (0.23, 1.98, -0.22), (0.23, 1.98, 0.16),
                                       (-0.24, 1.98, 0.16)], (0, -1, 0))))                                 # light
    return W


def write_cornell(dirpath, name="cornell"):
    """Write models/<name>.obj/.mtl; one usemtl group per material run (quads -> fan triangles)."""
    w = _ObjWriter()
    w.raw("# Cornell box authored for the MI355X path tracer parity fixtures")
    w.raw("mtllib %s.mtl" % name)
    cur = None
    for mat, q in cornell_quads():
        if mat != cur:
            w.raw("g %s_%d" % (mat, w.nv))
            w.raw("usemtl %s" % mat)
            cur = mat
        b = w.verts(q)
        w.faces(np.array([[0, 1, 2, 3]]), b)
    return _write(dirpath, name, w.text(), CORNELL_MTL)


# ----------------------------------------------------------------------------- blob

def write_blob(dirpath, level=3, seed=7, name="blob"):
    """Displaced icosphere (20*4^level triangles), outward normals; stand-in for teapot.obj."""
    v, f = _blob_points(level, seed)
    f = _orient_tris(v, f, lambda c: c)
    w = _ObjWriter()
    w.raw("mtllib %s.mtl" % name)
    w.raw("o blob")
    w.raw("usemtl clay")
    b = w.verts(v)
    w.faces(f, b)
    return _write(dirpath, name, w.text(), "newmtl clay\nKd 0.8 0.75 0.6\n")


# ----------------------------------------------------------------------------- quirks

QUIRKS_OBJ = (
    "# tinyobj 0.9.13 corner cases\r\n"
    "mtllib quirks.mtl\r\n"
    "o first_object\r\n"
    "v 0 0 0\r\n"
    "v 1.0 0 0\r\n"
    "v +1 1e0 -0.0\r\n"
    "v .5 1 0.25\r\n"
    "v 1.5E-1 2.25e+1 3\r\n"
    "v\t-2 -3 -4\r\n"
    "v 0.1 0.2 0.30000000000000004\r\n"
    "v 123456.789 -0.000123 7e-3\r\n"
    "vt 0.5 0.5\r\n"
    "vn 0 0 1\r\n"
    "usemtl matA\r\n"
    "f 1 2 3\r\n"
    "f 1/1 2/1 3/1 4/1\r\n"
    "g group1 extra_name\r\n"
    "usemtl matB\r\n"
    "f -3//1 -2//1 -1//1\r\n"
    "f 1/1/1 2/1/1 3/1/1 4/1/1 5/1/1\r\n"
    "  f   2 7 8  \r\n"
    "usemtl no_such_material\r\n"
    "f 2 3 4\r\n"
    "f 5 6\r\n"
    "usemtl glow\r\n"
    "f 6 7 8\r\n"
    "o second\r\n"
    "f 1 5 6\r\n"
)

QUIRKS_MTL = (
    "# materials\n"
    "newmtl matA\n"
    "Ka 0.1 0.1 0.1\n"
    "Kd 0.5 0.25 0.125\n"
    "Ns 10\n"
    "illum 2\n"
    "newmtl matB\n"
    "Kd\t1e-1 .7 -0.5\n"
    "d 0.5\n"
    "newmtl glow\n"
    "Kd 0.3 0.3 0.3\n"
    "Ke 2.5 0 1\n"
    "map_Kd tex.png\n"
    "foo bar baz\n"
)


def write_quirks(dirpath):
    return _write(dirpath, "quirks", QUIRKS_OBJ, QUIRKS_MTL)


# ----------------------------------------------------------------------------- Sponza stand-in

STANDIN_SCALE = 0.69  # -> 262,782 triangles (Sponza-class, ~262K)

STANDIN_MTL = """# Sponza-class procedural stand-in materials
newmtl floor
Kd 0.55 0.5 0.42
newmtl stone
Kd 0.62 0.58 0.5
newmtl column
Kd 0.7 0.66 0.58
newmtl cloth_red
Kd 0.6 0.08 0.06
newmtl cloth_blue
Kd 0.08 0.12 0.55
newmtl cloth_green
Kd 0.1 0.45 0.12
newmtl plant
Kd 0.2 0.5 0.15
newmtl vase
Kd 0.55 0.3 0.18
newmtl light
Kd 0.8 0.8 0.8
Ke 20 19 17
"""


def _cyl(cx, cz, r, y0, y1, nseg, nring):
    def fn(u, v):
        a = 2 * math.pi * u
        rr = r * (1.0 + 0.08 * np.cos(v * 2 * math.pi * 3) * (v < 0.15))
        return np.stack([cx + rr * np.cos(a), y0 + (y1 - y0) * v, cz + rr * np.sin(a)], 1)
    p, t = _grid(nseg, nring, fn)
    return p, _orient_tris(p, t, lambda c: c - np.stack([np.full(len(c), cx), c[:, 1], np.full(len(c), cz)], 1))


def _arch(x, z0, z1, y_spring, thick, depth, nseg):
    """Semicircular arch band between two columns at (x, z0) and (x, z1), extruded along x."""
    zc = 0.5 * (z0 + z1)
    R = 0.5 * (z1 - z0)
    out_p, out_t = [], []
    n = 0
    for (r_in, r_out) in [(R - thick, R)]:
        for face in range(4):
            def fn(u, v, face=face):
                a = math.pi * u
                if face == 0:      # intrados
                    rr = np.full_like(u, r_in); xx = x - depth / 2 + depth * v
                elif face == 1:    # extrados
                    rr = np.full_like(u, r_out); xx = x - depth / 2 + depth * v
                elif face == 2:    # front
                    rr = r_in + (r_out - r_in) * v; xx = np.full_like(u, x - depth / 2)
                else:              # back
                    rr = r_in + (r_out - r_in) * v; xx = np.full_like(u, x + depth / 2)
                return np.stack([xx, y_spring + rr * np.sin(a), zc - rr * np.cos(a)], 1)
            p, t = _grid(nseg, 2, fn)
            cen = np.array([x, y_spring, zc])
            if face == 0:
                t = _orient_tris(p, t, lambda c: cen - np.stack([np.full(len(c), x), c[:, 1], c[:, 2]], 1) + np.array([0, 0, 0]) * 0)
            elif face == 1:
                t = _orient_tris(p, t, lambda c: np.stack([np.zeros(len(c)), c[:, 1] - y_spring, c[:, 2] - zc], 1))
            elif face == 2:
                t = _orient_tris(p, t, lambda c: np.tile([-1.0, 0, 0], (len(c), 1)))
            else:
                t = _orient_tris(p, t, lambda c: np.tile([1.0, 0, 0], (len(c), 1)))
            out_p.append(p)
            out_t.append(t + n)
            n += len(p)
    return np.concatenate(out_p), np.concatenate(out_t)


def _drape(x, z0, z1, y0, y1, nu, nv, seed):
    rng = np.random.default_rng(seed)
    ph = rng.uniform(0, 2 * math.pi, 3)

    def fn(u, v):
        z = z0 + (z1 - z0) * u
        y = y1 - (y1 - y0) * v
        xx = x + 0.12 * np.sin(u * 2 * math.pi * 4 + ph[0]) * (0.3 + v) + 0.04 * np.sin(v * 9 + ph[1])
        y = y - 0.25 * np.sin(u * math.pi) * v
        return np.stack([xx, y, z], 1)
    return _grid(nu, nv, fn)


def sponza_standin_meshes(scale_tris=1.0):
    """Return [(material, verts(N,3), faces(M,3))] for the stand-in atrium."""
    S = scale_tris
    out = []
    X, Z, H = 6.0, 14.0, 12.0
    # floor (normal +y) and walls (normals inward)
    p, t = _grid(int(96 * S ** 0.5), int(224 * S ** 0.5),
                 lambda u, v: np.stack([-X + 2 * X * u, np.zeros_like(u), -Z + 2 * Z * v], 1))
    out.append(("floor", p, _orient_tris(p, t, lambda c: np.tile([0, 1.0, 0], (len(c), 1)))))
    for sx in (-1, 1):
        p, t = _grid(int(112 * S ** 0.5), int(48 * S ** 0.5),
                     lambda u, v, sx=sx: np.stack([np.full_like(u, sx * X), H * v, -Z + 2 * Z * u], 1))
        out.append(("stone", p, _orient_tris(p, t, lambda c, sx=sx: np.tile([-sx, 0, 0.0], (len(c), 1)))))
    for sz in (-1, 1):
        p, t = _grid(int(48 * S ** 0.5), int(48 * S ** 0.5),
                     lambda u, v, sz=sz: np.stack([-X + 2 * X * u, H * v, np.full_like(u, sz * Z)], 1))
        out.append(("stone", p, _orient_tris(p, t, lambda c, sz=sz: np.tile([0, 0, -sz * 1.0], (len(c), 1)))))
    # gallery slabs (ceilings of the side aisles at y=4.6 and 9.2), normals down and up
    for sx in (-1, 1):
        for y in (4.6, 9.2):
            for nrm in (-1.0, 1.0):
                yy = y + (0.0 if nrm < 0 else 0.3)
                p, t = _grid(int(16 * S ** 0.5), int(112 * S ** 0.5),
                             lambda u, v, sx=sx, yy=yy: np.stack([sx * (4.3 + 1.7 * u), np.full_like(u, yy), -Z + 2 * Z * v], 1))
                out.append(("stone", p, _orient_tris(p, t, lambda c, nrm=nrm: np.tile([0, nrm, 0.0], (len(c), 1)))))
    # columns: two storeys, two rows
    zs = np.arange(-12.0, 12.01, 3.0)
    nseg, nring = int(40 * S ** 0.5), int(20 * S ** 0.5)
    for sx in (-1, 1):
        for z in zs:
            for (y0, y1, r) in ((0.0, 4.6, 0.32), (4.9, 9.2, 0.24)):
                p, t = _cyl(sx * 4.3, z, r, y0, y1, nseg, nring)
                out.append(("column", p, t))
    # arcades between columns (springing at 3.2 / 7.9)
    for sx in (-1, 1):
        for i in range(len(zs) - 1):
            for ys in (3.2, 7.9):
                p, t = _arch(sx * 4.3, zs[i] + 0.3, zs[i + 1] - 0.3, ys, 0.35, 0.6, int(48 * S ** 0.5))
                out.append(("stone", p, t))
    # drapes hanging from the upper gallery
    cloths = ("cloth_red", "cloth_blue", "cloth_green")
    k = 0
    for sx in (-1, 1):
        for i in range(0, len(zs) - 1, 2):
            p, t = _drape(sx * 3.7, zs[i] + 0.4, zs[i + 1] - 0.4, 5.4, 8.9, int(48 * S ** 0.5), int(64 * S ** 0.5), 11 + k)
            out.append((cloths[k % 3], p, t))
            k += 1
    # vases with plants along the nave
    for j, z in enumerate(np.arange(-10.5, 10.6, 3.0)):
        for sx in (-1, 1):
            v, f = _blob_points(4, 100 + j * 2 + (sx > 0))
            cen = np.array([sx * 2.6, 0.55, z])
            vv = v * np.array([0.45, 0.55, 0.45]) + cen
            f = _orient_tris(vv, f, lambda c, cen=cen: c - cen)
            out.append(("vase", vv, f))
            v2, f2 = _blob_points(3, 500 + j * 2 + (sx > 0), amp=0.35)
            cen2 = np.array([sx * 2.6, 1.45, z])
            vv2 = v2 * np.array([0.6, 0.5, 0.6]) + cen2
            f2 = _orient_tris(vv2, f2, lambda c, cen2=cen2: c - cen2)
            out.append(("plant", vv2, f2))
    # roof light over the open atrium, facing -y (kernel.cu:503 assumes (0,-1,0))
    q = _oriented_quad([(-2.0, H - 0.05, -9.0), (2.0, H - 0.05, -9.0), (2.0, H - 0.05, 9.0), (-2.0, H - 0.05, 9.0)],
                       (0, -1, 0))
    out.append(("light", q, np.array([[0, 1, 2], [0, 2, 3]])))
    return out


def write_sponza_standin(dirpath, name="sponza_standin", scale_tris=STANDIN_SCALE):
    w = _ObjWriter()
    w.raw("# Procedural Sponza-class STAND-IN (not Sponza); authored for the MI355X path tracer bench")
    w.raw("mtllib %s.mtl" % name)
    for i, (mat, p, t) in enumerate(sponza_standin_meshes(scale_tris)):
        w.raw("g part%d" % i)
        w.raw("usemtl %s" % mat)
        b = w.verts(p)
        w.faces(t, b)
    return _write(dirpath, name, w.text(), STANDIN_MTL)


def standin_triangle_count(scale_tris=STANDIN_SCALE):
    return int(sum(len(t) for _, _, t in sponza_standin_meshes(scale_tris)))


# ----------------------------------------------------------------------------- spheres (C1)
# A Cornell box made of sphere.h spheres only: walls are radius-100
# spheres (f32-friendly: the quadratic's oc.oc - r^2 cancels ~1e4, not smallpt's 1e10), two
# diffuse balls and a small emissive sphere under the ceiling.  Camera: CORNELL_CAMERA.
CORNELL_SPHERES = [
    # pos, rad, diffuse, emission
    ((-101.0, 1.0, 0.0), 100.0, (0.75, 0.25, 0.25), (0.0, 0.0, 0.0)),     # left wall
    ((101.0, 1.0, 0.0), 100.0, (0.25, 0.25, 0.75), (0.0, 0.0, 0.0)),      # right wall
    ((0.0, 1.0, -101.0), 100.0, (0.75, 0.75, 0.75), (0.0, 0.0, 0.0)),     # back wall
    ((0.0, -100.0, 0.0), 100.0, (0.75, 0.75, 0.75), (0.0, 0.0, 0.0)),     # floor
    ((0.0, 102.0, 0.0), 100.0, (0.75, 0.75, 0.75), (0.0, 0.0, 0.0)),      # ceiling
    ((-0.45, 0.35, -0.3), 0.35, (0.9, 0.9, 0.9), (0.0, 0.0, 0.0)),
    ((0.45, 0.35, 0.3), 0.35, (0.9, 0.9, 0.9), (0.0, 0.0, 0.0)),
    ((0.0, 1.85, 0.0), 0.12, (0.0, 0.0, 0.0), (12.0, 12.0, 12.0)),         # light
]


def add_cornell_spheres(scene, spheres=CORNELL_SPHERES):
    """Append the C1 spheres to a pt.Scene (returns it)."""
    for pos, rad, diffuse, emission in spheres:
        scene.add_sphere(pos, rad, diffuse, emission)
    return scene


# ----------------------------------------------------------------------------- stack stress (C5 row)
# "Splinters": long thin triangles crossing the whole box in random directions.  Every BVH box
# then spans most of the volume and a ray enters nearly all of them, so a BVH4 walk pushes ~3
# entries per level on its way down -- deeper than the 16-entry per-lane LDS ring, i.e. the
# HBM spill tier (the reference's fixed stack[64], kernel.cu:114, + depth guard :627-631) runs.
SPLINTERS_MTL = """# splinters (stack-depth stress scene) materials
newmtl splinter
Kd 0.6 0.55 0.5
newmtl light
Kd 0.8 0.8 0.8
Ke 15 15 15
"""


def write_splinters(dirpath, n=1024, seed=5, name="splinters"):
    rng = np.random.default_rng(seed)
    lo, hi = np.array([-1.0, 0.05, -1.0]), np.array([1.0, 1.95, 1.0])
    a = rng.uniform(lo, hi, (n, 3))
    b = rng.uniform(lo, hi, (n, 3))
    far = np.linalg.norm(b - a, axis=1) < 1.2            # keep them long: re-draw the end point
    b[far] = lo + hi - a[far]
    c = a + rng.normal(scale=0.02, size=(n, 3))           # thin: a sliver along a -> b
    w = _ObjWriter()
    w.raw("# splinters: %d long thin triangles in random directions (stack-depth stress)" % n)
    w.raw("mtllib %s.mtl" % name)
    w.raw("usemtl splinter")
    base = w.verts(np.stack([a, b, c], axis=1).reshape(-1, 3))
    w.faces(np.arange(3 * n).reshape(n, 3), base)
    w.raw("usemtl light")
    lb = w.verts([(-0.3, 1.99, -0.3), (0.3, 1.99, -0.3), (0.3, 1.99, 0.3), (-0.3, 1.99, 0.3)])
    w.faces([(0, 2, 1), (0, 3, 2)], lb)                   # facing -y (the NEE light normal, kernel.cu:503)
    return _write(dirpath, name, w.text(), SPLINTERS_MTL)
