#!/usr/bin/env python3
"""Generate tests/golden/* from the REFERENCE's own sources (oracle/_ref/refgen) and the oracle.

Run in the build container (needs /root/reference to build refgen):
    make -C oracle && python tools/make_golden.py

Outputs (all small, committed):
  scenes/models/*.obj|.mtl           fixture scenes authored by cudapathtracer_amd.scenes
  scene_<name>.npz                   verts/tris/mats/lights/bvh + meta from the reference's
                                     loadOBJ (modelLoader.h:125) and buildBVH (BVH.h:443)
  standin.json                       sha256 of the same arrays for the 262K-tri stand-in
  kat_tri.npz / kat_aabb.npz         triIntersect / rayAABBIntersect inputs and reference outputs
  kat_cam.npz / kat_morton.npz       cameraRay / Morton maps
  kat_tone.npz                       PPM tone map (int)(gammaCorrect(normalized(c), 1/2.2) * 255)
  xorwow.npz                         oracle XORWOW streams (regression pin)
  render_*.npz                       oracle f64 mean images for small configs (regression pin)
  kat_trace_<scene>.npz              the reference's own trace() (kernel.cu:107-161, compiled from
                                     /root/reference/kernel.cu by oracle/Makefile) on the ray sets of
                                     tests/raysets.py: (triIndex, t) per ray + per-triangle test[]
                                     counts (kernel.cu:133) summed over the rays

  kat_ppm_morton.npz                 the reference's own PPM loop (kernel.cu:763-778, compiled verbatim:
                                     refgen ppm) over a Morton-indexed imgBuffer_host (64x64 f32 values
                                     incl. 0, huge, inf, NaN): the input buffer and the PPM bytes

`python tools/make_golden.py --only trace|ppm` regenerates only the kat_trace_* / kat_ppm_* files.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from cudapathtracer_amd import scenes  # noqa: E402
from cudapathtracer_amd.api import MAT, NODE, TRI, VEC3  # noqa: E402
import oracle  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tests"))
from raysets import bounce_rays, ray_sets  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
SCENES = os.path.join(GOLD, "scenes")
REFGEN = oracle.REFGEN

# name -> list of (obj, origin, scale, flip)   (kernel.cu:590-599 style load lists)
SCENE_SETS = {
    "cornell": [("models/cornell.obj", (0, 0, 0), 1.0, 0)],
    "cornell_blob": [("models/cornell.obj", (0, 0, 0), 1.0, 0), ("models/blob.obj", (0.35, 0.6, 0.3), 0.75, 0)],
    "quirks": [("models/quirks.obj", (0, 0, 0), 1.0, 0)],
    "blob_flip": [("models/blob.obj", (0.1, -0.2, 0.3), 1.5, 1)],
    "nomtl": [("models/nomtl.obj", (0, 0, 0), 1.0, 0)],
    "quad": [("models/quad.obj", (0, 0, 0), 1.0, 0)],
}

# two triangles only (one emissive quad facing the camera): the render path's tree is a root node with
# two single-triangle leaves (accel_build.cpp never makes the root a leaf)
QUAD_OBJ = ("mtllib quad.mtl\nusemtl panel\nv -1 0 -1\nv 1 0 -1\nv 1 2 -1\nv -1 2 -1\nf 1 2 3\nf 1 3 4\n")
QUAD_MTL = "newmtl panel\nKd 0.6 0.5 0.4\nKe 3 2.5 2\n"

NOMTL_OBJ = ("v 0 0 0\nv 1 0 0\nv 0 1 0\nv 1 1 0\nusemtl a\nf 1 2 3\n"
             "mtllib does_not_exist.mtl\nf 2 4 3\nusemtl b\nf 1 2 4\n")


def write_quad():
    os.makedirs(os.path.join(SCENES, "models"), exist_ok=True)
    with open(os.path.join(SCENES, "models", "quad.obj"), "w") as fh:
        fh.write(QUAD_OBJ)
    with open(os.path.join(SCENES, "models", "quad.mtl"), "w") as fh:
        fh.write(QUAD_MTL)


def run_ref(args, cwd=None):
    subprocess.check_call([REFGEN] + [str(a) for a in args], cwd=cwd, stdout=subprocess.DEVNULL)


def ref_scene(tmp, name, loads):
    pre = os.path.join(tmp, name)
    args = ["scene", pre]
    for obj, origin, scale, flip in loads:
        args += [obj, origin[0], origin[1], origin[2], scale, flip]
    run_ref(args, cwd=SCENES)
    meta = open(pre + ".meta.txt").read().split()
    return dict(
        verts=np.fromfile(pre + ".verts.bin", VEC3), tris=np.fromfile(pre + ".tris.bin", TRI),
        mats=np.fromfile(pre + ".mats.bin", MAT), lights=np.fromfile(pre + ".lights.bin", "<u4"),
        bvh=np.fromfile(pre + ".bvh.bin", NODE),
        total_light_area=np.float32(float.fromhex(meta[5])), bvh_depth=np.int32(int(meta[7])))


def kat_tri(tmp, rng):
    n = 6000
    o = rng.uniform(-2, 2, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    v0 = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    v1 = (v0 + rng.normal(scale=0.7, size=(n, 3))).astype(np.float32)
    v2 = (v0 + rng.normal(scale=0.7, size=(n, 3))).astype(np.float32)
    # aim half of the rays at a point inside the triangle (hits), some exactly at edges/vertices
    k = n // 2
    w = rng.dirichlet([1, 1, 1], size=k)
    w[: k // 8, 2] = 0.0
    w[: k // 8] /= w[: k // 8].sum(1, keepdims=True)
    w[k // 8: k // 4] = [1.0, 0.0, 0.0]
    p = w[:, :1] * v0[:k] + w[:, 1:2] * v1[:k] + w[:, 2:] * v2[:k]
    dd = p - o[:k]
    d[:k] = (dd / np.linalg.norm(dd, axis=1, keepdims=True)).astype(np.float32)
    # degenerate / parallel / axis-aligned cases
    d[k:k + 200] = np.array([0, 0, 1], np.float32)
    v1[k + 200:k + 400] = v0[k + 200:k + 400]                      # zero-area
    d[k + 400:k + 600] = (v1 - v0)[k + 400:k + 600] / np.linalg.norm((v1 - v0)[k + 400:k + 600], axis=1,
                                                                      keepdims=True)   # parallel to edge
    rec = np.concatenate([o, d, v0, v1, v2], 1).astype(np.float32)
    rec.tofile(os.path.join(tmp, "tri.in"))
    run_ref(["tri", os.path.join(tmp, "tri.in"), os.path.join(tmp, "tri.out")])
    t = np.fromfile(os.path.join(tmp, "tri.out"), "<f4")
    np.savez_compressed(os.path.join(GOLD, "kat_tri.npz"), rec=rec, t=t)


def kat_aabb(tmp, rng):
    n = 6000
    o = rng.uniform(-2, 2, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    lo = rng.uniform(-1, 0.5, (n, 3)).astype(np.float32)
    hi = (lo + rng.uniform(0, 1, (n, 3))).astype(np.float32)
    # axis-parallel rays, origins on slab planes (0/0 -> NaN), flat boxes
    d[:600, rng.integers(0, 3, 600)] = 0.0
    d[:300, 0] = 0.0
    o[100:400, 0] = lo[100:400, 0]
    hi[400:800, 1] = lo[400:800, 1]
    d[800:1000] = np.array([0, -1, 0], np.float32)
    d[1000:1100] = np.array([-0.0, 0.0, 1.0], np.float32)
    rec = np.concatenate([o, d, lo, hi], 1).astype(np.float32)
    rec.tofile(os.path.join(tmp, "aabb.in"))
    run_ref(["aabb", os.path.join(tmp, "aabb.in"), os.path.join(tmp, "aabb.out")])
    hit = np.fromfile(os.path.join(tmp, "aabb.out"), "<u1")
    np.savez_compressed(os.path.join(GOLD, "kat_aabb.npz"), rec=rec, hit=hit)


def kat_cam(tmp, rng):
    # radius-0 cameras: lens angle kept in (0, pi/2) so the reference's lens term r*cos, r*sin is +0
    # (with cos/sin < 0 it is -0 and only flips the sign of a zero direction component; in the
    # reference those draws come from the racy state[0], kernel.cu:547).  The last camera has a
    # real lens (compared within 1 ulp: cosf/sinf vs the deterministic kernel sin/cos).
    cams = [((0.0, 1.0, 3.0), 1.0, 3.0, 0.0, 512, 512), ((0.0, 2.6, 13.2), 1.0, 3.0, 0.0, 1920, 1080),
            ((0.5, -1.0, 2.0), 2.0, 1.5, 0.0, 97, 61), ((0.0, 1.0, 3.0), 1.0, 3.0, 0.05, 64, 64)]
    out = {}
    for ci, (pos, dist, focal, radius, w, h) in enumerate(cams):
        camb = np.zeros(8, dtype=np.float32)
        camb[:3] = pos
        camb[3:6] = (dist, focal, radius)
        camb = camb.tobytes()[:24] + np.array([w, h], dtype=np.int32).tobytes()
        n = 4000
        ys = rng.integers(0, h, n)
        xs = rng.integers(0, w, n)
        idx = np.array([scenes_morton(x, y) for x, y in zip(xs, ys)], dtype=np.uint32)
        u = rng.uniform(0, 1, (n, 2)).astype(np.float32)
        if radius == 0.0:
            u[:, 1] = rng.uniform(1e-3, 0.24, n).astype(np.float32)
        inb = camb + np.concatenate([idx[:, None].view(np.float32), u], 1).astype(np.float32).tobytes()
        open(os.path.join(tmp, "cam.in"), "wb").write(inb)
        run_ref(["cam", os.path.join(tmp, "cam.in"), os.path.join(tmp, "cam.out")])
        ray = np.fromfile(os.path.join(tmp, "cam.out"), "<f4").reshape(n, 6)
        out["cam%d" % ci] = np.array([*pos, dist, focal, radius, w, h], dtype=np.float64)
        out["idx%d" % ci] = idx
        out["u%d" % ci] = u
        out["ray%d" % ci] = ray
    np.savez_compressed(os.path.join(GOLD, "kat_cam.npz"), **out)


def scenes_morton(x, y):
    r = 0
    for b in range(16):
        r |= ((int(x) >> b) & 1) << (2 * b)
        r |= ((int(y) >> b) & 1) << (2 * b + 1)
    return r


def kat_morton(tmp):
    n = 1 << 16
    run_ref(["morton", os.path.join(tmp, "morton.out"), n])
    m = np.fromfile(os.path.join(tmp, "morton.out"), "<u4").reshape(n, 2)
    np.savez_compressed(os.path.join(GOLD, "kat_morton.npz"), xy=m[:, 0], back=m[:, 1])


def kat_helpers(tmp, rng):
    """getTangent (kernel.cu:44-54) and BRDF (:101-104) from the reference's own code (refgen helpers):
    random unit normals, the axis directions of both signs, ties |n.y| == |n.z| (where getTangent's strict
    '>' picks c2), and the fixture scenes' face normals; random albedos and the scenes' material albedos."""
    n_rand = 4000
    nr = rng.normal(size=(n_rand, 3))
    nr /= np.linalg.norm(nr, axis=1, keepdims=True)
    axes = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float64)
    a = rng.uniform(0.1, 1.0, 200)
    ties = np.stack([rng.uniform(-1, 1, 200), a, a * rng.choice([-1.0, 1.0], 200)], axis=1)
    ties /= np.linalg.norm(ties, axis=1, keepdims=True)
    face = [load_scene_normals(n) for n in ("cornell", "cornell_blob")]
    nrm = np.concatenate([nr, axes, ties] + face).astype(np.float32)
    alb = rng.uniform(0, 1, (len(nrm), 3))
    mats = np.concatenate([np.load(os.path.join(GOLD, "scene_%s.npz" % n))["mats"]["albedo"] for n in ("cornell", "quirks")])
    alb[: len(mats)] = mats
    rec = np.zeros(len(nrm), dtype=[("n", "<f4", (3,)), ("pad", "<f4"), ("alb", "<f8", (3,))])
    rec["n"] = nrm
    rec["alb"] = alb
    rec.tofile(os.path.join(tmp, "helpers.in"))
    run_ref(["helpers", os.path.join(tmp, "helpers.in"), os.path.join(tmp, "helpers.out")])
    out = np.fromfile(os.path.join(tmp, "helpers.out"), dtype=rec.dtype)
    np.savez_compressed(os.path.join(GOLD, "kat_helpers.npz"), normal=nrm, albedo=alb, tangent=out["n"], brdf=out["alb"])


def load_scene_normals(name):
    tris = np.load(os.path.join(GOLD, "scene_%s.npz" % name))["tris"]
    return np.stack([tris["nx"], tris["ny"], tris["nz"]], axis=1).astype(np.float64)


def kat_tone(tmp, rng):
    c = np.concatenate([rng.exponential(1.0, 3000), rng.uniform(0, 1e-3, 300), [0.0, 1e-300, 1.0, 3.0, 1e6, 1e300],
                        rng.uniform(0, 20, 700)]).astype(np.float64)
    c = c[: (len(c) // 3) * 3].reshape(-1, 3)
    c.tofile(os.path.join(tmp, "tone.in"))
    run_ref(["tone", os.path.join(tmp, "tone.in"), os.path.join(tmp, "tone.out")])
    v = np.fromfile(os.path.join(tmp, "tone.out"), "<i4").reshape(-1, 3)
    np.savez_compressed(os.path.join(GOLD, "kat_tone.npz"), c=c, v=v)


def xorwow_fixture():
    subs = [0, 1, 2, 3, 1023, 1 << 20, (1 << 22) - 1]
    out = {"subs": np.array(subs, dtype=np.uint64)}
    for s in subs:
        out["raw_%d" % s] = oracle.xorwow_stream(1234, s, 64)
        out["uni_%d" % s] = oracle.uniform_stream(1234, s, 64)
    np.savez_compressed(os.path.join(GOLD, "xorwow.npz"), **out)


def render_fixtures():
    import cudapathtracer_amd as pt
    cfgs = [("cornell_blob", 32, 32, 4, 3, 0), ("cornell_blob", 32, 32, 4, 3, 1), ("cornell", 24, 16, 3, 8, 0)]
    for name, w, h, spp, bounces, integ in cfgs:
        s = pt.Scene()
        for obj, origin, scale, flip in SCENE_SETS[name]:
            s.load_obj(os.path.join(SCENES, obj), origin, scale, flip, mtl_basepath=os.path.join(SCENES, "models") + "/")
        s.build_bvh()
        osc = oracle.OracleScene(s.arrays())
        cam = oracle.camera((0.0, 1.0, 3.0), 1.0, 3.0, 0.0, w, h)
        img, cnt = oracle.render(osc, cam, w, h, spp, bounces, integ, 1234)
        np.savez_compressed(os.path.join(GOLD, "render_%s_%dx%d_s%d_b%d_i%d.npz" % (name, w, h, spp, bounces, integ)),
                            img=img, traces=np.uint64(cnt["traces"]))


def ref_trace(tmp, rays, loads, cwd):
    """(tri, t, counts) from the reference's trace() on the scene of `loads` (refgen trace)."""
    rin, rout, rcnt = (os.path.join(tmp, "trace." + k) for k in ("in", "out", "cnt"))
    np.ascontiguousarray(rays, dtype=np.float32).tofile(rin)
    args = ["trace", rin, rout, rcnt]
    for obj, origin, scale, flip in loads:
        args += [obj, origin[0], origin[1], origin[2], scale, flip]
    run_ref(args, cwd=cwd)
    res = np.fromfile(rout, "<i4").reshape(-1, 2)
    return res[:, 0].copy(), res[:, 1].copy().view(np.float32), np.fromfile(rcnt, "<u4")


def kat_trace(tmp):
    """trace() goldens: the ray sets of tests/raysets.py plus first-bounce rays off the interior
    set's hits; for the stand-in, camera rays of the bench view and their bounces first."""
    jobs = [(name, SCENE_SETS[name], SCENES, 1024, None) for name in ("cornell", "cornell_blob", "quirks")]
    gen = os.path.join(tmp, "gen_trace")
    p = scenes.write_sponza_standin(gen)
    jobs.append(("standin", [(os.path.relpath(p, gen), (0, 0, 0), 1.0, 0)], gen, 512, p))
    for name, loads, cwd, n, standin in jobs:
        arrs = ref_scene(tmp, name, loads) if standin is None else None
        if standin is not None:
            import cudapathtracer_amd as pt
            s = pt.Scene()
            s.load_obj(standin, mtl_basepath=os.path.dirname(standin) + "/")
            s.build_bvh()
            arrs = s.arrays()
        sets = []
        if standin is not None:
            import cudapathtracer_amd as pt
            c = scenes.SPONZA_STANDIN_CAMERA
            cam = pt.make_camera(c["pos"], c["dist_from_film"], c["focal_length"], 0.0, 1920, 1080)
            idx = np.random.default_rng(9).integers(0, 1920 * 1080, 4 * n)
            cr = [pt.camera_ray(cam, int(i), lens=False) for i in idx]
            sets.append(("camera", np.array([r[0] for r in cr], np.float32), np.array([r[1] for r in cr], np.float32)))
        for k, (o, d) in ray_sets(arrs, n, 5 if standin is None else 11).items():
            sets.append((k, o, d))
        first = sets[0]
        tri0, t0, _ = ref_trace(tmp, np.concatenate([first[1], first[2]], 1), loads, cwd)
        bo, bd = bounce_rays(arrs, first[1], first[2], tri0, t0, 6 if standin is None else 10)
        sets.append(("bounce", bo, bd))
        rays = np.concatenate([np.concatenate([o, d], 1) for _, o, d in sets]).astype(np.float32)
        tri, t, counts = ref_trace(tmp, rays, loads, cwd)
        offs = np.cumsum([0] + [len(o) for _, o, _ in sets]).astype(np.int64)
        np.savez_compressed(os.path.join(GOLD, "kat_trace_%s.npz" % name), rays=rays, tri=tri, t=t, counts=counts,
                            set_names=np.array([k for k, _, _ in sets]), set_offsets=offs)
        print("kat_trace", name, len(rays), "rays,", int((tri >= 0).sum()), "hits,", int(counts.sum()), "tests")


def kat_ppm_morton(tmp):
    """The reference's PPM loop (kernel.cu:763-778) over a Morton-indexed 64x64 imgBuffer_host."""
    rng = np.random.default_rng(763)
    w = h = 64
    buf = (rng.random((w * h, 3)) * rng.choice([0.01, 1.0, 30.0], size=(w * h, 1))).astype(np.float32)
    buf[:8] = [[0, 0, 0], [1e30, 3e38, np.inf], [np.nan, 1, 2], [1e-30, 0.5, 1e-7], [2.0, 0.25, 255.0],
               [0.0123, 0.9, 7.5], [1.0, 1.0, 1.0], [100.0, 1000.0, 1e4]]
    d = os.path.join(tmp, "ppm")
    os.makedirs(d, exist_ok=True)
    ppm = oracle.ref_ppm_imgbuf(buf, w, h, d)
    np.savez_compressed(os.path.join(GOLD, "kat_ppm_morton.npz"), buf=buf, w=w, h=h,
                        ppm=np.frombuffer(ppm, dtype=np.uint8))
    print("kat_ppm_morton", len(ppm), "bytes")


def main():
    if not os.path.exists(REFGEN):
        sys.exit("oracle/_ref/refgen missing: run `make -C oracle` with /root/reference present")
    if sys.argv[1:] == ["--only", "trace"]:
        with tempfile.TemporaryDirectory() as tmp:
            kat_trace(tmp)
        return
    if sys.argv[1:] == ["--only", "helpers"]:
        with tempfile.TemporaryDirectory() as tmp:
            kat_helpers(tmp, np.random.default_rng(20261017))
        return
    if sys.argv[1:] == ["--only", "quad"]:
        write_quad()
        with tempfile.TemporaryDirectory() as tmp:
            arrs = ref_scene(tmp, "quad", SCENE_SETS["quad"])
            np.savez_compressed(os.path.join(GOLD, "scene_quad.npz"), **arrs)
            print("scene quad", len(arrs["tris"]), "tris, depth", int(arrs["bvh_depth"]))
        return
    if sys.argv[1:] == ["--only", "ppm"]:
        with tempfile.TemporaryDirectory() as tmp:
            kat_ppm_morton(tmp)
        return
    os.makedirs(GOLD, exist_ok=True)
    if os.path.isdir(SCENES):
        shutil.rmtree(SCENES)
    scenes.write_cornell(SCENES)
    scenes.write_blob(SCENES, level=3)
    scenes.write_quirks(SCENES)
    with open(os.path.join(SCENES, "models", "nomtl.obj"), "w") as fh:
        fh.write(NOMTL_OBJ)
    write_quad()
    rng = np.random.default_rng(20261015)
    with tempfile.TemporaryDirectory() as tmp:
        for name, loads in SCENE_SETS.items():
            arrs = ref_scene(tmp, name, loads)
            np.savez_compressed(os.path.join(GOLD, "scene_%s.npz" % name), **arrs)
            print("scene", name, len(arrs["tris"]), "tris, depth", int(arrs["bvh_depth"]))
        gen = os.path.join(tmp, "gen")
        p = scenes.write_sponza_standin(gen)
        pre = os.path.join(tmp, "standin")
        run_ref(["scene", pre, os.path.relpath(p, gen), 0, 0, 0, 1, 0], cwd=gen)
        digest = {}
        for part in ("verts", "tris", "mats", "lights", "bvh"):
            digest[part] = hashlib.sha256(open("%s.%s.bin" % (pre, part), "rb").read()).hexdigest()
        meta = open(pre + ".meta.txt").read().split()
        digest["meta"] = meta
        digest["obj_sha256"] = hashlib.sha256(open(p, "rb").read()).hexdigest()
        with open(os.path.join(GOLD, "standin.json"), "w") as fh:
            json.dump(digest, fh, indent=1)
        print("standin", meta)
        kat_tri(tmp, rng)
        kat_aabb(tmp, rng)
        kat_cam(tmp, rng)
        kat_morton(tmp)
        kat_tone(tmp, rng)
        kat_helpers(tmp, rng)
        kat_trace(tmp)
        kat_ppm_morton(tmp)
    xorwow_fixture()
    render_fixtures()
    print("golden fixtures written to", GOLD)


if __name__ == "__main__":
    main()
