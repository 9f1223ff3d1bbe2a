"""The CPU oracle (oracle/pt_oracle.c) pinned against the reference's own code and published data:
- triIntersect / rayAABBIntersect / cameraRay outputs of the reference sources (refgen), bit-exact;
- trace() (kernel.cu:107-161, the reference's own function compiled by oracle/Makefile): winners,
  closestT and per-triangle test counts on four scenes incl. the 262K stand-in, bit-exact;
- the XORWOW recurrence and 2^67 subsequence jump against rocRAND's precomputed matrices;
- its own committed render fixtures (regression pin) and a brute-force restatement of trace().
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import golden, load_scene

import oracle

ROCRAND_PRE = "/opt/rocm/include/rocrand/rocrand_xorwow_precomputed.h"


def test_tri_intersect_matches_reference():
    g = golden("kat_tri.npz")
    rec, t = g["rec"], g["t"]
    L = oracle.lib()
    for i in range(len(rec)):
        r = rec[i]
        verts = (oracle.OVec3 * 3)(oracle.OVec3(*r[6:9]), oracle.OVec3(*r[9:12]), oracle.OVec3(*r[12:15]))
        tri = oracle.OTri(0, 1, 2, oracle.OVec3(0, 0, 0), 0)
        got = L.or_tri_intersect(oracle.OVec3(*r[0:3]), oracle.OVec3(*r[3:6]), C.addressof(verts), C.addressof(tri))
        assert np.float32(got).tobytes() == np.float32(t[i]).tobytes(), i


def test_ray_aabb_matches_reference():
    """Including axis-parallel rays, origins on slab planes (0/0 = NaN) and flat boxes."""
    g = golden("kat_aabb.npz")
    rec, hit = g["rec"], g["hit"]
    L = oracle.lib()
    for i in range(len(rec)):
        r = rec[i]
        got = L.or_ray_aabb(oracle.OVec3(*r[0:3]), oracle.OVec3(*r[3:6]), oracle.OVec3(*r[6:9]), oracle.OVec3(*r[9:12]))
        assert got == int(hit[i]), i


def test_camera_matches_reference():
    g = golden("kat_cam.npz")
    L = oracle.lib()
    for ci in range(4):
        c = g["cam%d" % ci]
        cam = oracle.camera(tuple(c[:3]), c[3], c[4], c[5], int(c[6]), int(c[7]))
        for k in range(0, len(g["idx%d" % ci]), 5):
            o, d = oracle.OVec3(), oracle.OVec3()
            u1, u2 = (float("nan"), 0.0) if c[5] == 0 else (float(g["u%d" % ci][k][0]), float(g["u%d" % ci][k][1]))
            L.or_camera_ray(C.byref(cam), int(g["idx%d" % ci][k]), u1, u2, C.byref(o), C.byref(d))
            got = np.array([o.x, o.y, o.z, d.x, d.y, d.z], dtype=np.float32)
            ref = g["ray%d" % ci][k]
            if c[5] == 0:
                assert got.tobytes() == ref.tobytes()
            else:
                assert np.all(np.abs(got.view(np.int32).astype(np.int64) - ref.view(np.int32)) <= 2)


def _rocrand_tables(name):
    txt = open(ROCRAND_PRE).read()
    i = txt.index("static const unsigned int %s" % name)
    j = txt.index("};", i)
    nums = re.findall(r"(\d+)U?", txt[txt.index("=", i): j])
    return np.array([int(x) for x in nums], dtype=np.uint64).astype(np.uint32).reshape(32, 800)


@pytest.mark.skipif(not os.path.exists(ROCRAND_PRE), reason="rocRAND headers absent")
def test_xorwow_jump_matrices_match_rocrand():
    """rocRAND's h_xorwow_jump_matrices[0] is the one-step matrix A and
    h_xorwow_sequence_jump_matrices[k] = A^(4^k * 2^67): the recurrence and the subsequence
    spacing curand_init uses (kernel.cu:532) are pinned by a published table."""
    seq = _rocrand_tables("h_xorwow_sequence_jump_matrices")
    step = _rocrand_tables("h_xorwow_jump_matrices")
    assert np.array_equal(oracle.jump_images(0), step[0])
    assert np.array_equal(oracle.jump_images(2), step[1])
    assert np.array_equal(oracle.jump_images(67), seq[0])
    assert np.array_equal(oracle.jump_images(69), seq[1])


def test_xorwow_streams_regression():
    g = golden("xorwow.npz")
    for s in g["subs"]:
        s = int(s)
        assert np.array_equal(oracle.xorwow_stream(1234, s, 64), g["raw_%d" % s])
        u = oracle.uniform_stream(1234, s, 64)
        assert np.array_equal(u.view(np.uint32), g["uni_%d" % s].view(np.uint32))
        assert (u > 0).all() and (u <= 1).all()


def test_sincos_is_correctly_rounded_nearly_always():
    """The deterministic sin/cos (shared spec with the kernels) vs numpy's double sin/cos rounded
    to float: at most 1 ulp apart, equal almost everywhere on the sampling range (0, 2*pi]."""
    L = oracle.lib()
    rng = np.random.default_rng(3)
    th = np.concatenate([rng.uniform(0, 6.28318, 20000), [6.28318, 1e-7, np.pi / 2, np.pi, 4.712389]]).astype(np.float32)
    diff = 0
    for x in th:
        s, c = C.c_float(), C.c_float()
        L.or_sincos(float(x), C.byref(s), C.byref(c))
        es, ec = np.float32(np.sin(np.float64(x))), np.float32(np.cos(np.float64(x)))
        for got, exp in ((s.value, es), (c.value, ec)):
            gi = np.float32(got).view(np.int32)
            ei = np.float32(exp).view(np.int32)
            assert abs(int(gi) - int(ei)) <= 1
            diff += int(gi != ei)
    assert diff <= len(th) * 2 // 1000


@pytest.mark.parametrize("fname,name,w,h,spp,b,i", [
    ("render_cornell_blob_32x32_s4_b3_i0.npz", "cornell_blob", 32, 32, 4, 3, 0),
    ("render_cornell_blob_32x32_s4_b3_i1.npz", "cornell_blob", 32, 32, 4, 3, 1),
    ("render_cornell_24x16_s3_b8_i0.npz", "cornell", 24, 16, 3, 8, 0)])
def test_oracle_render_regression(fname, name, w, h, spp, b, i):
    g = golden(fname)
    s = load_scene(name)
    osc = oracle.OracleScene(s.arrays())
    cam = oracle.camera((0.0, 1.0, 3.0), 1.0, 3.0, 0.0, w, h)
    img, cnt = oracle.render(osc, cam, w, h, spp, b, i, 1234)
    assert img.tobytes() == g["img"].tobytes()
    assert cnt["traces"] == int(g["traces"])


@pytest.mark.parametrize("name", ["cornell", "cornell_blob", "quirks", "standin"])
def test_oracle_trace_matches_reference_trace(name, request):
    """or_trace == the reference's own trace() (refgen trace, kernel.cu:107-161 compiled from
    /root/reference) on the committed ray sets: (triIndex, closestT) bit for bit and the test[]
    increments (kernel.cu:133) per triangle."""
    g = golden("kat_trace_%s.npz" % name)
    s = request.getfixturevalue("standin_scene") if name == "standin" else load_scene(name)
    osc = oracle.OracleScene(s.arrays())
    assert len(g["counts"]) == len(osc.tris)
    counts = np.zeros(len(osc.tris), dtype=np.uint32)
    tri, t = oracle.trace_batch(osc, g["rays"][:, :3], g["rays"][:, 3:], tri_counts=counts)
    assert np.array_equal(tri, g["tri"])
    assert np.array_equal(t.view(np.uint32), g["t"].view(np.uint32))
    assert np.array_equal(counts, g["counts"])
    names = [str(x) for x in g["set_names"]]
    assert {"axis", "tiny", "outside", "vertex_planes", "bounce"} <= set(names)


def test_trace_equals_bruteforce_restatement():
    """trace() (kernel.cu:112-161) == min over the triangles whose every ancestor box passes the
    slab test of (t, left-first DFS rank), 0 < t < MAX_FLOAT -- a brute-force statement of what
    the reference's stack walk selects."""
    s = load_scene("cornell_blob")
    a = s.arrays()
    osc = oracle.OracleScene(a)
    bvh = a["bvh"]
    L = oracle.lib()
    parent, leaf_parent = {}, {}
    for i, nd in enumerate(bvh):
        for ch in (int(nd["left"]), int(nd["right"])):
            if ch & 0x80000000:
                leaf_parent[ch ^ 0x80000000] = i
            else:
                parent[ch] = i
    rank, st = {}, [0]
    while st:
        e = st.pop()
        if e & 0x80000000:
            rank[e ^ 0x80000000] = len(rank)
        else:
            st += [int(bvh[e]["right"]), int(bvh[e]["left"])]
    verts = a["verts"]
    rng = np.random.default_rng(11)
    for _ in range(300):
        o = rng.uniform([-0.9, 0.1, -0.9], [0.9, 1.9, 2.5]).astype(np.float32)
        d = rng.normal(size=3)
        d = (d / np.linalg.norm(d)).astype(np.float32)
        O, D = oracle.OVec3(*o), oracle.OVec3(*d)
        passes = {}

        def ok(n):
            if n not in passes:
                nd = bvh[n]
                passes[n] = bool(L.or_ray_aabb(O, D, oracle.OVec3(*nd["lo"]), oracle.OVec3(*nd["hi"])))
            return passes[n]

        best = (np.float32(1e5), -1, -1)
        for k in range(len(a["tris"])):
            n = leaf_parent[k]
            good = True
            while True:
                if not ok(n):
                    good = False
                    break
                if n == 0:
                    break
                n = parent[n]
            if not good:
                continue
            t = np.float32(L.or_tri_intersect(O, D, verts.ctypes.data, a["tris"][k:k + 1].ctypes.data))
            if 0 < t and (t < best[0] or (t == best[0] and best[1] >= 0 and rank[k] < best[1])):
                best = (t, rank[k], k)
        tri, t = oracle.trace(osc, o, d)
        assert tri == best[2]
        assert np.float32(t).tobytes() == np.float32(best[0]).tobytes()


def test_sampling_frame_and_brdf_match_reference():
    """getTangent (kernel.cu:44-54: the larger of n x z and n x y, strict '>' so ties take n x y) and BRDF
    (:101-104: albedo * (1/3.14159) in double), compiled from the reference's own lines (refgen helpers,
    extracted verbatim at build time): the restatement equals them bit for bit on random, axis-aligned,
    tied and mesh normals and on random and material albedos.  (The rest of kernel.cu's sampling code --
    randRay, cosineWeightedRay -- draws through cuRAND and is not built here)"""
    g = golden("kat_helpers.npz")
    tan, brdf = oracle.helpers(g["normal"], g["albedo"])
    assert np.array_equal(tan.view(np.uint32), g["tangent"].astype(np.float32).view(np.uint32))
    assert np.array_equal(brdf.view(np.uint64), g["brdf"].view(np.uint64))
