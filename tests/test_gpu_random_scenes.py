"""Randomised triangle soups, GPU against the oracle, bit-exact (kernel.cu:112-161 trace, :417-515 /
:217-415 integrators).

The fixed fixtures (Cornell, blob, quirks, the stand-in) are well-formed meshes.  These soups are
not: triangles at random orientations and sizes, exact duplicates under another material (equal
distances: the reference's first-visited triangle must win, DESIGN.md "Traversal"), fans sharing
edges and a vertex (rays through shared edges), axis-aligned triangles (zero-thickness boxes),
zero-area triangles, and one emissive quad.  The render path's SAH BVH4 walk and winner check
must return the reference walk's (triangle, t) for every ray, and the renders must match bit for bit.
"""
import os

import numpy as np
import pytest

import cudapathtracer_amd as pt

pytestmark = pytest.mark.gpu

CAM = dict(pos=(0.0, 1.0, 3.0), dist_from_film=1.0, focal_length=3.0, radius=0.0)


def write_soup(dirpath, seed):
    rng = np.random.default_rng(seed)
    verts, faces, mats = [], [], []

    def tri(a, b, c, m):
        base = len(verts)
        verts.extend([a, b, c])
        faces.append((base + 1, base + 2, base + 3))
        mats.append(m)

    for _ in range(220):                                   # random triangles in [-2, 2]^3
        c = rng.uniform(-2, 2, 3)
        s = rng.choice([0.05, 0.3, 1.0])
        tri(c + rng.normal(0, s, 3), c + rng.normal(0, s, 3), c + rng.normal(0, s, 3), "m%d" % rng.integers(3))
    dup = list(range(0, 60, 3))                            # exact duplicates under another material
    for k in dup:
        a, b, c = (verts[3 * k + j] for j in range(3))
        tri(a, b, c, "m%d" % ((int(mats[k][1]) + 1) % 3))
    for f in range(4):                                     # fans: 8 triangles around a shared vertex
        ctr = rng.uniform(-1.5, 1.5, 3)
        ang = np.sort(rng.uniform(0, 2 * np.pi, 9))
        ring = [ctr + 0.6 * np.array([np.cos(t), np.sin(t), 0.2 * np.sin(3 * t)]) for t in ang]
        for j in range(8):
            tri(ctr, ring[j], ring[j + 1], "m%d" % (j % 3))
    for ax in range(3):                                    # axis-aligned quads (flat boxes)
        for _ in range(4):
            o = rng.uniform(-2, 2, 3)
            e1, e2 = np.zeros(3), np.zeros(3)
            e1[(ax + 1) % 3] = rng.uniform(0.2, 1.0)
            e2[(ax + 2) % 3] = rng.uniform(0.2, 1.0)
            tri(o, o + e1, o + e1 + e2, "m0")
            tri(o, o + e1 + e2, o + e2, "m1")
    for _ in range(6):                                     # zero-area triangles
        p = rng.uniform(-2, 2, 3)
        q = rng.uniform(-2, 2, 3)
        tri(p, q, p + 0.5 * (q - p), "m2")
        tri(p, p, q, "m1")
    # the light: a quad facing -y above the soup (kernel.cu:503 assumes (0, -1, 0))
    tri(np.array([-1.0, 2.6, -1.0]), np.array([-1.0, 2.6, 1.0]), np.array([1.0, 2.6, 1.0]), "light")
    tri(np.array([-1.0, 2.6, -1.0]), np.array([1.0, 2.6, 1.0]), np.array([1.0, 2.6, -1.0]), "light")
    obj = ["mtllib soup.mtl"]
    obj += ["v %.9g %.9g %.9g" % tuple(float(x) for x in v) for v in verts]
    cur = None
    for f, m in zip(faces, mats):
        if m != cur:
            obj.append("usemtl " + m)
            cur = m
        obj.append("f %d %d %d" % f)
    mtl = []
    for k, kd in enumerate(rng.uniform(0.2, 0.9, (3, 3))):
        mtl += ["newmtl m%d" % k, "Kd %.6g %.6g %.6g" % tuple(kd)]
    mtl += ["newmtl light", "Kd 0.8 0.8 0.8", "Ke 12 11 10"]
    os.makedirs(dirpath, exist_ok=True)
    with open(os.path.join(dirpath, "soup.mtl"), "w") as fh:
        fh.write("\n".join(mtl) + "\n")
    p = os.path.join(dirpath, "soup.obj")
    with open(p, "w") as fh:
        fh.write("\n".join(obj) + "\n")
    return p


@pytest.fixture(scope="module", params=[11, 12, 13, 14, 15, 16])
def soup(request, tmp_path_factory):
    d = tmp_path_factory.mktemp("soup%d" % request.param)
    p = write_soup(str(d), request.param)
    s = pt.Scene()
    s.load_obj(p, mtl_basepath=str(d) + "/")
    s.build_bvh()
    r = pt.Renderer(s, 0)
    yield request.param, s, r
    r.close()


def test_trace_matches_the_reference_walk(soup):
    import oracle
    seed, s, r = soup
    rng = np.random.default_rng(100 + seed)
    n = 20000
    o = rng.uniform(-2.5, 2.5, (n, 3)).astype(np.float32)
    d = rng.normal(0, 1, (n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(np.float32)
    # a quarter of the rays aimed at vertices (shared edges, fan centres, duplicate triangles' corners)
    v = s.arrays()["verts"]
    vv = np.stack([v["x"], v["y"], v["z"]], axis=1).astype(np.float64)
    tgt = vv[rng.integers(len(vv), size=n // 4)]
    dd = tgt - o[: n // 4]
    d[: n // 4] = (dd / np.maximum(np.linalg.norm(dd, axis=1, keepdims=True), 1e-30)).astype(np.float32)
    # a tenth with one or two zero direction components (0/0 slab values; the zero-direction ancestor check)
    z = slice(n // 4, n // 4 + n // 10)
    k1 = rng.integers(3, size=n // 10)
    dz = d[z].copy()
    dz[np.arange(n // 10), k1] = 0.0
    two = rng.random(n // 10) < 0.3
    dz[two, (k1[two] + 1) % 3] = 0.0
    dz /= np.maximum(np.linalg.norm(dz, axis=1, keepdims=True), 1e-30)
    dz[np.linalg.norm(dz, axis=1) == 0] = (0.0, -1.0, 0.0)
    d[z] = dz.astype(np.float32)
    osc = oracle.OracleScene(s.arrays())
    rt, rtt = oracle.trace_batch(osc, o, d)
    for ref_bvh in (False, True):
        gt, gtt = r.trace(o, d, reference_bvh=ref_bvh)
        assert np.array_equal(gt, rt), (ref_bvh, int(np.count_nonzero(gt != rt)))
        assert np.array_equal(gtt.view(np.uint32), rtt.view(np.uint32)), ref_bvh
    assert np.count_nonzero(rt >= 0) > n // 10   # the soup is hit


@pytest.mark.parametrize("flags", [0, pt.PT_FLAG_REFERENCE_TRAVERSAL, pt.PT_FLAG_REFERENCE_BVH])
@pytest.mark.parametrize("integ", [0, 1])
def test_render_matches_the_oracle(soup, integ, flags):
    """The wavefront kernel (flags 0), the tile kernel in the reference's traversal order and the
    reference-BVH walk, each against the oracle; the default path also as three tile shards summed."""
    import oracle
    seed, s, r = soup
    w, h, spp = 32, 24, 4
    cam = pt.make_camera(width=w, height=h, **CAM)
    img, st = r.render(cam, w, h, spp, bounces=3, integrator=integ, flags=flags)
    osc = oracle.OracleScene(s.arrays())
    ocam = oracle.camera(CAM["pos"], CAM["dist_from_film"], CAM["focal_length"], CAM["radius"], w, h)
    ref, cnt = oracle.render(osc, ocam, w, h, spp, 3, integ, 1234)
    ref32 = ref.astype(np.float32).view(np.uint32)
    diff = int(np.count_nonzero(img.view(np.uint32) != ref32))
    assert diff == 0, diff
    assert st["rays_reference"] == cnt["traces"]
    assert np.count_nonzero(img) > 0
    if flags == 0:
        acc = np.zeros_like(img)
        for k in range(3):
            part, _ = r.render(cam, w, h, spp, bounces=3, integrator=integ, shard_index=k, shard_count=3)
            acc += part
        assert int(np.count_nonzero(acc.view(np.uint32) != ref32)) == 0
