"""Ray-level parity: pt_trace (the reference's trace(), kernel.cu:112-161, batched) vs the CPU
oracle's or_trace, bit-exact in (winning triangle, closestT), on both walks the library has:
the render path's (BVH4 over the private SAH BVH + winner check + exact slow path) and the
reference's own stack walk.  Ray sets cover what the integrator produces (camera rays, rays
leaving surfaces at t - 0.001) plus the edge cases of the slab test (axis-parallel rays, zero
direction components, origins on box planes and vertices, tiny components that leave the
Markstein range, rays from outside the scene)."""
import os

import numpy as np
import pytest

from conftest import load_scene

import cudapathtracer_amd as pt
from cudapathtracer_amd import scenes

pytestmark = pytest.mark.gpu


def _unit(v):
    return (v / np.linalg.norm(v, axis=1)[:, None]).astype(np.float32)


def ray_sets(arrays, n, seed):
    """Dict of named (origins, directions) float32 arrays over the scene's bounds."""
    rng = np.random.default_rng(seed)
    v = arrays["verts"]
    P = np.stack([v["x"], v["y"], v["z"]], axis=1).astype(np.float64)
    lo, hi = P.min(0), P.max(0)
    ext = hi - lo
    out = {}
    o = rng.uniform(lo + 0.05 * ext, hi - 0.05 * ext, (n, 3))
    out["interior"] = (o.astype(np.float32), _unit(rng.normal(size=(n, 3))))
    d = rng.normal(size=(n, 3))
    axis = rng.integers(0, 3, n)
    zero = rng.integers(0, 3, n)
    d[np.arange(n), zero] = 0.0                     # one zero component
    d[: n // 3] = 0.0
    d[np.arange(n // 3), axis[: n // 3]] = rng.choice([-1.0, 1.0], n // 3)   # axis-parallel
    out["axis"] = (o.astype(np.float32), _unit(d))
    # origins on vertices and on their coordinate planes
    pick = P[rng.integers(0, len(P), n)]
    o2 = pick.copy()
    o2[n // 2:, 0] = rng.uniform(lo[0], hi[0], n - n // 2)
    out["vertex_planes"] = (o2.astype(np.float32), _unit(rng.normal(size=(n, 3))))
    # tiny components: outside the Markstein preconditions (exact slow path)
    d3 = rng.normal(size=(n, 3))
    d3[:, 1] = rng.choice([1e-31, -1e-36, 3e-39, 1e-20], n)
    out["tiny"] = (o.astype(np.float32), _unit(d3))
    # from outside: aimed at the scene
    c = 0.5 * (lo + hi)
    far = c + _unit(rng.normal(size=(n, 3))) * (2.0 * np.linalg.norm(ext) + 1.0)
    tgt = rng.uniform(lo, hi, (n, 3))
    out["outside"] = (far.astype(np.float32), _unit(tgt - far))
    return out


def bounce_rays(arrays, o, d, tri, t, seed):
    """Rays leaving the surfaces hit by (o, d) the way the integrator builds them
    (kernel.cu:455-470: pos = o + d * (float)(t - 0.001))."""
    rng = np.random.default_rng(seed)
    hit = tri >= 0
    tt = (t[hit].astype(np.float64) - 0.001).astype(np.float32)
    pos = (o[hit] + d[hit] * tt[:, None]).astype(np.float32)
    return pos, _unit(rng.normal(size=(len(pos), 3)))


def _check(r, osc, oracle_mod, o, d, name):
    etri, et = oracle_mod.trace_batch(osc, o, d)
    for ref in (False, True):
        tri, t = r.trace(o, d, reference_bvh=ref)
        bad = np.nonzero((tri != etri) | (t.view(np.uint32) != et.view(np.uint32)))[0]
        assert len(bad) == 0, (name, ref, len(bad), bad[:5].tolist(), tri[bad[:3]].tolist(), etri[bad[:3]].tolist(),
                               t[bad[:3]].tolist(), et[bad[:3]].tolist())
    return etri, et


@pytest.mark.parametrize("name", ["cornell", "cornell_blob"])
def test_trace_bit_exact_small_scenes(name):
    import oracle as oracle_mod
    s = load_scene(name)
    a = s.arrays()
    osc = oracle_mod.OracleScene(a)
    with pt.Renderer(s, 0) as r:
        for k, (o, d) in ray_sets(a, 20000, 5).items():
            etri, et = _check(r, osc, oracle_mod, o, d, k)
            if k == "interior":
                bo, bd = bounce_rays(a, o, d, etri, et, 6)
                _check(r, osc, oracle_mod, bo, bd, "bounce")


def test_trace_bit_exact_standin(tmp_path):
    """The 262K-triangle stand-in: camera rays of the bench view and their first bounces."""
    import oracle as oracle_mod
    p = scenes.write_sponza_standin(str(tmp_path))
    s = pt.Scene()
    s.load_obj(p, mtl_basepath=os.path.dirname(p) + "/")
    s.build_bvh()
    a = s.arrays()
    osc = oracle_mod.OracleScene(a)
    cam = pt.make_camera(scenes.SPONZA_STANDIN_CAMERA["pos"], scenes.SPONZA_STANDIN_CAMERA["dist_from_film"],
                         scenes.SPONZA_STANDIN_CAMERA["focal_length"], 0.0, 1920, 1080)
    idx = np.random.default_rng(9).integers(0, 1920 * 1080, 20000)
    rays = [pt.camera_ray(cam, int(i), lens=False) for i in idx]
    o = np.array([r[0] for r in rays], dtype=np.float32)
    d = np.array([r[1] for r in rays], dtype=np.float32)
    with pt.Renderer(s, 0) as r:
        etri, et = _check(r, osc, oracle_mod, o, d, "camera")
        bo, bd = bounce_rays(a, o, d, etri, et, 10)
        _check(r, osc, oracle_mod, bo, bd, "bounce")
        for k, (o2, d2) in ray_sets(a, 5000, 11).items():
            _check(r, osc, oracle_mod, o2, d2, k)
