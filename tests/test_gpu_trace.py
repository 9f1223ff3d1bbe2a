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

from conftest import golden, load_scene
from raysets import bounce_rays, ray_sets

import cudapathtracer_amd as pt
from cudapathtracer_amd import scenes

pytestmark = pytest.mark.gpu


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


@pytest.mark.parametrize("name", ["cornell", "cornell_blob", "quirks", "standin"])
def test_trace_matches_reference_trace_goldens(name, request):
    """Both walks against the reference's OWN trace() (kernel.cu:107-161 compiled from
    /root/reference by oracle/Makefile; tests/golden/kat_trace_*.npz): (triIndex, closestT)
    bit for bit, and the reference walk's per-triangle test counts (kernel.cu:133) exactly."""
    g = golden("kat_trace_%s.npz" % name)
    s = request.getfixturevalue("standin_scene") if name == "standin" else load_scene(name)
    o, d = g["rays"][:, :3], g["rays"][:, 3:]
    with pt.Renderer(s, 0) as r:
        for ref in (False, True):
            tri, t = r.trace(o, d, reference_bvh=ref)
            bad = np.nonzero((tri != g["tri"]) | (t.view(np.uint32) != g["t"].view(np.uint32)))[0]
            assert len(bad) == 0, (name, ref, len(bad), bad[:5].tolist())
        tri, t, counts, _ = r.trace_counts(o, d, reference_bvh=True)
        assert np.array_equal(tri, g["tri"])
        assert np.array_equal(counts, g["counts"]), int(np.abs(counts.astype(np.int64) - g["counts"]).sum())
        # the render path's walk reports the tests it performed (on the large scene far fewer)
        _, _, fast_counts, _ = r.trace_counts(o, d)
        assert fast_counts.sum() > 0
        if name == "standin":
            assert fast_counts.sum() < counts.sum()


def test_lds_ring_spill_path_runs_and_is_exact(tmp_path):
    """The BVH4 walk's stack beyond the 16-entry LDS ring (HBM spill column; the reference's
    fixed stack[64] + depth guard, kernel.cu:114, :627-631): on the splinters scene every ray
    enters nearly every box, the walk spills (counted), and results stay bit-exact vs the
    oracle -- for batched trace() and for a rendered image."""
    import oracle as oracle_mod
    p = scenes.write_splinters(str(tmp_path))
    s = pt.Scene()
    s.load_obj(p, mtl_basepath=os.path.dirname(p) + "/")
    s.build_bvh()
    a = s.arrays()
    osc = oracle_mod.OracleScene(a)
    w = h = 24
    cam = pt.make_camera(width=w, height=h, **scenes.CORNELL_CAMERA)
    cr = [pt.camera_ray(cam, pt.morton_pxl_to_i(x, y)) for y in range(h) for x in range(w)]
    o = np.array([c[0] for c in cr], np.float32)
    d = np.array([c[1] for c in cr], np.float32)
    sets = ray_sets(a, 1000, 21)
    o = np.concatenate([o] + [v[0] for v in sets.values()])
    d = np.concatenate([d] + [v[1] for v in sets.values()])
    with pt.Renderer(s, 0) as r:
        tri, t, _, spills = r.trace_counts(o, d)
        assert spills > 0
        etri, et = oracle_mod.trace_batch(osc, o, d)
        assert np.array_equal(tri, etri) and np.array_equal(t.view(np.uint32), et.view(np.uint32))
        img, st = r.render(cam, w, h, 4, bounces=3, flags=pt.PT_FLAG_COUNT)
        assert st["spill_entries"] > 0
        img2, _ = r.render(cam, w, h, 4, bounces=3)
    ocam = oracle_mod.camera(scenes.CORNELL_CAMERA["pos"], 1.0, 3.0, 0.0, w, h)
    ref, _ = oracle_mod.render(osc, ocam, w, h, 4, 3, 0, 1234)
    assert np.array_equal(img.view(np.uint32), img2.view(np.uint32))
    assert np.array_equal(img.view(np.uint32), ref.astype(np.float32).view(np.uint32))


@pytest.mark.parametrize("w,h,spp", [(24, 24, 4), (160, 96, 8)])
def test_lds_ring_spill_path_integrator1_wavefront_vs_tile_vs_oracle(tmp_path, monkeypatch, w, h, spp):
    """Integrator 1 (radianceAlongSingleStep, kernel.cu:217-415) on the splinters scene, where walks
    spill past the 16-entry LDS stack ring into the lane's HBM spill column (the only
    spilling build of round 3 was the one whose integrator-1 full frame diverged).  The wavefront
    kernel (render_head_wf: bounded any-hit visibility walks, split units at these small sizes) must
    spill (counted), equal itself without the counting build, equal the tile kernel (PT_HEAD_WF=0)
    and the oracle, bit for bit."""
    import oracle as oracle_mod
    p = scenes.write_splinters(str(tmp_path))
    s = pt.Scene()
    s.load_obj(p, mtl_basepath=os.path.dirname(p) + "/")
    s.build_bvh()
    osc = oracle_mod.OracleScene(s.arrays())
    cam = pt.make_camera(width=w, height=h, **scenes.CORNELL_CAMERA)
    with pt.Renderer(s, 0) as r:
        a, sa = r.render(cam, w, h, spp, bounces=3, integrator=1, flags=pt.PT_FLAG_COUNT)
        assert sa["spill_entries"] > 0
        a2, sa2 = r.render(cam, w, h, spp, bounces=3, integrator=1)
    assert sa2["samples"] == w * h * spp
    monkeypatch.setenv("PT_HEAD_WF", "0")
    with pt.Renderer(s, 0) as r2:
        b, _ = r2.render(cam, w, h, spp, bounces=3, integrator=1)
    ocam = oracle_mod.camera(scenes.CORNELL_CAMERA["pos"], 1.0, 3.0, 0.0, w, h)
    ref, _ = oracle_mod.render(osc, ocam, w, h, spp, 3, 1, 1234)
    assert np.array_equal(a.view(np.uint32), a2.view(np.uint32))
    assert np.array_equal(a2.view(np.uint32), b.view(np.uint32))
    assert np.array_equal(a2.view(np.uint32), ref.astype(np.float32).view(np.uint32))
