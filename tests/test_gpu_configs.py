"""SURVEY 8 configs at their full sizes on one MI355X.  The whole image is rendered on the GPU;
the oracle (CPU, test infrastructure) recomputes a spread subset of pixels at full spp and
depth, which must match bit-for-bit; the rest is checked through properties (finite,
non-negative, sample counts, shard disjointness).

C2  Cornell mesh 1024x1024, 64 spp, depth 8
C3  262K-triangle stand-in 1920x1080, 256 spp, depth 3 (the bench workload)
C4  same at 1024 spp: all 8 shards of the 8-GPU partition rendered in turn and summed ==
    the full frame (sample-chunk work units at scale)
C5  stand-in 3840x2160, 4096 spp, depth 16
"""
import os

import numpy as np
import pytest

from conftest import load_scene

import cudapathtracer_amd as pt
from cudapathtracer_amd import scenes, shard

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def standin(tmp_path_factory):
    d = tmp_path_factory.mktemp("standin")
    p = scenes.write_sponza_standin(str(d))
    s = pt.Scene()
    s.load_obj(p, mtl_basepath=os.path.dirname(p) + "/")
    s.build_bvh()
    r = pt.Renderer(s, 0)
    yield s, r
    r.close()


def _check(scene, img, cam_kw, w, h, spp, bounces, pixels):
    import oracle
    osc = oracle.OracleScene(scene.arrays())
    ocam = oracle.camera(cam_kw["pos"], cam_kw["dist_from_film"], cam_kw["focal_length"], cam_kw["radius"], w, h)
    ref, _ = oracle.render(osc, ocam, w, h, spp, bounces, 0, 1234, pixels=pixels)
    a = img.reshape(-1, 3)[pixels]
    b = ref.reshape(-1, 3)[pixels].astype(np.float32)
    bad = np.nonzero(np.any(a.view(np.uint32) != b.view(np.uint32), axis=1))[0]
    assert len(bad) == 0, (len(bad), [int(pixels[i]) for i in bad[:5]])


def _spread(w, h, n, seed):
    rng = np.random.default_rng(seed)
    pix = rng.choice(w * h, size=n, replace=False).astype(np.uint32)
    return np.unique(np.concatenate([pix, [0, w * h - 1]]).astype(np.uint32))


def test_c2_cornell_1024_64spp_depth8():
    s = load_scene("cornell")
    w = h = 1024
    cam_kw = scenes.CORNELL_CAMERA
    with pt.Renderer(s, 0) as r:
        img, st = r.render(pt.make_camera(width=w, height=h, **cam_kw), w, h, 64, bounces=8)
    assert np.isfinite(img).all() and (img >= 0).all()
    assert st["samples"] == w * h * 64
    _check(s, img, cam_kw, w, h, 64, 8, _spread(w, h, 4096, 1))


def test_c3_standin_1080p_256spp(standin):
    s, r = standin
    w, h = 1920, 1080
    cam_kw = scenes.SPONZA_STANDIN_CAMERA
    img, st = r.render(pt.make_camera(width=w, height=h, **cam_kw), w, h, 256, bounces=3)
    assert np.isfinite(img).all() and (img >= 0).all()
    assert st["samples"] == w * h * 256
    _check(s, img, cam_kw, w, h, 256, 3, _spread(w, h, 4096, 2))


def test_c4_standin_1080p_1024spp_eight_shards_sum_to_full_frame(standin):
    """C4 as the 8-GPU job partitions it, on one GPU: all 8 image-tile shards rendered in turn
    (each with its split-pixel work units), disjoint, summed (what the RCCL reduce computes) --
    bit-identical to the full-frame render, whose spread of pixels equals the oracle."""
    s, r = standin
    w, h, spp = 1920, 1080, 1024
    cam_kw = scenes.SPONZA_STANDIN_CAMERA
    cam = pt.make_camera(width=w, height=h, **cam_kw)
    full, st = r.render(cam, w, h, spp, bounces=3)
    assert st["samples"] == w * h * spp
    acc = np.zeros_like(full)
    seen = np.zeros(w * h, dtype=np.int32)
    samples = 0
    for k in range(8):
        part, sk = r.render(cam, w, h, spp, bounces=3, shard_index=k, shard_count=8)
        mine = shard.shard_pixels(w, h, k, 8)
        mask = np.zeros(w * h, dtype=bool)
        mask[mine] = True
        assert np.all(part.reshape(-1, 3)[~mask] == 0)
        seen[mine] += 1
        samples += sk["samples"]
        acc += part
    assert np.all(seen == 1) and samples == w * h * spp
    assert np.array_equal(acc.view(np.uint32), full.view(np.uint32))
    _check(s, full, cam_kw, w, h, spp, 3, _spread(w, h, 2048, 3))


@pytest.mark.parametrize("nshards", [2, 4])
def test_c3_standin_shards_sum_to_full_frame(standin, nshards):
    """C3 as the 2- and 4-GPU jobs partition it: the half shard splits a tail of its pixels, the quarter
    shard (1.58 pixels per lane) renders whole pixels for half its lanes and splits the rest into three
    grades (round 5) -- summed, bit-identical to the full frame."""
    s, r = standin
    w, h, spp = 1920, 1080, 256
    cam = pt.make_camera(width=w, height=h, **scenes.SPONZA_STANDIN_CAMERA)
    full, st = r.render(cam, w, h, spp, bounces=3)
    acc = np.zeros_like(full)
    samples = 0
    for k in range(nshards):
        part, sk = r.render(cam, w, h, spp, bounces=3, shard_index=k, shard_count=nshards)
        mask = np.zeros(w * h, dtype=bool)
        mask[shard.shard_pixels(w, h, k, nshards)] = True
        assert np.all(part.reshape(-1, 3)[~mask] == 0)
        samples += sk["samples"]
        acc += part
    assert samples == w * h * spp
    assert np.array_equal(acc.view(np.uint32), full.view(np.uint32))


def test_c3_fast_walk_equals_reference_walk_full_frame(standin):
    """Every pixel of C3: the measured wavefront kernel (BVH4 walk, culling, winner check, memo,
    dead-path skip, split units) equals the tile kernel walking the reference BVH in the
    reference's own node order (PT_FLAG_REFERENCE_TRAVERSAL), bit for bit."""
    s, r = standin
    w, h, spp = 1920, 1080, 256
    cam = pt.make_camera(width=w, height=h, **scenes.SPONZA_STANDIN_CAMERA)
    a, sa = r.render(cam, w, h, spp, bounces=3)
    b, sb = r.render(cam, w, h, spp, bounces=3, flags=pt.PT_FLAG_REFERENCE_TRAVERSAL)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert sa["rays_reference"] == sb["rays_reference"] and sa["samples"] == sb["samples"]


def test_c5_standin_4k_4096spp_depth16(standin):
    s, r = standin
    w, h = 3840, 2160
    cam_kw = scenes.SPONZA_STANDIN_CAMERA
    img, st = r.render(pt.make_camera(width=w, height=h, **cam_kw), w, h, 4096, bounces=16)
    assert np.isfinite(img).all() and (img >= 0).all()
    assert st["samples"] == w * h * 4096
    _check(s, img, cam_kw, w, h, 4096, 16, _spread(w, h, 512, 4))


@pytest.mark.parametrize("top", ["0", "17", "64"])
def test_lds_top_nodes_bit_identical(standin, monkeypatch, top):
    """The BVH4 top staged in LDS (PT_WF_TOP nodes; default 101, at least 1: 0 stages the root
    alone) changes where node records are read from, never the result: images with 1, 17 and 64
    staged nodes equal the default's bit for bit, and a spread of pixels equals the oracle."""
    s, r = standin
    w, h, spp = 320, 180, 8
    cam_kw = scenes.SPONZA_STANDIN_CAMERA
    cam = pt.make_camera(width=w, height=h, **cam_kw)
    ref, _ = r.render(cam, w, h, spp, bounces=3)
    monkeypatch.setenv("PT_WF_TOP", top)
    with pt.Renderer(s, 0) as r2:
        img, st = r2.render(cam, w, h, spp, bounces=3)
    assert st["samples"] == w * h * spp
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
    if top == "0":
        _check(s, img, cam_kw, w, h, spp, 3, _spread(w, h, 32, 5))


@pytest.mark.parametrize("jump_bytes", ["1", "0"])
def test_wide_image_seeding_beyond_24_morton_bits(monkeypatch, jump_bytes):
    """curand_init of a pixel whose Morton index has bits >= 24 (x >= 4096): the byte-position jump
    tables cover bits 0..23, the rest are applied bit by bit (init_pixel_states); both seeding
    forms (PT_JUMP_BYTES) equal the oracle's curand_init bit for bit there and elsewhere."""
    monkeypatch.setenv("PT_JUMP_BYTES", jump_bytes)
    s = load_scene("cornell")
    w, h, spp = 4104, 2, 2
    cam_kw = scenes.CORNELL_CAMERA
    with pt.Renderer(s, 0) as r:
        img, st = r.render(pt.make_camera(width=w, height=h, **cam_kw), w, h, spp, bounces=3)
    assert st["samples"] == w * h * spp
    pix = np.array([0, 1, 255, 256, 4095, 4096, 4097, 4103, w + 4096, w + 4103, w * h - 1], dtype=np.uint32)
    _check(s, img, cam_kw, w, h, spp, 3, pix)


@pytest.mark.parametrize("mode", ["wavefront", "tile4", "tileref"])
def test_head_integrator_walks_bit_identical(standin, monkeypatch, mode):
    """Integrator 1 (radianceAlongSingleStep, kernel.cu:217-415) on the 262K stand-in: the wavefront
    state machine (default: T1 light bounce, T2 camera memo, T3 camera bounce, bounded visibility walks),
    the tile kernel on the render-path BVH4 walk (PT_HEAD_WF=0) and on the reference-BVH culled walk
    (PT_HEAD_WF=0 PT_TILE_FAST4=0) render the same bits as the reference-order walk, and a spread of
    pixels equals the oracle."""
    s, r = standin
    w, h, spp = 160, 96, 4
    cam_kw = scenes.SPONZA_STANDIN_CAMERA
    cam = pt.make_camera(width=w, height=h, **cam_kw)
    ref, sref = r.render(cam, w, h, spp, bounces=3, integrator=1, flags=pt.PT_FLAG_REFERENCE_TRAVERSAL)
    if mode != "wavefront":
        monkeypatch.setenv("PT_HEAD_WF", "0")
        monkeypatch.setenv("PT_TILE_FAST4", "1" if mode == "tile4" else "0")
    with pt.Renderer(s, 0) as r2:
        img, st = r2.render(cam, w, h, spp, bounces=3, integrator=1)
    assert st["samples"] == w * h * spp
    assert st["rays_reference"] == sref["rays_reference"]
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
    if mode == "wavefront":
        assert st["work_units"] > 0   # (the wavefront kernel ran)
        import oracle
        osc = oracle.OracleScene(s.arrays())
        ocam = oracle.camera(cam_kw["pos"], cam_kw["dist_from_film"], cam_kw["focal_length"], cam_kw["radius"], w, h)
        pix = _spread(w, h, 24, 6)
        o, cnt = oracle.render(osc, ocam, w, h, spp, 3, 1, 1234, pixels=pix)
        a = img.reshape(-1, 3)[pix]
        b = o.reshape(-1, 3)[pix].astype(np.float32)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_c3_head_integrator_full_frame(standin, monkeypatch):
    """C3 (1920x1080, 256 spp) with integrator 1: the wavefront kernel (the measured path, with its
    split units and bounded visibility walks) equals the tile kernel on every pixel, and a spread of
    pixels equals the oracle."""
    s, r = standin
    w, h, spp = 1920, 1080, 256
    cam_kw = scenes.SPONZA_STANDIN_CAMERA
    cam = pt.make_camera(width=w, height=h, **cam_kw)
    a, sa = r.render(cam, w, h, spp, bounces=3, integrator=1)
    assert sa["work_units"] > w * h   # (split units in the tail)
    monkeypatch.setenv("PT_HEAD_WF", "0")
    with pt.Renderer(s, 0) as r2:
        b, sb = r2.render(cam, w, h, spp, bounces=3, integrator=1)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert sa["rays_reference"] == sb["rays_reference"] and sa["samples"] == sb["samples"] == w * h * spp
    import oracle
    osc = oracle.OracleScene(s.arrays())
    ocam = oracle.camera(cam_kw["pos"], cam_kw["dist_from_film"], cam_kw["focal_length"], cam_kw["radius"], w, h)
    pix = _spread(w, h, 256, 7)
    o, _ = oracle.render(osc, ocam, w, h, spp, 3, 1, 1234, pixels=pix)
    assert np.array_equal(a.reshape(-1, 3)[pix].view(np.uint32), o.reshape(-1, 3)[pix].astype(np.float32).view(np.uint32))


def test_merged_shading_records_bit_identical(standin, monkeypatch):
    """The wavefront bounce reads a triangle's normal and its material's colours from one merged
    48-B record (Args::shade_m, used when every material colour is a float); PT_NO_SHADE_M=1 reads
    the shading record and then the material (two dependent fetches): the same bits."""
    s, r = standin
    w, h, spp = 320, 180, 8
    cam = pt.make_camera(width=w, height=h, **scenes.SPONZA_STANDIN_CAMERA)
    a, _ = r.render(cam, w, h, spp, bounces=5)
    monkeypatch.setenv("PT_NO_SHADE_M", "1")
    with pt.Renderer(s, 0) as r2:
        b, _ = r2.render(cam, w, h, spp, bounces=5)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_c3_full_frame_repeatable(standin):
    """The full C3 frame is the same bits on every render, for both integrators: nothing the persistent
    kernel shares between lanes (unit counters, the published primary-hit words of split pixels, the
    LDS queues) may change a result, only which lane computes it.  (Round 3's full-precision 8-wide
    experiment once failed the integrator-1 full-frame comparison and did not on re-running the same
    build, profiles/r04_w8f: this checks the product for run-to-run differences directly.)"""
    s, r = standin
    w, h, spp = 1920, 1080, 256
    cam = pt.make_camera(width=w, height=h, **scenes.SPONZA_STANDIN_CAMERA)
    for integ in (0, 1):
        a, _ = r.render(cam, w, h, spp, bounces=3, integrator=integ)
        b, _ = r.render(cam, w, h, spp, bounces=3, integrator=integ)
        with pt.Renderer(s, 0) as r2:   # a fresh context: fresh buffers and seed tables
            c, _ = r2.render(cam, w, h, spp, bounces=3, integrator=integ)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), integ
        assert np.array_equal(a.view(np.uint32), c.view(np.uint32)), integ
