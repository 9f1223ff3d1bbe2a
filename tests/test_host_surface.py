"""Host surface (C++ in libptamd.so) vs arrays produced by the REFERENCE's own loadOBJ/buildBVH/
camera/PPM code (compiled from /root/reference by oracle/refgen; fixtures in tests/golden).
Bar: byte-identical."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLD, MODELS, SCENE_SETS, golden, load_scene

import cudapathtracer_amd as pt
from cudapathtracer_amd import api


@pytest.mark.parametrize("name", sorted(SCENE_SETS))
def test_scene_arrays_match_reference(name):
    """verts/tris/mats/lights/totalLightArea (modelLoader.h:125-210) and the BVH node array
    (BVH.h:443-474) are byte-identical to the reference's."""
    g = golden("scene_%s.npz" % name)
    s = load_scene(name, build_bvh=False)
    if len(g["tris"]) >= 2:
        s.build_bvh()
    a = s.arrays()
    for k in ("verts", "tris", "mats", "lights", "bvh"):
        assert a[k].tobytes() == g[k].tobytes(), k
    assert np.float32(a["total_light_area"]).tobytes() == np.float32(g["total_light_area"]).tobytes()
    assert a["bvh_depth"] == int(g["bvh_depth"])


def test_standin_262k_matches_reference_hashes(tmp_path):
    """The ~262K-triangle stand-in: every array's sha256 equals the reference build's."""
    from cudapathtracer_amd import scenes
    ref = json.load(open(os.path.join(GOLD, "standin.json")))
    p = scenes.write_sponza_standin(str(tmp_path))
    assert hashlib.sha256(open(p, "rb").read()).hexdigest() == ref["obj_sha256"]
    s = pt.Scene()
    s.load_obj(p, mtl_basepath=os.path.dirname(p) + "/")
    s.build_bvh()
    a = s.arrays()
    for k in ("verts", "tris", "mats", "lights", "bvh"):
        assert hashlib.sha256(a[k].tobytes()).hexdigest() == ref[k], k
    assert a["bvh_depth"] == int(ref["meta"][7])
    assert len(a["tris"]) == int(ref["meta"][1]) == 262782


def test_quirks_semantics():
    """tinyobj 0.9.13 corners: fan triangulation, vt/vn-keyed vertex dedupe, unknown material
    (-1 -> matsOffset-1), unparseable '.5' -> 0, shape split at usemtl/g/o, first-face material."""
    s = load_scene("quirks", build_bvh=False)
    a = s.arrays()
    v = a["verts"]
    assert v[0]["x"] == 0 and v[2]["y"] == np.float32(1.0)
    # 'v .5 1 0.25': x fails to parse -> 0 ; '1.5E-1' parses
    xs = sorted(set(np.round(v["x"].astype(np.float64), 6)))
    assert 0.15 in [round(x, 6) for x in xs]
    # materials pushed twice: 3 from quirks.mtl (matA, matB, glow) -> 6
    assert len(a["mats"]) == 6
    # the 'glow' material (Ke 2.5 0 1) makes its triangles lights
    assert len(a["lights"]) >= 1
    assert s.warning == ""


def test_missing_mtl_stops_reading_like_tinyobj():
    """A missing .mtl makes tinyobj return at the mtllib line (tiny_obj_loader.cc:794-810):
    no triangles, one default material (pushed twice), and a warning, not an error."""
    s = load_scene("nomtl", build_bvh=False)
    a = s.arrays()
    assert len(a["tris"]) == 0 and len(a["mats"]) == 2
    assert "not found" in s.warning
    with pytest.raises(pt.PtError) as e:
        s.build_bvh()
    assert e.value.code == -3     # decision d5: fewer than 2 triangles


def test_load_errors():
    s = pt.Scene()
    with pytest.raises(pt.PtError) as e:
        s.load_obj(os.path.join(MODELS, "does_not_exist.obj"), mtl_basepath=MODELS + "/")
    assert e.value.code == -2
    bad = os.path.join(GOLD, "..", "bad_index.obj")
    try:
        with open(bad, "w") as fh:
            fh.write("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 9\n")
        with pytest.raises(pt.PtError):
            pt.Scene().load_obj(bad, mtl_basepath=MODELS + "/")
    finally:
        os.remove(bad)


def test_morton_matches_reference():
    g = golden("kat_morton.npz")
    xy = g["xy"]
    for i in list(range(0, 1 << 16, 257)) + [0, 1, 2, 3, 65535]:
        x, y = pt.morton_i_to_pxl(i)
        assert (x | (y << 16)) == int(xy[i])
        assert pt.morton_pxl_to_i(x, y) == int(g["back"][i])


def test_camera_ray_matches_reference():
    """cameraRay (camera.h:77-97).  Radius 0: exact bits with no lens draws (the reference's
    lens term is +0 for the KAT's draws).  Radius > 0: within 1 ulp (the lens angle goes
    through the deterministic kernel sin/cos instead of cosf/sinf)."""
    g = golden("kat_cam.npz")
    for ci in range(4):
        c = g["cam%d" % ci]
        cam = pt.make_camera(tuple(c[:3]), c[3], c[4], c[5], int(c[6]), int(c[7]))
        for k in range(0, len(g["idx%d" % ci]), 7):
            u1, u2 = g["u%d" % ci][k]
            o, d = pt.camera_ray(cam, int(g["idx%d" % ci][k]), lens=c[5] != 0, u1=u1, u2=u2)
            got = np.array(o + d, dtype=np.float32)
            ref = g["ray%d" % ci][k]
            if c[5] == 0:
                assert got.tobytes() == ref.tobytes(), (ci, k)
            else:
                assert np.all(np.abs(got.view(np.int32).astype(np.int64) - ref.view(np.int32)) <= 2), (ci, k)


def test_tonemap_and_ppm_match_reference(tmp_path):
    """kernel.cu:763-778: tone map (int)(gammaCorrect(normalized(c), 1/2.2)*255) and the PPM
    text layout (rows top-down, x mirrored, trailing-space separated)."""
    g = golden("kat_tone.npz")
    c, v = g["c"], g["v"]
    for i in range(len(c)):
        for ch in range(3):
            assert pt.tonemap_u8(float(c[i, ch])) == int(v[i, ch])
    w, h = 5, 3
    img = np.arange(w * h * 3, dtype=np.float64).reshape(h, w, 3) / 7.0
    p = str(tmp_path / "x.ppm")
    pt.write_ppm(p, img)
    txt = open(p).read()
    assert txt.startswith("P3 5 3 255\n")
    vals = [int(t) for t in txt.split("\n", 1)[1].split()]
    exp = []
    for y in range(h):
        for x in range(w - 1, -1, -1):
            exp += [pt.tonemap_u8(img[y, x, k]) for k in range(3)]
    assert vals == exp
    pt.write_ppm(str(tmp_path / "y.ppm"), img.astype(np.float32))
    assert os.path.getsize(str(tmp_path / "y.ppm")) > 0


def test_morton_framebuffer_ppm_matches_reference_loop(tmp_path):
    """The reference's framebuffer is Morton-indexed (drawPixel writes imgBuff[idx], kernel.cu:543,552)
    and its PPM loop reads imgBuffer_host[cam.mortonPxltoI(x,y)] (kernel.cu:771).  Fixture: that loop
    compiled verbatim from kernel.cu:763-778 (refgen ppm) over a 64x64 Morton buffer.  Byte-identical:
    pt_write_ppm_order(MORTON) on the buffer, pt_write_ppm on its scanline reordering, and the
    oracle's restatement of the loop."""
    import oracle
    from cudapathtracer_amd import shard
    g = golden("kat_ppm_morton.npz")
    buf, w, h, ref = g["buf"], int(g["w"]), int(g["h"]), g["ppm"].tobytes()
    pm, ps, po = str(tmp_path / "m.ppm"), str(tmp_path / "s.ppm"), str(tmp_path / "o.ppm")
    pt.write_ppm(pm, buf, pixel_order=pt.PT_ORDER_MORTON, width=w, height=h)
    pt.write_ppm(ps, shard.to_scanline(buf, w, h))
    oracle.write_ppm_imgbuf(po, buf, w, h)
    for p in (pm, ps, po):
        assert open(p, "rb").read() == ref, p
    if oracle.refgen_available():   # build container: the reference's loop, live
        assert oracle.ref_ppm_imgbuf(buf, w, h, str(tmp_path)) == ref
    # the reference's Morton buffer covers the image only for square power-of-two sizes
    for bw, bh in ((64, 32), (48, 48), (3, 3)):
        with pytest.raises(pt.PtError) as e:
            pt.write_ppm(str(tmp_path / "bad.ppm"), np.zeros((bw * bh, 3), np.float32), pixel_order=pt.PT_ORDER_MORTON,
                         width=bw, height=bh)
        assert e.value.code == pt.PT_E_INVALID
    # the buffer must hold width*height*3 values (the C loop reads rgb[morton(x,y)*3 ..]): checked before the call
    for bad_buf, bw, bh in ((buf[: w * h // 2], w, h), (buf, None, h), (buf, w, None), (buf, 2 * w, 2 * h)):
        with pytest.raises(ValueError):
            pt.write_ppm(str(tmp_path / "bad.ppm"), bad_buf, pixel_order=pt.PT_ORDER_MORTON, width=bw, height=bh)


def test_shard_tiles_partition_the_image():
    """Tile shards (tile t -> shard t % N, tile_w x tile_h tiles of 8x8 blocks) partition every image."""
    from cudapathtracer_amd import shard
    for w, h in ((64, 64), (100, 77), (1, 1), (8, 200)):
        for tw, th in ((0, 0), (16, 24), (32, 8), (256, 256)):
            for n in (1, 3, 8):
                allp = np.concatenate([shard.shard_pixels(w, h, k, n, tw, th) for k in range(n)])
                assert len(allp) == w * h and len(np.unique(allp)) == w * h
    with pytest.raises(ValueError):
        shard.tiles_shape(64, 64, 12, 8)


def test_structs_match_reference_layouts():
    assert api.VEC3.itemsize == 12 and api.TRI.itemsize == 28 and api.MAT.itemsize == 48 and api.NODE.itemsize == 32


def test_ppm_from_codes_and_pfm_roundtrip(tmp_path):
    """pt_write_ppm_codes(pt_tonemap_u8(img)) is byte-identical to pt_write_ppm(img); the PFM
    dump round-trips every float bit."""
    rng = np.random.default_rng(4)
    img = (rng.exponential(0.3, size=(7, 11, 3))).astype(np.float32)
    img[0, 0] = [0.0, np.float32(1e-30), np.float32(3e38)]
    a, b, c = (str(tmp_path / n) for n in ("a.ppm", "b.ppm", "c.pfm"))
    pt.write_ppm(a, img)
    codes = np.vectorize(pt.tonemap_u8)(img.astype(np.float64)).astype(np.int32)
    pt.write_ppm_codes(b, codes)
    assert open(a, "rb").read() == open(b, "rb").read()
    pt.write_pfm(c, img)
    back = pt.read_pfm(c)
    assert back.tobytes() == img.tobytes()


def _tone_thresholds():
    t = [0.0]
    for k in range(1, 256):
        lo, hi = 0, 0x7F7FFFFF
        while lo < hi:
            mid = (lo + hi) // 2
            if pt.tonemap_u8(float(np.uint32(mid).view(np.float32))) >= k:
                hi = mid
            else:
                lo = mid + 1
        t.append(float(np.uint32(lo).view(np.float32)))
    return np.array(t, dtype=np.float32)


def test_tonemap_threshold_table_reproduces_host_function():
    """The GPU output step's premise: for finite c >= 0 the code is the number of host-libm
    bisected thresholds <= c (monotone map).  Checked at every threshold, one float below it,
    and on 200K random floats across [0, 1e6]."""
    t = _tone_thresholds()
    assert np.all(np.diff(t) >= 0)
    below = (t[1:].view(np.uint32) - 1).view(np.float32)
    probe = np.concatenate([t, below, np.random.default_rng(5).uniform(0, 1, 100000).astype(np.float32),
                            np.exp(np.random.default_rng(6).uniform(-30, 14, 100000)).astype(np.float32)])
    got = np.searchsorted(t[1:], probe, side="right")
    ref = np.array([pt.tonemap_u8(float(c)) for c in probe])
    assert np.array_equal(got, ref)


def test_parallel_host_builds_are_deterministic(tmp_path, monkeypatch):
    """The reference BVH (BVH.h) and the render path's SAH/BVH4 structure are built on several
    host threads; both must equal the single-thread build exactly (the BVH.h array is also
    pinned by the reference hashes above)."""
    from cudapathtracer_amd import scenes
    p = scenes.write_sponza_standin(str(tmp_path))
    out = {}
    for threads in ("1", "3", "8"):
        monkeypatch.setenv("PT_HOST_THREADS", threads)
        s = pt.Scene()
        s.load_obj(p, mtl_basepath=os.path.dirname(p) + "/")
        s.build_bvh()
        out[threads] = (hashlib.sha256(s.arrays()["bvh"].tobytes()).hexdigest(), s.accel_digest())
    assert out["1"] == out["3"] == out["8"]
    assert out["1"][1][1] > 0 and out["1"][1][2] > 0


@pytest.mark.parametrize("name", sorted(SCENE_SETS))
def test_bvh4_collapse_is_a_valid_tree(name, monkeypatch):
    """The render path's 4-wide tree, from the SAH-optimal DP collapse (default) and from the old
    greedy one: pt_accel_digest validates it (every inner node and every binary leaf slot reached
    exactly once, at most 8 leaf triangles per node, child boxes nested in their parent's box) and
    fails with PT_E_SCENE otherwise.  The DP never needs more nodes than the greedy collapse."""
    s = load_scene(name, build_bvh=False)
    if s.view().num_tris < 2:
        pytest.skip("the render path needs >= 2 triangles")
    got = {}
    for mode in ("dp", "greedy"):
        monkeypatch.setenv("PT_COLLAPSE", mode)
        got[mode] = s.accel_digest()
    assert got["dp"][1] <= got["greedy"][1]


def test_bvh4_dp_collapse_on_the_standin(tmp_path, monkeypatch):
    """The same on a reduced stand-in (~24K triangles): valid, and fewer nodes than greedy."""
    from cudapathtracer_amd import scenes
    p = scenes.write_sponza_standin(str(tmp_path), scale_tris=0.06)
    s = pt.Scene()
    s.load_obj(p, mtl_basepath=os.path.dirname(p) + "/")
    got = {}
    for mode in ("dp", "greedy"):
        monkeypatch.setenv("PT_COLLAPSE", mode)
        got[mode] = s.accel_digest()
    assert got["dp"][1] < got["greedy"][1]


@pytest.mark.parametrize("knob", ["PT_COLLAPSE_CN", "PT_COLLAPSE_CT"])
@pytest.mark.parametrize("value", ["nan", "inf", "-1", "0", "abc", ""])
def test_bvh4_collapse_rejects_bad_cost_knobs(knob, value, monkeypatch):
    """The DP collapse's cost knobs must be finite and positive: with NaN/inf costs every comparison of
    the DP fails, no slot split is chosen and the emitted node could overflow its 4 slots.  A bad
    value is refused with PT_E_INVALID (naming the knob) instead of building a malformed tree; a good
    one still builds (accel_build.cpp)."""
    s = load_scene("cornell", build_bvh=False)
    monkeypatch.delenv("PT_COLLAPSE", raising=False)
    monkeypatch.setenv(knob, value)
    with pytest.raises(pt.PtError) as ei:
        s.accel_digest()
    assert knob in str(ei.value)
    monkeypatch.setenv(knob, "0.5")
    assert s.accel_digest()[1] > 0
