"""gfx950 render path vs the CPU oracle (kernel.cu:417-515 / 217-415 restated), through the C-ABI.

Bar: bit-exact.  The kernel and the oracle implement one arithmetic spec -- IEEE
float/double ops in the reference's order, no contraction, correctly rounded '/' and sqrt,
the same deterministic sin/cos -- so the fp32 image the kernel writes must equal the oracle's
f64 mean rounded to fp32 in every bit, for every traversal/skip/cache mode.  The north-star
tolerance (RMSE <= 1e-4 on c/(c+1), pixel 0 excluded) is checked as well, at sizes where only
properties can be checked.
"""
import os

import numpy as np
import pytest

from conftest import GOLD, load_scene

import cudapathtracer_amd as pt
from cudapathtracer_amd import shard

pytestmark = pytest.mark.gpu

CAM = dict(pos=(0.0, 1.0, 3.0), dist_from_film=1.0, focal_length=3.0, radius=0.0)   # kernel.cu:642-648


@pytest.fixture(scope="module")
def oracle_mod():
    import oracle
    return oracle


@pytest.fixture(scope="module")
def cb():
    s = load_scene("cornell_blob")
    r = pt.Renderer(s, 0)
    yield s, r
    r.close()


def _oracle(oracle_mod, scene, w, h, spp, bounces, integ, seed=1234, radius=0.0, pixels=None):
    osc = oracle_mod.OracleScene(scene.arrays())
    ocam = oracle_mod.camera(CAM["pos"], CAM["dist_from_film"], CAM["focal_length"], radius, w, h)
    img, cnt = oracle_mod.render(osc, ocam, w, h, spp, bounces, integ, seed, pixels=pixels)
    return img, cnt


def _bits_equal(a32, ref64):
    return int(np.count_nonzero(a32.view(np.uint32) != ref64.astype(np.float32).view(np.uint32)))


def _rmse_tonemapped(a, b):
    a = a.astype(np.float64).reshape(-1, 3)[1:]
    b = b.astype(np.float64).reshape(-1, 3)[1:]
    return float(np.sqrt(np.mean((a / (a + 1) - b / (b + 1)) ** 2)))


MODES = [0, pt.PT_FLAG_REFERENCE_TRAVERSAL, pt.PT_FLAG_NO_DEAD_PATH_SKIP | pt.PT_FLAG_NO_PRIMARY_CACHE,
         pt.PT_FLAG_REFERENCE_TRAVERSAL | pt.PT_FLAG_NO_DEAD_PATH_SKIP, pt.PT_FLAG_COUNT, pt.PT_FLAG_REFERENCE_BVH,
         pt.PT_FLAG_REFERENCE_BVH | pt.PT_FLAG_COUNT]


@pytest.mark.parametrize("flags", MODES)
@pytest.mark.parametrize("integ", [0, 1])
def test_bit_exact_vs_oracle(oracle_mod, cb, integ, flags):
    s, r = cb
    w, h, spp = 32, 32, 4
    img, st = r.render(pt.make_camera(width=w, height=h, **CAM), w, h, spp, bounces=3, integrator=integ,
                       flags=flags)
    ref, cnt = _oracle(oracle_mod, s, w, h, spp, 3, integ)
    assert _bits_equal(img, ref) == 0
    assert st["samples"] == w * h * spp
    # the reference's own trace count is reproduced exactly (traced <= reference)
    assert st["rays_reference"] == cnt["traces"]
    assert st["rays_traced"] <= st["rays_reference"]
    if flags & pt.PT_FLAG_NO_DEAD_PATH_SKIP and flags & pt.PT_FLAG_NO_PRIMARY_CACHE:
        assert st["rays_traced"] == cnt["traces"]
    if flags & pt.PT_FLAG_COUNT:
        assert st["node_tests"] > 0 and st["tri_tests"] > 0


@pytest.mark.parametrize("integ", [0, 1])
def test_two_triangle_scene(oracle_mod, integ):
    """One emissive quad (two triangles): the render path's tree is a root node with two single-
    triangle leaves -- pt_create used to fail on it (the SAH made the root a leaf)."""
    s = load_scene("quad")
    r = pt.Renderer(s, 0)
    try:
        w, h, spp = 24, 16, 3
        img, st = r.render(pt.make_camera(width=w, height=h, **CAM), w, h, spp, bounces=3, integrator=integ)
        ref, cnt = _oracle(oracle_mod, s, w, h, spp, 3, integ)
        assert _bits_equal(img, ref) == 0
        assert np.count_nonzero(img) > 0
        assert st["rays_reference"] == cnt["traces"]
    finally:
        r.close()


def test_matches_committed_fixture(cb):
    """The committed oracle render (tests/golden) pins both sides across rebuilds."""
    s, r = cb
    for integ in (0, 1):
        g = np.load(os.path.join(GOLD, "render_cornell_blob_32x32_s4_b3_i%d.npz" % integ))
        img, _ = r.render(pt.make_camera(width=32, height=32, **CAM), 32, 32, 4, bounces=3, integrator=integ)
        assert _bits_equal(img, g["img"]) == 0


@pytest.mark.parametrize("w,h,spp,bounces", [(24, 16, 3, 8), (13, 7, 5, 1), (1, 1, 3, 3), (40, 9, 2, 16)])
def test_ragged_images_and_depths(oracle_mod, w, h, spp, bounces):
    """Non-square, non-power-of-two and tile-ragged images (decision d3), depth 1..16."""
    s = load_scene("cornell")
    with pt.Renderer(s, 0) as r:
        img, st = r.render(pt.make_camera(width=w, height=h, **CAM), w, h, spp, bounces=bounces)
    ref, cnt = _oracle(oracle_mod, s, w, h, spp, bounces, 0)
    assert _bits_equal(img, ref) == 0
    assert st["rays_reference"] == cnt["traces"]


@pytest.mark.parametrize("lds_tree", ["1", "0"])
def test_tree_held_whole_in_lds(oracle_mod, monkeypatch, lds_tree):
    """A tree the LDS top holds whole (the Cornell box, C2's scene): integrator 0's walk steps read
    it from LDS (render_unidir_wf<false, 5, true>, with walk threshold 62 and two root-first visits)
    or, with PT_WF_LDS_TREE=0, from memory like a large tree's -- both bit-exact, both integrators."""
    monkeypatch.setenv("PT_WF_LDS_TREE", lds_tree)
    s = load_scene("cornell")
    w, h, spp = 24, 24, 4
    with pt.Renderer(s, 0) as r:
        for integ in (0, 1):
            img, st = r.render(pt.make_camera(width=w, height=h, **CAM), w, h, spp, bounces=8, integrator=integ)
            ref, cnt = _oracle(oracle_mod, s, w, h, spp, 8, integ)
            assert _bits_equal(img, ref) == 0, integ
            assert st["rays_reference"] == cnt["traces"]
            # the counting variant walks the same way: the same image, and (LDS walk) every node visit an LDS read
            img2, st2 = r.render(pt.make_camera(width=w, height=h, **CAM), w, h, spp, bounces=8, integrator=integ,
                                 flags=pt.PT_FLAG_COUNT)
            assert _bits_equal(img2, ref) == 0, integ
            assert st2["node_tests"] > 0
            if integ == 0 and lds_tree == "1":
                assert st2["lds_node_tests"] == st2["node_tests"]


def test_lens_radius_and_seed(oracle_mod, cb):
    """radius > 0 consumes the two lens draws per sample from the pixel's stream (decision d1)."""
    s, r = cb
    w, h = 16, 16
    cam = pt.make_camera(pos=CAM["pos"], dist_from_film=1.0, focal_length=3.0, radius=0.05, width=w, height=h)
    img, _ = r.render(cam, w, h, 3, bounces=3, seed=99)
    ref, _ = _oracle(oracle_mod, s, w, h, 3, 3, 0, seed=99, radius=0.05)
    assert _bits_equal(img, ref) == 0


def test_shards_sum_to_full_render(cb):
    """Tile sharding: every shard writes only its tiles and the sum is bit-identical."""
    s, r = cb
    w, h, spp = 40, 24, 2
    cam = pt.make_camera(width=w, height=h, **CAM)
    full, st = r.render(cam, w, h, spp)
    for n in (2, 3, 8):
        acc = np.zeros_like(full)
        tot = 0
        for k in range(n):
            part, stk = r.render(cam, w, h, spp, shard_index=k, shard_count=n)
            mask = np.zeros(w * h, dtype=bool)
            mask[shard.shard_pixels(w, h, k, n)] = True
            assert np.all(part.reshape(-1, 3)[~mask] == 0)
            acc += part
            tot += stk["samples"]
        assert _bits_equal(acc, full.astype(np.float64)) == 0
        assert tot == st["samples"]


@pytest.mark.parametrize("chunks,radius", [("1", 0.0), ("3", 0.0), ("7", 0.05), ("64", 0.0)])
def test_sample_chunk_units_bit_exact(oracle_mod, monkeypatch, chunks, radius):
    """Work units = (pixel, sample chunk): the XORWOW state fast-forwarded over earlier samples,
    per-sample radiance combined in order by finalize_pixels, the primary hit shared by a pixel's
    chunks.  Chunk counts that do not divide spp (7 of 9 samples: chunks of 1 and 2), more chunks
    than samples (64 -> capped at spp), lens draws in the replay, and whole-pixel units (1)."""
    monkeypatch.setenv("PT_WF_CHUNKS", chunks)
    s = load_scene("cornell_blob")
    w, h, spp = 24, 16, 9
    cam = pt.make_camera(pos=CAM["pos"], dist_from_film=1.0, focal_length=3.0, radius=radius, width=w, height=h)
    with pt.Renderer(s, 0) as r:
        img, st = r.render(cam, w, h, spp, bounces=3)
        parts = np.zeros_like(img)
        for k in range(3):
            part, _ = r.render(cam, w, h, spp, bounces=3, shard_index=k, shard_count=3)
            parts += part
    ref, cnt = _oracle(oracle_mod, s, w, h, spp, 3, 0, radius=radius)
    assert _bits_equal(img, ref) == 0
    assert _bits_equal(parts, img.astype(np.float64)) == 0
    assert st["samples"] == w * h * spp
    assert st["rays_reference"] == cnt["traces"]


@pytest.mark.parametrize("chunks,radius,tail", [("1", 0.0, None), ("3", 0.0, None), ("7", 0.05, None), ("2", 0.05, "100"),
                                               ("4", 0.0, "37")])
def test_head_wavefront_units_bit_exact(oracle_mod, monkeypatch, chunks, radius, tail):
    """Integrator 1 on the wavefront kernel with sample-chunk work units: a chunk's XORWOW state is
    fast-forwarded by the fixed 7 (+2 lens) draws per sample, its per-sample radiance combined in
    order, the camera hit shared by the pixel's chunks (pinhole); lens draws per sample.  Shards of 3
    sum to the same bits."""
    monkeypatch.setenv("PT_WF_CHUNKS", chunks)
    if tail is not None:
        monkeypatch.setenv("PT_WF_TAIL_NPIX", tail)
    s = load_scene("cornell_blob")
    w, h, spp = 24, 16, 9
    cam = pt.make_camera(pos=CAM["pos"], dist_from_film=1.0, focal_length=3.0, radius=radius, width=w, height=h)
    with pt.Renderer(s, 0) as r:
        img, st = r.render(cam, w, h, spp, bounces=3, integrator=1)
        parts = np.zeros_like(img)
        for k in range(3):
            part, _ = r.render(cam, w, h, spp, bounces=3, integrator=1, shard_index=k, shard_count=3)
            parts += part
    ref, cnt = _oracle(oracle_mod, s, w, h, spp, 3, 1, radius=radius)
    assert _bits_equal(img, ref) == 0
    assert _bits_equal(parts, img.astype(np.float64)) == 0
    assert st["samples"] == w * h * spp
    assert st["rays_reference"] == cnt["traces"]
    assert st["work_units"] >= w * h


@pytest.mark.parametrize("tail,chunks,radius", [("100", "3", 0.0), ("1", "9", 0.0), ("383", "2", 0.05),
                                               ("0", "4", 0.0)])
def test_tail_split_units_bit_exact(oracle_mod, monkeypatch, tail, chunks, radius):
    """Hybrid work units: whole pixels first, the last `tail` pixel slots split into sample chunks
    (PT_WF_TAIL_NPIX / PT_WF_CHUNKS; by default the last 0.75 pixel per resident lane in 6 chunks
    on large shards).  The split pixels' radiance is stored per sample and combined in order, the
    whole ones keep their running mean in the record: the same image bits as the oracle."""
    monkeypatch.setenv("PT_WF_TAIL_NPIX", tail)
    monkeypatch.setenv("PT_WF_CHUNKS", chunks)
    s = load_scene("cornell_blob")
    w, h, spp = 24, 16, 9
    cam = pt.make_camera(pos=CAM["pos"], dist_from_film=1.0, focal_length=3.0, radius=radius, width=w, height=h)
    with pt.Renderer(s, 0) as r:
        img, st = r.render(cam, w, h, spp, bounces=3)
        parts = np.zeros_like(img)
        for k in range(2):
            part, _ = r.render(cam, w, h, spp, bounces=3, shard_index=k, shard_count=2)
            parts += part
    ref, cnt = _oracle(oracle_mod, s, w, h, spp, 3, 0, radius=radius)
    assert _bits_equal(img, ref) == 0
    assert _bits_equal(parts, img.astype(np.float64)) == 0
    assert st["samples"] == w * h * spp
    assert st["rays_reference"] == cnt["traces"]


@pytest.mark.parametrize("mid,fine_px,fine,radius", [("2", "0.0003", "5", 0.0), ("4", "0.0001", "9", 0.05),
                                                    ("3", "0", "4", 0.0)])
def test_two_level_split_units_bit_exact(oracle_mod, monkeypatch, mid, fine_px, fine, radius):
    """Small shards split every pixel: all but the last pixels into `mid` chunks (longer units),
    the last ~fine_px x resident lanes pixels into `fine` chunks (PT_WF_MID_CHUNKS /
    PT_WF_FINE_PX / PT_WF_FINE_CHUNKS): the same image bits as the oracle."""
    monkeypatch.setenv("PT_WF_MID_CHUNKS", mid)
    monkeypatch.setenv("PT_WF_FINE_PX", fine_px)
    monkeypatch.setenv("PT_WF_FINE_CHUNKS", fine)
    s = load_scene("cornell_blob")
    w, h, spp = 24, 16, 9
    cam = pt.make_camera(pos=CAM["pos"], dist_from_film=1.0, focal_length=3.0, radius=radius, width=w, height=h)
    with pt.Renderer(s, 0) as r:
        img, st = r.render(cam, w, h, spp, bounces=3)
    ref, cnt = _oracle(oracle_mod, s, w, h, spp, 3, 0, radius=radius)
    assert _bits_equal(img, ref) == 0
    assert st["samples"] == w * h * spp
    assert st["rays_reference"] == cnt["traces"]


@pytest.mark.parametrize("mid,fine_px,fine,fin_px,fin,radius", [("2", "0.0003", "4", "0.0001", "9", 0.0),
                                                              ("3", "0.0005", "3", "0.0002", "5", 0.05),
                                                              ("0", "0", "3", "0.0003", "7", 0.0)])
def test_three_grade_split_units_bit_exact(oracle_mod, monkeypatch, mid, fine_px, fine, fin_px, fin, radius):
    """A third, final grade of split units (PT_WF_FIN_PX / PT_WF_FIN_CHUNKS: the queue's last
    pixels in the most chunks, down to one sample per unit): the same image bits as the oracle."""
    monkeypatch.setenv("PT_WF_MID_CHUNKS", mid)
    monkeypatch.setenv("PT_WF_FINE_PX", fine_px)
    monkeypatch.setenv("PT_WF_FINE_CHUNKS", fine)
    monkeypatch.setenv("PT_WF_FIN_PX", fin_px)
    monkeypatch.setenv("PT_WF_FIN_CHUNKS", fin)
    s = load_scene("cornell_blob")
    w, h, spp = 24, 16, 9
    cam = pt.make_camera(pos=CAM["pos"], dist_from_film=1.0, focal_length=3.0, radius=radius, width=w, height=h)
    with pt.Renderer(s, 0) as r:
        img, st = r.render(cam, w, h, spp, bounces=3)
    ref, cnt = _oracle(oracle_mod, s, w, h, spp, 3, 0, radius=radius)
    assert _bits_equal(img, ref) == 0
    assert st["samples"] == w * h * spp
    assert st["rays_reference"] == cnt["traces"]


def test_rmse_and_properties_larger(oracle_mod, cb):
    """North-star tolerance on a subset of a larger render (oracle only on the subset)."""
    s, r = cb
    w = h = 256
    spp = 8
    cam = pt.make_camera(width=w, height=h, **CAM)
    img, st = r.render(cam, w, h, spp, bounces=3)
    assert np.isfinite(img).all() and (img >= 0).all()
    pix = shard.shard_pixels(w, h, 5, 97)
    ref, _ = _oracle(oracle_mod, s, w, h, spp, 3, 0, pixels=pix)
    a = img.reshape(-1, 3)[pix]
    b = ref.reshape(-1, 3)[pix]
    assert _rmse_tonemapped(a, b) <= 1e-4
    assert int(np.count_nonzero(a.view(np.uint32) != b.astype(np.float32).view(np.uint32))) == 0


def test_culled_walk_agrees_with_reference_walk_standin(tmp_path):
    """On the 262K-triangle stand-in the culled near-first walk returns the reference walk's
    hits: the two renders must agree bit-for-bit (and so must their reference ray counts)."""
    from cudapathtracer_amd import scenes
    p = scenes.write_sponza_standin(str(tmp_path))
    s = pt.Scene()
    s.load_obj(p, mtl_basepath=os.path.dirname(p) + "/")
    s.build_bvh()
    w, h = 96, 64
    cam = pt.make_camera(width=w, height=h, **scenes.SPONZA_STANDIN_CAMERA)
    with pt.Renderer(s, 0) as r:
        a, sa = r.render(cam, w, h, 4, bounces=3, flags=pt.PT_FLAG_COUNT)
        b, sb = r.render(cam, w, h, 4, bounces=3, flags=pt.PT_FLAG_REFERENCE_TRAVERSAL)
        c, sc = r.render(cam, w, h, 4, bounces=3, flags=pt.PT_FLAG_REFERENCE_BVH)
    assert _bits_equal(a, b.astype(np.float64)) == 0
    assert _bits_equal(c, b.astype(np.float64)) == 0
    assert sa["rays_reference"] == sb["rays_reference"] == sc["rays_reference"]
    # the SAH walk's winners are checked against the reference BVH; re-walks must be rare
    assert sa["accel_fallbacks"] <= max(10, sa["rays_traced"] // 10000)


def test_gpu_output_step_equals_host_tonemap(cb, tmp_path):
    """pt_tonemap (GPU threshold table) == pt_tonemap_u8 (host libm) on a render and on edge
    values (0, -0, subnormal, FLT_MAX, inf, NaN, negatives redone on the host); the PPM written
    from GPU codes is byte-identical to the host writer's."""
    s, r = cb
    w, h = 40, 24
    img, _ = r.render(pt.make_camera(width=w, height=h, **CAM), w, h, 3)
    codes = r.tonemap(img)
    ref = np.vectorize(pt.tonemap_u8)(img.astype(np.float64))
    assert np.array_equal(codes, ref)
    a, b = str(tmp_path / "a.ppm"), str(tmp_path / "b.ppm")
    pt.write_ppm(a, img)
    pt.write_ppm_codes(b, codes)
    assert open(a, "rb").read() == open(b, "rb").read()
    edge = np.array([0.0, -0.0, 1e-45, 1e-38, 3.4028235e38, np.inf, np.nan, -0.5, -1.0, -2.0, 1.0, 0.25],
                    dtype=np.float32)
    e = np.resize(edge, (1, 4, 3))
    assert np.array_equal(r.tonemap(e), np.vectorize(pt.tonemap_u8)(e.astype(np.float64)))


@pytest.mark.parametrize("integ", [0, 1])
def test_per_triangle_counts_match_reference(oracle_mod, cb, integ):
    """The reference's test[] buffer (kernel.cu:133, :694-697): with the reference traversal and
    both shortcuts off the render performs exactly the reference's trace() calls, so the
    per-triangle test counts equal the oracle's (whose trace is pinned to the reference's own
    trace(), tests/test_oracle.py); the default fast path reports the tests it performed."""
    s, r = cb
    w, h, spp = 24, 16, 3
    cam = pt.make_camera(width=w, height=h, **CAM)
    flags = (pt.PT_FLAG_REFERENCE_TRAVERSAL | pt.PT_FLAG_NO_PRIMARY_CACHE | pt.PT_FLAG_NO_DEAD_PATH_SKIP |
             pt.PT_FLAG_COUNT | pt.PT_FLAG_TRI_COUNTS)
    img, st = r.render(cam, w, h, spp, bounces=3, integrator=integ, flags=flags)
    counts = r.tri_counts()
    osc = oracle_mod.OracleScene(s.arrays())
    ocam = oracle_mod.camera(CAM["pos"], CAM["dist_from_film"], CAM["focal_length"], 0.0, w, h)
    ocounts = np.zeros(len(osc.tris), dtype=np.uint32)
    ref, cnt = oracle_mod.render(osc, ocam, w, h, spp, 3, integ, 1234, tri_counts=ocounts)
    assert _bits_equal(img, ref) == 0
    assert np.array_equal(counts, ocounts)
    assert int(counts.sum()) == st["tri_tests"] == cnt["tri_tests"]
    # the fast path's own counts: fewer tests, same image
    img2, st2 = r.render(cam, w, h, spp, bounces=3, integrator=integ, flags=pt.PT_FLAG_COUNT | pt.PT_FLAG_TRI_COUNTS)
    fast = r.tri_counts()
    assert _bits_equal(img2, ref) == 0
    assert 0 < int(fast.sum()) < int(counts.sum())
    assert int(fast.sum()) >= st2["tri_tests"]


@pytest.mark.parametrize("budget", ["0", "0.002"])
def test_split_buffer_budget_fallback_bit_exact(oracle_mod, monkeypatch, budget):
    """Split pixels keep per-sample radiance (24 B per sample); over the memory budget
    (PT_LBUF_BUDGET_MB) the split shrinks -- to nothing at 0, to a few slots at 2 KB (the partial
    cap: 14 slots of 144 B, the rest whole-pixel units) -- and the shards still sum to the oracle's
    image bit for bit."""
    s = load_scene("cornell_blob")
    w, h, spp = 64, 48, 6
    cam = pt.make_camera(width=w, height=h, **CAM)
    with pt.Renderer(s, 0) as r:
        _, st0 = r.render(cam, w, h, spp, bounces=3)   # (no budget set: every pixel of this small image split)
    assert st0["split_pixels"] == w * h
    monkeypatch.setenv("PT_LBUF_BUDGET_MB", budget)
    with pt.Renderer(s, 0) as r:
        full, st = r.render(cam, w, h, spp, bounces=3)
        if budget == "0":
            assert st["split_pixels"] == 0 and st["work_units"] == w * h
        else:
            assert st["split_pixels"] == (2097 // (spp * 24))
            assert w * h < st["work_units"] < st0["work_units"]
        parts = np.zeros_like(full)
        for k in range(4):
            part, _ = r.render(cam, w, h, spp, bounces=3, shard_index=k, shard_count=4)
            parts += part
    ref, cnt = _oracle(oracle_mod, s, w, h, spp, 3, 0)
    assert _bits_equal(full, ref) == 0
    assert _bits_equal(parts, ref) == 0
    assert st["rays_reference"] == cnt["traces"]


def test_group_render_one_device_equals_render(cb):
    """pt_render_group (RCCL reduce of the image-tile shards) on the box's one device: a
    1-communicator group, bit-identical to pt_render, stats summed; a second context on the same
    device is refused (one context per device)."""
    s, r = cb
    w, h, spp = 40, 24, 4
    cam = pt.make_camera(width=w, height=h, **CAM)
    ref, st = r.render(cam, w, h, spp, bounces=3)
    with pt.Group([r]) as g:
        img, gst = g.render(cam, w, h, spp, bounces=3)
        img2, _ = g.render(cam, w, h, spp, bounces=3)   # buffers and communicator reused
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(img2.view(np.uint32), ref.view(np.uint32))
    assert gst["samples"] == st["samples"] == w * h * spp
    assert gst["rays_nominal"] == st["rays_nominal"] == w * h * spp * 4
    assert gst["work_units"] == st["work_units"] > 0
    assert gst["split_pixels"] == st["split_pixels"]
    with pt.Renderer(s, 0) as r2:
        with pytest.raises(pt.PtError) as e:
            pt.Group([r, r2])
        assert e.value.code == pt.PT_E_INVALID


@pytest.mark.parametrize("integ", [0, 1])
def test_morton_pixel_order_and_tile_sizes(oracle_mod, cb, tmp_path, integ):
    """pt_params.pixel_order = PT_ORDER_MORTON writes pixel (x,y) at out[mortonPxltoI(x,y)] -- the
    reference's imgBuff (kernel.cu:543,552) -- so the reference's own PPM loop (kernel.cu:763-778,
    restated by the oracle and pinned to the compiled loop by kat_ppm_morton.npz) turns the buffer into
    the bytes pt_write_ppm makes from the scanline render.  tile_w/tile_h change only which shard renders
    a pixel: shards of 16x24 and 32x8 tiles sum to the same bits, in either order."""
    s, r = cb
    w = h = 64
    spp = 3
    cam = pt.make_camera(width=w, height=h, **CAM)
    scan, st = r.render(cam, w, h, spp, bounces=3, integrator=integ)
    mort, stm = r.render(cam, w, h, spp, bounces=3, integrator=integ, pixel_order=pt.PT_ORDER_MORTON)
    assert mort.shape == (w * h, 3)
    assert np.array_equal(shard.to_scanline(mort, w, h).view(np.uint32), scan.view(np.uint32))
    ref, _ = _oracle(oracle_mod, s, w, h, spp, 3, integ)
    assert _bits_equal(scan, ref) == 0
    a, b, c = str(tmp_path / "a.ppm"), str(tmp_path / "b.ppm"), str(tmp_path / "c.ppm")
    pt.write_ppm(a, scan)
    oracle_mod.write_ppm_imgbuf(b, mort, w, h)                       # the reference's loop, unchanged
    pt.write_ppm(c, mort, pixel_order=pt.PT_ORDER_MORTON, width=w, height=h)
    assert open(a, "rb").read() == open(b, "rb").read() == open(c, "rb").read()
    for tw, th, n in ((16, 24, 3), (32, 8, 2), (64, 64, 5)):
        for order, full in ((pt.PT_ORDER_SCANLINE, scan), (pt.PT_ORDER_MORTON, mort)):
            acc = np.zeros_like(full)
            for k in range(n):
                part, _ = r.render(cam, w, h, spp, bounces=3, integrator=integ, shard_index=k, shard_count=n,
                                   pixel_order=order, tile_w=tw, tile_h=th)
                pix = shard.shard_pixels(w, h, k, n, tw, th)
                if order == pt.PT_ORDER_MORTON:
                    pix = shard.morton_index(pix % w, pix // w).astype(np.int64)
                mask = np.zeros(w * h, dtype=bool)
                mask[pix] = True
                assert np.all(part.reshape(-1, 3)[~mask] == 0)
                acc += part
            assert np.array_equal(acc.view(np.uint32), full.view(np.uint32))
    # the reference's Morton buffer is defined for square power-of-two images only
    for bw, bh in ((64, 32), (48, 48)):
        with pytest.raises(pt.PtError) as e:
            r.render(pt.make_camera(width=bw, height=bh, **CAM), bw, bh, 1, pixel_order=pt.PT_ORDER_MORTON)
        assert e.value.code == pt.PT_E_INVALID
    with pytest.raises(pt.PtError):
        r.render(cam, w, h, 1, tile_w=12, tile_h=8)


def _devices():
    import torch
    return torch.cuda.device_count()


def test_group_render_multi_device_equals_render():
    """pt_render_group on every visible device (>= 2; skipped on a one-GPU box): shards rendered
    concurrently, one ncclReduce over xGMI -- bit-identical to one device, also on a second frame that
    reuses the group's buffers."""
    n = _devices()
    if n < 2:
        pytest.skip("one visible device")
    s = load_scene("cornell_blob")
    w, h, spp = 64, 48, 4
    cam = pt.make_camera(width=w, height=h, **CAM)
    rs = [pt.Renderer(s, d) for d in range(n)]
    try:
        ref, st = rs[0].render(cam, w, h, spp, bounces=3)
        with pt.Group(rs) as g:
            for _ in range(2):
                img, gst = g.render(cam, w, h, spp, bounces=3)
                assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
                assert gst["samples"] == st["samples"]
            cam64 = pt.make_camera(width=64, height=64, **CAM)
            mort, _ = g.render(cam64, 64, 64, spp, bounces=3, pixel_order=pt.PT_ORDER_MORTON)
            scan, _ = rs[0].render(cam64, 64, 64, spp, bounces=3)
            assert np.array_equal(shard.to_scanline(mort, 64, 64).view(np.uint32), scan.view(np.uint32))
    finally:
        for r in rs:
            r.close()


def test_async_renders_queue_back_to_back(cb):
    """pt_render_device_async / pt_render_wait: two frames queued on one stream (different shards, one
    with the other integrator), collected oldest first -- the same bits and stats as blocking renders;
    a third enqueue and a blocking render are refused while two are in flight."""
    import torch
    s, r = cb
    w, h, spp = 40, 24, 3
    cam = pt.make_camera(width=w, height=h, **CAM)
    ref0, st0 = r.render(cam, w, h, spp, bounces=3, shard_index=0, shard_count=2)
    ref1, st1 = r.render(cam, w, h, spp, bounces=3, integrator=1, shard_index=1, shard_count=2)
    a = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda")
    b = torch.zeros_like(a)
    stream = torch.cuda.current_stream().cuda_stream
    r.render_device_async(cam, a.data_ptr(), w, h, spp, bounces=3, shard_index=0, shard_count=2, stream_ptr=stream)
    r.render_device_async(cam, b.data_ptr(), w, h, spp, bounces=3, integrator=1, shard_index=1, shard_count=2,
                          stream_ptr=stream)
    with pytest.raises(pt.PtError):
        r.render_device_async(cam, b.data_ptr(), w, h, spp, stream_ptr=stream)
    with pytest.raises(pt.PtError):
        r.render(cam, w, h, spp)
    sa = r.wait()
    sb = r.wait()
    with pytest.raises(pt.PtError):
        r.wait()
    assert np.array_equal(a.cpu().numpy().view(np.uint32), ref0.view(np.uint32))
    assert np.array_equal(b.cpu().numpy().view(np.uint32), ref1.view(np.uint32))
    for k in ("samples", "rays_reference", "work_units"):
        assert sa[k] == st0[k] and sb[k] == st1[k]
    # traced rays may differ by a few: a split pixel's later chunk traces its primary ray itself when
    # the pixel's chunk 0 has not yet published it (a race of timing, not of results)
    for x, y in ((sa, st0), (sb, st1)):
        assert 0 < x["rays_traced"] <= x["rays_reference"] and abs(x["rays_traced"] - y["rays_traced"]) <= x["samples"]
    # the per-triangle counts are one context-wide buffer: a render filling them is refused while
    # another render is in flight
    r.render_device_async(cam, a.data_ptr(), w, h, spp, bounces=3, stream_ptr=stream)
    with pytest.raises(pt.PtError) as e:
        r.render_device_async(cam, b.data_ptr(), w, h, spp, bounces=3, stream_ptr=stream,
                              flags=pt.PT_FLAG_COUNT | pt.PT_FLAG_TRI_COUNTS)
    assert e.value.code == pt.PT_E_INVALID
    r.wait()


@pytest.mark.gpu
def test_async_renders_on_two_streams(cb):
    """Two renders queued on two streams (frames that may run concurrently: each in-flight slot has its own
    scratch -- records, unit table, split-pixel samples, memo words, queues, seed table), repeated so that
    both slots are reused: every image and count equals the blocking render's."""
    import torch
    s, r = cb
    w, h, spp = 96, 64, 6
    cam = pt.make_camera(width=w, height=h, **CAM)
    cases = [dict(shard_index=0, shard_count=3), dict(shard_index=2, shard_count=3, integrator=1),
             dict(shard_index=1, shard_count=3)]
    refs = [r.render(cam, w, h, spp, bounces=3, **kw) for kw in cases]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bufs = [torch.zeros((h, w, 3), dtype=torch.float32, device="cuda") for _ in range(2)]
    got = []
    for rep in range(2):
        for k, kw in enumerate(cases):
            st = streams[k % 2]
            with torch.cuda.stream(st):
                bufs[k % 2].zero_()
                r.render_device_async(cam, bufs[k % 2].data_ptr(), w, h, spp, bounces=3, stream_ptr=st.cuda_stream, **kw)
            if k % 2 == 1 or k == len(cases) - 1:   # collect after both slots were queued
                while True:
                    try:
                        got.append(r.wait())
                    except pt.PtError:
                        break
                torch.cuda.synchronize()
                for j in range(k - (1 if k % 2 == 1 else 0), k + 1):
                    img = bufs[j % 2].cpu().numpy()
                    assert np.array_equal(img.view(np.uint32), refs[j][0].view(np.uint32)), (rep, j)
    assert len(got) == 2 * len(cases)
    for j, st in enumerate(got):
        ref = refs[j % len(cases)][1]
        for key in ("samples", "rays_reference", "work_units", "split_pixels"):
            assert st[key] == ref[key], (j, key)
