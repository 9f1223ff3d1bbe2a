"""Whole frames against the oracle: the product renders a BASELINE config's entire image on the GPU, the CPU oracle
(oracle/pt_oracle.c, all host threads) renders every pixel of the same frame, and the fp32 images must be equal bit for
bit (kernel.cu:417-515 via the oracle's restatement).  The default GPU suite compares pixel subsets at these sizes;
this covers every pixel.

Opt-in (CPU-heavy): PT_FULL_FRAME=C2,C3,C4,C3H selects the configs (C3H: C3 with the HEAD integrator, kernel.cu:217-415;
skipped otherwise); PT_FULL_FRAME_LOG=path receives a progress line per band of rows and a result line per config.  C3
takes ~2 min of 16 host threads, C4 ~9 min, C3H ~6 min; PT_FULL_FRAME_PART=k/n checks the k-th of n horizontal bands
only (a long frame split over several runs; the GPU still renders the whole frame).
"""
import json
import os
import sys
import time

import numpy as np
import pytest

import cudapathtracer_amd as pt

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEL = [c for c in os.environ.get("PT_FULL_FRAME", "").split(",") if c]


def _log(msg):
    p = os.environ.get("PT_FULL_FRAME_LOG")
    if p:
        with open(p, "a") as fh:
            fh.write(msg + "\n")


@pytest.mark.parametrize("cfg", ["C2", "C3", "C4", "C3H", "C2H", "C4H", "C5"])
def test_full_frame_matches_the_oracle(cfg, tmp_path):
    if cfg not in SEL:
        pytest.skip("PT_FULL_FRAME does not select %s" % cfg)
    sys.path.insert(0, ROOT)
    import bench
    import oracle
    from cudapathtracer_amd import scenes
    integ = 1 if cfg.endswith("H") else 0
    c = bench.CONFIGS[cfg.rstrip("H")]
    W, H, spp, D = c["width"], c["height"], c["spp"], c["bounces"]
    path, mtl, _ = bench.scene_path(str(tmp_path), c["scene"])
    s = pt.Scene()
    s.load_obj(path, mtl_basepath=mtl)
    s.build_bvh()
    cam_kw = dict(scenes.CORNELL_CAMERA if c["scene"] == "cornell" else scenes.SPONZA_STANDIN_CAMERA)
    with pt.Renderer(s, 0) as r:
        cam = pt.make_camera(width=W, height=H, **cam_kw)
        t0 = time.time()
        img, st = r.render(cam, W, H, spp, bounces=D, integrator=integ)
        gpu_s = time.time() - t0
    osc = oracle.OracleScene(s.arrays())
    ocam = oracle.camera(cam_kw["pos"], cam_kw["dist_from_film"], cam_kw["focal_length"], cam_kw["radius"], W, H)
    threads = int(os.environ.get("PT_FULL_FRAME_THREADS", "0")) or bench.host_cores()
    ref = np.zeros((H, W, 3), dtype=np.float64)
    traces = 0
    k, n = (int(x) for x in os.environ.get("PT_FULL_FRAME_PART", "0/1").split("/"))
    ya, yb = k * H // n, (k + 1) * H // n
    band = max(1, min(H // 24, (yb - ya) // 8))
    t0 = time.time()
    for y0 in range(ya, yb, band):
        y1 = min(yb, y0 + band)
        pix = np.arange(y0 * W, y1 * W, dtype=np.uint32)
        part, cnt = oracle.render(osc, ocam, W, H, spp, D, integ, 1234, pixels=pix, threads=threads)
        ref[y0:y1] = part[y0:y1]
        traces += cnt["traces"]
        _log("%s rows %d-%d done, %.0f s" % (cfg, y0, y1, time.time() - t0))
    cpu_s = time.time() - t0
    img, ref = img[ya:yb], ref[ya:yb]
    diff = int(np.count_nonzero(img.view(np.uint32) != ref.astype(np.float32).view(np.uint32)))
    _log(json.dumps(dict(config=cfg, integrator=integ, width=W, height=H, rows=[ya, yb], spp=spp, bounces=D,
                         pixels=W * (yb - ya), samples=W * (yb - ya) * spp,
                         differing_values=diff, rays_reference_gpu=int(st["rays_reference"]), traces_oracle=int(traces),
                         gpu_render_s=round(gpu_s, 3), oracle_s=round(cpu_s, 1), oracle_threads=threads,
                         nonzero=int(np.count_nonzero(img)))))
    assert diff == 0, (cfg, diff)
    if (ya, yb) == (0, H):
        assert st["rays_reference"] == traces, cfg
