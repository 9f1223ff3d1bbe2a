"""Diagnostics: render a small config on the GPU under several flag sets and report where the
image differs from the oracle (pixel, Morton index, values).  Usage: python tools/debug/render_diff.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
from conftest import load_scene  # noqa: E402

import cudapathtracer_amd as pt  # noqa: E402

W = H = int(os.environ.get("DBG_SIZE", "32"))
SPP = int(os.environ.get("DBG_SPP", "4"))
scene = os.environ.get("DBG_SCENE", "cornell_blob")
s = load_scene(scene)
osc = oracle.OracleScene(s.arrays())
ocam = oracle.camera((0.0, 1.0, 3.0), 1.0, 3.0, 0.0, W, H)
ref, _ = oracle.render(osc, ocam, W, H, SPP, 3, 0, 1234)
ref = ref.astype(np.float32)
cam = pt.make_camera((0.0, 1.0, 3.0), 1.0, 3.0, 0.0, W, H)
with pt.Renderer(s, 0) as r:
    for name, fl in [("default", 0), ("no_cache", pt.PT_FLAG_NO_PRIMARY_CACHE), ("no_skip", pt.PT_FLAG_NO_DEAD_PATH_SKIP),
                     ("no_cache_no_skip", pt.PT_FLAG_NO_PRIMARY_CACHE | pt.PT_FLAG_NO_DEAD_PATH_SKIP),
                     ("count", pt.PT_FLAG_COUNT), ("reference_bvh", pt.PT_FLAG_REFERENCE_BVH)]:
        img, st = r.render(cam, W, H, SPP, 3, 0, 1234, fl)
        bad = np.nonzero(np.any(img.view(np.uint32) != ref.view(np.uint32), axis=2))
        print("%-18s bad_pixels=%d fallbacks=%d traced=%d" % (name, len(bad[0]), st["accel_fallbacks"], st["rays_traced"]))
        for y, x in list(zip(*bad))[:6]:
            print("   px=(%d,%d) morton=%d got=%s ref=%s" % (x, y, pt.morton_pxl_to_i(x, y), img[y, x].tolist(), ref[y, x].tolist()))
