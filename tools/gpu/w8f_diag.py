#!/usr/bin/env python3
"""Diagnose the full-precision 8-wide experiment's integrator-1 divergence (round 3, profiles/r03_w8f):
render C3 with integrator 1 on the wavefront kernel and on the tile kernel (PT_HEAD_WF=0) of the variant
library (PT_LIB=variants/w8f/libptamd.so, built from the round-3 tree + wide8_full_precision.diff), list
the pixels that differ and check each against the CPU oracle, to tell which kernel is wrong."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import cudapathtracer_amd as pt  # noqa: E402
from cudapathtracer_amd import scenes  # noqa: E402
import oracle  # noqa: E402

out_dir = sys.argv[1]
os.makedirs(out_dir, exist_ok=True)
d = os.path.join("/tmp", "w8f_scene")
os.makedirs(d, exist_ok=True)
p = scenes.write_sponza_standin(d)
s = pt.Scene()
s.load_obj(p, mtl_basepath=os.path.dirname(p) + "/")
s.build_bvh()
w, h, spp = 1920, 1080, int(os.environ.get("W8F_SPP", "256"))
cam_kw = scenes.SPONZA_STANDIN_CAMERA
cam = pt.make_camera(width=w, height=h, **cam_kw)
with pt.Renderer(s, 0) as r:
    a, sa = r.render(cam, w, h, spp, bounces=3, integrator=1)
os.environ["PT_HEAD_WF"] = "0"
with pt.Renderer(s, 0) as r2:
    b, sb = r2.render(cam, w, h, spp, bounces=3, integrator=1)
diff = np.any(a.view(np.uint32) != b.view(np.uint32), axis=2)
ys, xs = np.nonzero(diff)
res = {"lib": pt.LIB_PATH, "spp": spp, "differing_pixels": int(diff.sum()), "pixels": []}
print("differing pixels:", int(diff.sum()), flush=True)
if len(xs):
    osc = oracle.OracleScene(s.arrays())
    ocam = oracle.camera(cam_kw["pos"], cam_kw["dist_from_film"], cam_kw["focal_length"], cam_kw["radius"], w, h)
    pix = (ys * w + xs)[:32].astype(np.uint32)
    ref, _ = oracle.render(osc, ocam, w, h, spp, 3, 1, 1234, pixels=pix)
    for q in pix:
        x, y = int(q) % w, int(q) // w
        o = ref[y, x].astype(np.float32)
        row = {"x": x, "y": y, "wavefront": a[y, x].tolist(), "tile": b[y, x].tolist(), "oracle": o.tolist(),
               "wavefront_eq_oracle": bool(np.array_equal(a[y, x].view(np.uint32), o.view(np.uint32))),
               "tile_eq_oracle": bool(np.array_equal(b[y, x].view(np.uint32), o.view(np.uint32)))}
        res["pixels"].append(row)
        print(row, flush=True)
json.dump(res, open(os.path.join(out_dir, "w8f_diag.json"), "w"), indent=1)
