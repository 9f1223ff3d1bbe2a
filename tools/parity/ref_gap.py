#!/usr/bin/env python3
"""Gap between this build's arithmetic spec and the reference's own binary, on the CPU.

The GPU kernels are bit-exact to the oracle (oracle/pt_oracle.c), whose spec fixes three things the
reference's CUDA binary does differently or unknowably ("What's missing" 1):
  (i)   FMA contraction: nvcc's default -fmad=true fuses the a*b+c shapes of kernel.cu / modelLoader.h /
        camera.h (compile.bat:4 passes no -fmad=false); this build compiles with -ffp-contract=off;
  (ii)  sin/cos of the sampling angles: det_sincos instead of CUDA's cosf/sinf (kernel.cu:68,86-87),
        whose documented error bound is 2 ulp;
  (iii) curand_uniform's x*2^-32 + 2^-33 (kernel.cu:58): fused here, as nvcc would contract it.
Each sensitivity build of the oracle (oracle/Makefile VARIANTS) changes ONE of these; this script
renders the same pixel subset with each and reports, against the default oracle, the RMSE of the
tone-mapped value c/(c+1) (pixel index 0 excluded), the fraction of pixels whose fp32
mean differs, and the largest per-channel difference.  (cuRAND's seeding salts, the third unpinned
item, cannot be varied meaningfully: a different salt is a different random stream, i.e. Monte Carlo
noise of the full estimator, not a perturbation.)

Workloads (pixel subsets sized for seconds of CPU each):
  C2  the build's Cornell mesh, 1024x1024, 64 spp, depth 8 -- every k-th 8x8 tile
  C3  the ~262K-triangle stand-in, 1920x1080, 256 spp, depth 3 -- every k-th 8x8 tile
Usage: python tools/parity/ref_gap.py [--tiles-c2 N] [--tiles-c3 N] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402  (checker; this is a measurement tool, never the product)

WORKLOADS = {
    "C2": dict(scene="cornell", width=1024, height=1024, spp=64, bounces=8),
    "C3": dict(scene="standin", width=1920, height=1080, spp=256, bounces=3),
}


def load_scene(kind, cache_dir):
    import cudapathtracer_amd as pt
    from cudapathtracer_amd import scenes
    if kind == "cornell":
        p = os.path.join(cache_dir, "models", "cornell.obj")
        if not os.path.exists(p):
            scenes.write_cornell(cache_dir)
        cam = scenes.CORNELL_CAMERA
    else:
        p = os.path.join(cache_dir, "models", "sponza_standin.obj")
        if not os.path.exists(p):
            scenes.write_sponza_standin(cache_dir)
        cam = scenes.SPONZA_STANDIN_CAMERA
    s = pt.Scene()
    s.load_obj(p, mtl_basepath=os.path.dirname(p) + "/")
    s.build_bvh()
    return oracle.OracleScene(s.arrays()), cam


def subset_pixels(w, h, ntiles_want):
    from cudapathtracer_amd import shard
    tx, ty = shard.tiles_shape(w, h)
    n = tx * ty
    stride = max(1, n // max(1, ntiles_want))
    tiles = np.arange(stride // 2, n, stride)[:ntiles_want]
    pix = shard.tile_pixels(w, h, tiles)
    pix = pix[pix != 0]   # pixel (0,0) = Morton index 0: the reference's racy camera draws (d1)
    return pix, stride


def primary_hits(osc, ocam, w, pix, variant):
    """(triangle, t bits) of each pixel's camera ray (sample-invariant without lens draws: the memo)
    as the given build computes cameraRay and trace()."""
    import ctypes as C
    L = oracle.lib(variant)
    rays = np.empty((len(pix), 6), dtype=np.float32)
    o, d = oracle.OVec3(), oracle.OVec3()
    for k, p in enumerate(pix):
        idx = L.or_morton_pxl_to_i(int(p) % w, int(p) // w)
        L.or_camera_ray(C.byref(ocam), idx, float("nan"), float("nan"), C.byref(o), C.byref(d))
        rays[k] = (o.x, o.y, o.z, d.x, d.y, d.z)
    tri = np.empty(len(pix), dtype=np.int32)
    t = np.empty(len(pix), dtype=np.float32)
    L.or_trace_batch(C.byref(osc.c), len(pix), rays.ctypes.data, tri.ctypes.data, t.ctypes.data)
    return tri, t.view(np.uint32)


def gap(ref, var, pix, prim_flip, prim_tri_flip=None):
    """Metrics of var against ref over the subset's pixels (f64 means, (H, W, 3)); prim_flip marks the
    pixels whose camera ray hits another triangle (or another t) in the variant build, prim_tri_flip
    those whose camera ray hits another triangle."""
    a = ref.reshape(-1, 3)[pix]
    b = var.reshape(-1, 3)[pix]
    ta, tb = a / (a + 1.0), b / (b + 1.0)
    d = tb - ta
    diff32 = np.any(a.astype(np.float32) != b.astype(np.float32), axis=1)
    keep = ~prim_flip
    dk = d[keep]
    out = {
        "rmse_tonemapped": float(np.sqrt(np.mean(d * d))),
        "max_abs_tonemapped": float(np.max(np.abs(d))) if d.size else 0.0,
        "pixels_differing_fp32": int(diff32.sum()),
        "pixels": int(len(pix)),
        "frac_pixels_differing": float(diff32.mean()) if len(pix) else 0.0,
        "nan_pixels": int(np.isnan(b).any(axis=1).sum()),
        "primary_hit_flips": int(prim_flip.sum()),
        "rmse_tonemapped_no_primary_flips": float(np.sqrt(np.mean(dk * dk))) if dk.size else 0.0,
        "max_abs_tonemapped_no_primary_flips": float(np.max(np.abs(dk))) if dk.size else 0.0,
    }
    if prim_tri_flip is not None:
        dt = d[~prim_tri_flip]
        out["primary_triangle_flips"] = int(prim_tri_flip.sum())
        out["rmse_tonemapped_no_primary_triangle_flips"] = float(np.sqrt(np.mean(dt * dt))) if dt.size else 0.0
    return out


def run(name, tiles, threads, cache_dir, variants, pairs=()):
    cfg = WORKLOADS[name]
    osc, cam_kw = load_scene(cfg["scene"], cache_dir)
    w, h, spp, bounces = cfg["width"], cfg["height"], cfg["spp"], cfg["bounces"]
    ocam = oracle.camera(cam_kw["pos"], cam_kw["dist_from_film"], cam_kw["focal_length"], cam_kw["radius"], w, h)
    pix, stride = subset_pixels(w, h, tiles)
    t0 = time.time()
    ref, _ = oracle.render(osc, ocam, w, h, spp, bounces, 0, 1234, pixels=pix, threads=threads)
    t_ref = time.time() - t0
    rows = {}
    tri0, t0b = primary_hits(osc, ocam, w, pix, None)
    imgs = {}
    for v in variants:
        t0 = time.time()
        img, _ = oracle.render(osc, ocam, w, h, spp, bounces, 0, 1234, pixels=pix, threads=threads, variant=v)
        imgs[v] = img
        tri1, t1b = primary_hits(osc, ocam, w, pix, v)
        flip = (tri0 != tri1) | (t0b != t1b)
        rows[v] = dict(gap(ref, img, pix, flip, tri0 != tri1), seconds=round(time.time() - t0, 2))
        if flip.any():   # where the flipped camera rays are (image coordinates)
            fp = pix[flip]
            rows[v]["primary_flip_columns"] = sorted({int(p) % w for p in fp})[:16]
            rows[v]["primary_flip_examples"] = [[int(p) % w, int(p) // w, int(a), int(b)] for p, a, b in
                                                zip(fp[:8], tri0[flip][:8], tri1[flip][:8])]
        r = rows[v]
        print("%s %-9s rmse %.3e (%.3e without %d primary triangle changes, %.3e without %d primary t/triangle "
              "changes)  max %.3e  differing %d / %d pixels" % (
                  name, v, r["rmse_tonemapped"], r["rmse_tonemapped_no_primary_triangle_flips"], r["primary_triangle_flips"],
                  r["rmse_tonemapped_no_primary_flips"], r["primary_hit_flips"], r["max_abs_tonemapped"],
                  r["pixels_differing_fp32"], r["pixels"]), flush=True)
    # variant against variant (e.g. the two contraction shapes of triIntersect: how much the image depends on
    # WHICH product a compiler fuses, not only on whether it fuses)
    prow = {}
    for a, b in pairs:
        if a not in imgs or b not in imgs:
            continue
        ta, tab = primary_hits(osc, ocam, w, pix, a)
        tb, tbb = primary_hits(osc, ocam, w, pix, b)
        r = gap(imgs[a], imgs[b], pix, (ta != tb) | (tab != tbb), ta != tb)
        prow["%s:%s" % (a, b)] = r
        print("%s %s vs %s rmse %.3e (%.3e without %d primary triangle changes)  differing %d / %d pixels  "
              "bit-identical %s" % (name, a, b, r["rmse_tonemapped"], r["rmse_tonemapped_no_primary_triangle_flips"],
                                    r["primary_triangle_flips"], r["pixels_differing_fp32"], r["pixels"],
                                    bool(np.array_equal(imgs[a].reshape(-1, 3)[pix], imgs[b].reshape(-1, 3)[pix]))),
              flush=True)
    return {"workload": "%s %s %dx%d %dspp depth %d, every %d-th 8x8 tile (%d pixels)" % (
        name, cfg["scene"], w, h, spp, bounces, stride, len(pix)), "oracle_seconds": round(t_ref, 2), "variants": rows,
        "pairs": prow}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles-c2", type=int, default=1024)
    ap.add_argument("--tiles-c3", type=int, default=512)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--variants", default=",".join(oracle.VARIANTS))
    ap.add_argument("--workloads", default="C2,C3")
    ap.add_argument("--json", default=None)
    ap.add_argument("--pairs", default="", help="variant:variant,... compared with each other")
    ap.add_argument("--cache-dir", default=os.path.join(tempfile.gettempdir(), "pt_bench_scene"))
    args = ap.parse_args()
    os.makedirs(args.cache_dir, exist_ok=True)
    variants = [v for v in args.variants.split(",") if v]
    out = {"tool": "tools/parity/ref_gap.py", "threshold_north_star": 1e-4, "results": {}}
    for name in args.workloads.split(","):
        tiles = args.tiles_c2 if name == "C2" else args.tiles_c3
        pairs = [tuple(x.split(":")) for x in args.pairs.split(",") if x]
        out["results"][name] = run(name, tiles, args.threads, args.cache_dir, variants, pairs)
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(out, fh, indent=1)
    print(json.dumps({k: {v: r["rmse_tonemapped"] for v, r in res["variants"].items()}
                      for k, res in out["results"].items()}))


if __name__ == "__main__":
    main()
