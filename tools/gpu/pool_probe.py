#!/usr/bin/env python3
"""Walk-only probe (GPU box): how fast does the render-path walk trace C3-like rays when nothing but
the walk holds registers?  Traces one batch of bounce rays of the C3 stand-in (primary hits of random
pixels, then a cosine-distributed direction about the reversed ray, as tools/sim/wide_sim.cpp does)
with pt_trace's one-ray-per-lane kernel and with the persistent ray pool (PT_TRACE_POOL=6 / 8), checks
the three results are identical, and prints host wall times; run it under `rocprofv3 --kernel-trace
--stats` for the kernels' own durations.  A measurement aid for DESIGN.md §10, not part of the product:
the pool kernel was not kept, so PT_TRACE_POOL needs profiles/r03_pool/trace_pool.diff applied (without
it the three runs are the same kernel).

usage: python3 tools/gpu/pool_probe.py [n_rays]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import cudapathtracer_amd as pt  # noqa: E402
from cudapathtracer_amd import scenes  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8 << 20
    d = "/tmp/pool_probe_scene"
    path = scenes.write_sponza_standin(d)
    sc = pt.Scene()
    sc.load_obj(path, mtl_basepath=os.path.dirname(path) + "/")
    sc.build_bvh()
    r = pt.Renderer(sc, device=0)
    cam = pt.make_camera(width=1920, height=1080, **scenes.SPONZA_STANDIN_CAMERA)
    rng = np.random.default_rng(1234)
    npx = 1 << 18
    xs, ys = rng.integers(0, 1920, npx), rng.integers(0, 1080, npx)
    o = np.empty((npx, 3), np.float32)
    dd = np.empty((npx, 3), np.float32)
    for i in range(npx):
        ro, rd = pt.camera_ray(cam, pt.morton_pxl_to_i(int(xs[i]), int(ys[i])))
        o[i], dd[i] = ro, rd
    tri, t = r.trace(o, dd)
    hit = tri >= 0
    o, dd, t = o[hit], dd[hit], t[hit]
    p = o + dd * (t - 1e-3)[:, None]
    nrm = -dd
    reps = (n + len(p) - 1) // len(p)
    P = np.tile(p, (reps, 1))[:n]
    N = np.tile(nrm, (reps, 1))[:n]
    u1, u2 = rng.random(n, dtype=np.float32), rng.random(n, dtype=np.float32)
    tx = np.where(np.abs(N[:, :1]) > 0.1, np.array([[0, 1, 0]], np.float32), np.array([[1, 0, 0]], np.float32))
    t1 = np.cross(N, tx)
    t1 /= np.linalg.norm(t1, axis=1, keepdims=True)
    t2 = np.cross(N, t1)
    rr, th = np.sqrt(u1), np.float32(6.2831853) * u2
    z = np.sqrt(np.maximum(0, 1 - u1))
    D = (t1 * (rr * np.cos(th))[:, None] + t2 * (rr * np.sin(th))[:, None] + N * z[:, None]).astype(np.float32)
    out = {"rays": n}
    res = {}
    for mode in ("lanes", "6", "8"):
        if mode == "lanes":
            os.environ.pop("PT_TRACE_POOL", None)
        else:
            os.environ["PT_TRACE_POOL"] = mode
        r.trace(P[:4096], D[:4096])   # warm-up
        t0 = time.perf_counter()
        res[mode] = r.trace(P, D)
        out[f"wall_s_{mode}"] = round(time.perf_counter() - t0, 4)
    out["pool6_identical"] = bool(np.array_equal(res["6"][0], res["lanes"][0]) and
                                  np.array_equal(res["6"][1].view(np.uint32), res["lanes"][1].view(np.uint32)))
    out["pool8_identical"] = bool(np.array_equal(res["8"][0], res["lanes"][0]) and
                                  np.array_equal(res["8"][1].view(np.uint32), res["lanes"][1].view(np.uint32)))
    out["hit_frac"] = round(float((res["lanes"][0] >= 0).mean()), 4)
    print(json.dumps(out))
    r.close()
    sc.close()


if __name__ == "__main__":
    main()
