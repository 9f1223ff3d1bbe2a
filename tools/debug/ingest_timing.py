"""Host ingest timings on the 262K stand-in: OBJ parse, reference BVH build, pt_create phases
(PT_TIMING=1 prints them).  Usage: PT_TIMING=1 python tools/debug/ingest_timing.py"""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import cudapathtracer_amd as pt  # noqa: E402
from cudapathtracer_amd import scenes  # noqa: E402

d = tempfile.mkdtemp()
p = scenes.write_sponza_standin(d)
for rep in range(2):
    t0 = time.perf_counter()
    s = pt.Scene()
    s.load_obj(p, mtl_basepath=os.path.dirname(p) + "/")
    t1 = time.perf_counter()
    s.build_bvh()
    t2 = time.perf_counter()
    print("OBJ parse %.1f ms, BVH.h build %.1f ms" % ((t1 - t0) * 1e3, (t2 - t1) * 1e3), flush=True)
if len(sys.argv) < 2 or sys.argv[1] != "--no-gpu":
    for rep in range(2):
        t0 = time.perf_counter()
        r = pt.Renderer(s, 0)
        print("pt_create total %.1f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
        r.close()
