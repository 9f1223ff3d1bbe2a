#!/usr/bin/env python3
"""Pool-mode (PT_WF_POOL) debugging: render the same frame with the pool on and off (separate processes: the mode is
read at pt_create) and report where they differ.  usage: pool_debug.py out_dir"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
out = sys.argv[1]
os.makedirs(out, exist_ok=True)
CHILD = r'''
import os, sys, numpy as np
sys.path.insert(0, %r); sys.path.insert(0, os.path.join(%r, "tests"))
import cudapathtracer_amd as pt
from conftest import load_scene
s = load_scene(sys.argv[1])
w, h, spp, b = [int(x) for x in sys.argv[2:6]]
cam = pt.make_camera((0.0, 1.0, 3.0), 1.0, 3.0, 0.0, w, h)
with pt.Renderer(s, 0) as r:
    img, st = r.render(cam, w, h, spp, bounces=b, flags=int(sys.argv[7]))
np.save(sys.argv[6], img)
print(st)
''' % (ROOT, ROOT)
MODES = os.environ.get("MODES", "PT_WF_POOL=1").split()
for scene, w, h, spp, b in [("cornell_blob", 24, 16, 3, 3), ("cornell_blob", 64, 64, 4, 3)]:
  for mode in MODES:
    for flags in (6,):   # 2 no dead-path skip (no light probe), 4 no primary memo
        imgs = {}
        for env in ("0", "1"):
            f = os.path.join(out, "%s_%d_%d_%d_%d_f%d_pool%s.npy" % (scene, w, h, spp, b, flags, env))
            e = dict(os.environ, PT_WF_POOL="0")
            if env == "1":
                e.update(dict(kv.split("=") for kv in mode.split(",")))
            r = subprocess.run([sys.executable, "-c", CHILD, scene, str(w), str(h), str(spp), str(b), f, str(flags)],
                               env=e, capture_output=True, text=True, timeout=120)
            if r.returncode != 0:
                print("child failed", env, r.stderr[-2000:])
                sys.exit(1)
            imgs[env] = np.load(f)
            dbg = [ln for ln in r.stdout.splitlines() if ln.startswith("pool:")]
            if dbg:
                print("   %d debug lines, first: %s" % (len(dbg), dbg[:5]))
        a, p = imgs["0"], imgs["1"]
        d = np.any(a.view(np.uint32) != p.view(np.uint32), axis=2)
        ys, xs = np.nonzero(d)
        print("%s %s %dx%d spp %d b %d flags %d: %d of %d pixels differ; first %s" % (
            mode, scene, w, h, spp, b, flags, int(d.sum()), d.size, list(zip(xs[:8].tolist(), ys[:8].tolist()))))
        for x, y in list(zip(xs, ys))[:4]:
            print("   px (%d,%d) off %s pool %s" % (x, y, a[y, x].tolist(), p[y, x].tolist()))
