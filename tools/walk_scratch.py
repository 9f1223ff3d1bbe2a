#!/usr/bin/env python3
"""Scratch (spill) instructions inside the walk phase of each wavefront kernel in the ISA listing
(cudapathtracer_amd/csrc/build/pt_render.s, `make -C cudapathtracer_amd/csrc asm`): the walk phase
runs between `s_setprio 1` and the next `s_setprio 0` (wf_main).  A spill there costs every walk step."""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "cudapathtracer_amd/csrc/build/pt_render.s"
s = open(path).read()
for m in re.finditer(r"^(_Z\S*render_(?:unidir|head)_wf\S*):", s, re.M):
    i = m.end()
    j = s.index(".Lfunc_end", i)
    b = s[i:j].split("\n")
    p1 = [k for k, l in enumerate(b) if "s_setprio 1" in l]
    p0 = [k for k, l in enumerate(b) if "s_setprio 0" in l]
    walk = 0
    for a in p1:
        z = [x for x in p0 if x > a]
        if z:
            walk += sum(1 for l in b[a:z[0]] if "scratch_" in l)
    print("%-60s lines %6d  scratch in walk %4d  total scratch %4d" % (m.group(1)[:60], len(b), walk,
                                                                          sum(1 for l in b if "scratch_" in l)))
