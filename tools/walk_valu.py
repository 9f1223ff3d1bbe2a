#!/usr/bin/env python3
"""Static instruction counts of the wavefront kernel's walk loop (the first depth-2 loop of
render_unidir_wf<false,5>) in build/pt_render.s (`make -C cudapathtracer_amd/csrc asm`)."""
import collections
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "cudapathtracer_amd/csrc/build/pt_render.s"
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_ZN12_GLOBAL__N_116render_unidir_wfILb0ELi5E(Lb0E)?EEvNS_4ArgsE:", l))
lines = lines[start:]
h = next(i for i, l in enumerate(lines) if "This Loop Header: Depth=2" in l)
hdr = re.search(r"^(\.LBB\d+_\d+):", lines[h - 1] if lines[h - 1].startswith(".LBB") else lines[h]).group(1) \
    if re.search(r"^(\.LBB\d+_\d+):", lines[h - 1] if lines[h - 1].startswith(".LBB") else lines[h]) else None
# the loop spans the blocks annotated "in Loop: Header=<hdr> Depth=2" (and deeper) after the header
name = hdr[1:].replace("LBB", "BB")
cnt = collections.Counter()
inloop = False
for l in lines[h - 1:]:
    m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):\s*;(.*)", l)
    if m:
        ann = m.group(2)
        inloop = ("Header=%s " % name) in ann or ("Parent Loop %s" % name) in ann or "This Loop Header: Depth=2" in ann \
            or "Depth=3" in ann
        if not inloop and cnt["v"] > 0 and "Depth=1" in ann:
            break
        continue
    if not inloop:
        continue
    s = l.strip()
    if s.startswith("v_"):
        cnt["v"] += 1
    elif s.startswith("s_"):
        cnt["s"] += 1
    elif s.startswith(("global_", "buffer_")):
        cnt["vmem"] += 1
    elif s.startswith("ds_"):
        cnt["ds"] += 1
print("walk loop %s: VALU %d  SALU %d  VMEM %d  DS %d" % (name, cnt["v"], cnt["s"], cnt["vmem"], cnt["ds"]))
