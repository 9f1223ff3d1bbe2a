#!/usr/bin/env python3
"""Read the kernel trace of tools/gpu/overlap.py (rocprofv3 --kernel-trace csv): for every side kernel
(sleep / copy / elementwise) whether it ran beside a render frame's kernels (seeding pre-pass, render,
finalisation) and where: started before the next render's integration kernel and overlapped its start,
inside a running integration kernel, or in a gap between frames; and the integration kernel's durations
with and without a side kernel beside them."""
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows), key=lambda x: x[0])
renders = [(s, e) for s, e, n in ev if "render_unidir_wf" in n or "render_head_wf" in n]
frame_k = [(s, e) for s, e, n in ev if any(k in n for k in ("init_pixel_states", "finalize_pixels", "render_unidir_wf"))]
side = [(s, e, n) for s, e, n in ev if ("sleep" in n.lower() or "spin" in n.lower() or "copy" in n.lower()
                                       or "elementwise" in n.lower()) and "render" not in n]
res = []
cls = {"overlaps_render_start": 0, "inside_running_render": 0, "beside_prepass_only": 0, "alone": 0}
beside = set()
for s, e, n in side:
    inside = any(rs < s and e <= re_ for rs, re_ in renders)
    over_start = any(s <= rs < e for rs, re_ in renders)
    over_any = any(fs < e and s < fe for fs, fe in frame_k)
    c = ("inside_running_render" if inside else "overlaps_render_start" if over_start
         else "beside_prepass_only" if over_any else "alone")
    cls[c] += 1
    for i, (rs, re_) in enumerate(renders):
        if rs < e and s < re_:
            beside.add(i)
    res.append({"kernel": n[:40], "class": c, "us": round((e - s) / 1e3, 1)})
durs = [(e - s) / 1e6 for s, e in renders]
with_side = [d for i, d in enumerate(durs) if i in beside]
without = [d for i, d in enumerate(durs) if i not in beside]


def med(x):
    return round(sorted(x)[len(x) // 2], 3) if x else None


print(json.dumps({"side_kernels": len(side), "classes": cls,
                  "render_ms_median_with_side_kernel": med(with_side), "n_with": len(with_side),
                  "render_ms_median_without": med(without), "n_without": len(without),
                  "side_sample": res[:16]}, indent=1))
