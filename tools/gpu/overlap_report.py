#!/usr/bin/env python3
"""Read the kernel trace of tools/gpu/overlap.py (rocprofv3 --kernel-trace csv): for every side kernel
(sleep / copy) the render kernel running when it started, whether it ended inside that render's span, and
the render durations with and without a side kernel beside them."""
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows), key=lambda x: x[0])
renders = [(s, e) for s, e, n in ev if "render_unidir_wf" in n]
side = [(s, e, n) for s, e, n in ev if ("sleep" in n.lower() or "copy" in n.lower() or "elementwise" in n.lower())
        and "render" not in n]
inside = 0
res = []
for s, e, n in side:
    host = [(rs, re_) for rs, re_ in renders if rs <= s < re_]
    ok = bool(host) and e <= host[0][1]
    inside += ok
    res.append({"kernel": n[:60], "start_in_render": bool(host), "ended_in_render": ok, "us": round((e - s) / 1e3, 1),
                "render_left_at_start_us": round((host[0][1] - s) / 1e3, 1) if host else None})
durs = [round((e - s) / 1e6, 3) for s, e in renders]
print(json.dumps({"side_kernels": len(side), "side_inside_a_render": inside, "render_ms": durs, "side": res[:12]}, indent=1))
