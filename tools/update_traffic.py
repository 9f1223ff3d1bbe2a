#!/usr/bin/env python3
"""profiles/traffic.json from a profile's pmc_summary.json: HBM-side bytes per launch of the render
kernel (FETCH_SIZE x2 per the gfx950 correction of MI355X_MICROARCH.md + WRITE_SIZE), which bench.py
reports as roofline.traffic when its config and accel tag match."""
import json
import sys

src, accel = sys.argv[1], sys.argv[2]
p = json.load(open(src))
c = p["counters_per_launch"]
out = {
    "config": [1920, 1080, 256, 3, 0, 1],
    "accel": accel,
    "kernel": p["kernels"][0] if p["kernels"] else "render_unidir_wf",
    "fetch_size_kb": c["FETCH_SIZE"],
    "write_size_kb": c["WRITE_SIZE"],
    "hbm_bytes_per_launch": int(c["FETCH_SIZE"] * 1024 * 2 + c["WRITE_SIZE"] * 1024),
    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (one launch each); FETCH_SIZE "
              "x1024 (KB->B) x2 (gfx950 reports 1/2 of wide reads, MI355X_MICROARCH.md HBM) + WRITE_SIZE x1024",
    "source": src,
}
json.dump(out, open("profiles/traffic.json", "w"), indent=1)
print(json.dumps(out, indent=1))
