#!/usr/bin/env python3
"""Summarize a tools/gpu/profile.sh output dir into profiles/<name>/ (kernel stats + PMC JSON)."""
import collections, csv, json, os, shutil, sys

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "ktrace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
shutil.copy(os.path.join(src, "bench_ktrace.json"), os.path.join(dst, "bench_ktrace.json"))
out, kernels = {}, set()
for d in sorted(os.listdir(src)):
    if not d.startswith("pmc_"):
        continue
    rows = list(csv.DictReader(open(os.path.join(src, d, "run_counter_collection.csv"))))
    agg = collections.defaultdict(float)
    for r in rows:
        if "render" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            kernels.add(r["Kernel_Name"])
    out.update(agg)
kt = list(csv.DictReader(open(os.path.join(src, "ktrace", "run_kernel_trace.csv"))))
durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in kt if "render" in r["Kernel_Name"]]
json.dump({"kernels": sorted(kernels), "counters_per_launch": out,
           "kernel_trace_durations_ns": durs,
           "note": "FETCH_SIZE/WRITE_SIZE in KB as rocprofv3 reports them (gfx950: FETCH_SIZE may read ~1/2 of "
                   "wide streaming reads); each counter group from its own --pmc pass of one launch"},
          open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
