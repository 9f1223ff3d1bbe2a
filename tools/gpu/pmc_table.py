#!/usr/bin/env python3
"""Table of render-kernel PMC counters per variant from a tools/gpu/r04_pmc_rejected.sh output dir.

usage: tools/gpu/pmc_table.py gpurun_out/<tag> > profiles/<tag>/pmc_table.txt
Each variant dir holds one --pmc pass per counter group (pmc_<group>/run_counter_collection.csv);
counters are summed over the render kernel's dispatch, durations are the render kernel's trace spans.
"""
import collections
import csv
import json
import os
import sys

src = sys.argv[1]
rows = {}
for v in sorted(os.listdir(src)):
    d = os.path.join(src, v)
    if not os.path.isdir(d):
        continue
    agg, durs = collections.defaultdict(float), []
    for g in sorted(os.listdir(d)):
        cc = os.path.join(d, g, "run_counter_collection.csv")
        if not g.startswith("pmc_") or not os.path.exists(cc):
            continue
        for r in csv.DictReader(open(cc)):
            if "render" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
        kt = os.path.join(d, g, "run_kernel_trace.csv")
        if os.path.exists(kt):
            durs += [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                     for r in csv.DictReader(open(kt)) if "render" in r["Kernel_Name"]]
    cyc = agg.get("GRBM_GUI_ACTIVE", 0.0) / 8.0   # summed over the 8 XCDs
    durs.sort()
    out = {"kernel_ms_median": durs[len(durs) // 2] / 1e6 if durs else None}
    if cyc:
        out["td_busy"] = agg.get("TD_TD_BUSY_sum", 0) / 256 / cyc
        out["td_tc_stall"] = agg.get("TD_TC_STALL_sum", 0) / 256 / cyc
        out["ta_busy"] = agg.get("TA_TA_BUSY_sum", 0) / 256 / cyc
        out["valu_per_simd_cycle"] = agg.get("SQ_INSTS_VALU", 0) / 1024 / cyc
        out["l1_lookups_per_cu_cycle"] = agg.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0) / 256 / cyc
        out["ta_stalled_by_tc"] = agg.get("TA_ADDR_STALLED_BY_TC_CYCLES_sum", 0) / 256 / cyc
    hits, misses = agg.get("TCC_HIT_sum", 0.0), agg.get("TCC_MISS_sum", 0.0)
    if hits + misses:
        out["l2_hit_rate"] = hits / (hits + misses)
        out["l2_requests_G"] = (hits + misses) / 1e9
    out["l1_lookups_G"] = agg.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0) / 1e9
    out["valu_G"] = agg.get("SQ_INSTS_VALU", 0) / 1e9
    out["fetch_GB_x2"] = agg.get("FETCH_SIZE", 0) * 1024 * 2 / 1e9
    out["write_GB"] = agg.get("WRITE_SIZE", 0) * 1024 / 1e9
    out["cycles_M"] = cyc / 1e6
    rows[v] = out
for v, o in rows.items():
    print(v, " ".join(f"{k} {x:.4g}" if isinstance(x, float) else f"{k} {x}" for k, x in o.items()))
print(json.dumps(rows))
