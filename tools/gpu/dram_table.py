"""Summarise a tools/gpu/dram_calib.sh run: per dispatch of the calibration probe and
of the render launch, the L2's memory-side read/write requests (TCC_EA0_RDREQ / WRREQ), the part of them
addressed to DRAM (TCC_EA0_RDREQ_DRAM / WRREQ_DRAM), FETCH_SIZE / WRITE_SIZE and the L2 hit rate.

usage: python tools/gpu/dram_table.py gpurun_out/<tag> [> profiles/<dir>/dram_table.txt]"""
import collections
import csv
import glob
import json
import os
import sys


def kname(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def load(d, kind):
    vals = collections.defaultdict(dict)   # (dispatch, kernel) -> counter -> value
    durs = {}
    for p in sorted(glob.glob(os.path.join(d, "%s_p*" % kind, "run_counter_collection.csv"))):
        for r in csv.DictReader(open(p)):
            k = (int(r["Dispatch_Id"]), kname(r["Kernel_Name"]))
            vals[k][r["Counter_Name"]] = vals[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        t = p.replace("counter_collection", "kernel_trace")
        for r in csv.DictReader(open(t)):
            k = (int(r["Dispatch_Id"]), kname(r["Kernel_Name"]))
            durs.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return vals, durs


def main():
    d = sys.argv[1]
    out = {}
    for kind in ("calib", "bench"):
        vals, durs = load(d, kind)
        print("== %s" % kind)
        print("%-4s %-24s %9s %13s %13s %6s %13s %13s %11s %11s %6s" % (
            "disp", "kernel", "ms", "RDREQ", "RDREQ_DRAM", "DRAM%", "WRREQ", "WRREQ_DRAM", "FETCH GB*2", "WRITE GB", "L2hit"))
        for k in sorted(vals):
            if kind == "bench" and "render" not in k[1]:
                continue
            v = vals[k]
            rd, rdd = v.get("TCC_EA0_RDREQ_sum", 0), v.get("TCC_EA0_RDREQ_DRAM_sum", 0)
            wr, wrd = v.get("TCC_EA0_WRREQ_sum", 0), v.get("TCC_EA0_WRREQ_DRAM_sum", 0)
            h, m = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0)
            ms = sorted(durs.get(k, [0]))[len(durs.get(k, [0])) // 2]
            print("%-4d %-24s %9.3f %13.0f %13.0f %6.1f %13.0f %13.0f %11.3f %11.3f %6.3f" % (
                k[0], k[1][:24], ms, rd, rdd, 100.0 * rdd / rd if rd else 0.0, wr, wrd,
                v.get("FETCH_SIZE", 0) * 1024 * 2 / 1e9, v.get("WRITE_SIZE", 0) * 1024 / 1e9, h / (h + m) if h + m else 0))
            out["%s:%d:%s" % (kind, k[0], k[1])] = dict(v, ms=ms)
    known = os.path.join(d, "known.txt")
    if os.path.exists(known):
        print("== known byte counts (probe stdout)")
        print(open(known).read().rstrip())
    json.dump(out, open(os.path.join(d, "dram_table.json"), "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
