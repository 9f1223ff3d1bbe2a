#!/usr/bin/env python3
"""Aggregate the whole-frame oracle parity logs (tests/test_gpu_fullframe_oracle.py result lines) under
profiles/r06_fullframe into summary.txt: per config, the rows covered, samples compared and differing values."""
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
d = os.path.join(ROOT, "profiles", "r06_fullframe")
res = {}
for p in sorted(glob.glob(os.path.join(d, "log*.txt"))):
    for line in open(p):
        line = line.strip()
        if not line.startswith("{"):
            continue
        r = json.loads(line)
        rows = tuple(r.get("rows", [0, r["height"]]))
        res[(r["config"], rows)] = r
by = {}
for (cfg, rows), r in sorted(res.items()):
    b = by.setdefault(cfg, dict(rows=0, height=r["height"], samples=0, diff=0, bands=[]))
    b["rows"] += rows[1] - rows[0]
    b["samples"] += r["samples"]
    b["diff"] += r["differing_values"]
    b["bands"].append(list(rows))
lines = ["config  rows covered      samples compared  differing values  bands"]
tot = 0
for cfg, b in by.items():
    tot += b["samples"]
    lines.append("%-6s  %5d of %-5d  %16d  %16d  %s" % (cfg, b["rows"], b["height"], b["samples"], b["diff"], b["bands"]))
lines.append("total samples compared: %d (%.2f G)" % (tot, tot / 1e9))
open(os.path.join(d, "summary.txt"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
