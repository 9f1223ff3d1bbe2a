#!/usr/bin/env python3
"""profiles/traffic.json from a profile's pmc_summary.json (tools/summarize_profile.py output).

traffic = FETCH_SIZE x 2 + WRITE_SIZE per launch of the render kernel, in bytes: rocprofv3 reports
both in KB; the x2 is the gfx950 correction of MI355X_MICROARCH.md, calibrated on this kernel's own
access shapes (node / triangle gathers, lane-major record cells: profiles/r02_fetch_calibration).
The file is stamped with the render kernel's source hash (bench.kernel_source_sha256) and the bench
config, so bench.py uses it only for the kernel and workload it was measured on.

usage: tools/update_traffic.py profiles/<tag> [W H SPP BOUNCES INTEGRATOR SHARDS]
(entries of other configs are kept; the entry of this config is replaced)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

prof = sys.argv[1]
cfg = [int(x) for x in sys.argv[2:8]] if len(sys.argv) >= 8 else [1920, 1080, 256, 3, 0, 1]
p = json.load(open(os.path.join(prof, "pmc_summary.json")))
c = p["counters_per_launch"]
durs = sorted(p["kernel_trace_durations_ns"])
kms = durs[len(durs) // 2] / 1e6 if durs else None
out = {
    "config": cfg,
    "kernel": p["kernels"][0] if p["kernels"] else "render_unidir_wf",
    "kernel_source_sha256": bench.kernel_source_sha256(),
    "profile": os.path.relpath(prof, ROOT),
    "kernel_ms": kms,
    "fetch_size_kb": c["FETCH_SIZE"],
    "write_size_kb": c["WRITE_SIZE"],
    "traffic_bytes_per_launch": int(c["FETCH_SIZE"] * 1024 * 2 + c["WRITE_SIZE"] * 1024),
    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (one launch each): "
              "FETCH_SIZE x1024 x2 + WRITE_SIZE x1024 (x2 calibrated on the kernel's gather shapes, "
              "profiles/r02_fetch_calibration)",
}
if "GRBM_GUI_ACTIVE" in c:
    cyc = c["GRBM_GUI_ACTIVE"] / 8.0     # summed over the 8 XCDs
    if cfg[:4] == [1024, 1024, 64, 8]:   # C2: the 32-triangle Cornell tree, held whole in LDS
        lim = ("C2's tree (32 triangles) is read from LDS and every other record hits L2: not bytes -- the path "
               "state held in registers removed 37-42% of the memory-side bytes for -0.8% (profiles/r04_c2_regstate); "
               "the walk (56% of the wave-clock, SIMD utilisation ~0.39 at walk threshold 62) is bound by the VALU it "
               "issues, not by its phase structure or LDS round trips -- an exhaustive LDS trace with no walk phase and "
               "12x the triangle tests lost 20% (profiles/r06_exhaustive); the f64 shading pass (44%) spreads over "
               "sampling, sample ends, trace begins and dead-path replays with none dominant (profiles/r06_sections); "
               "VALU issue 0.276 per SIMD-cycle, the rate at which integrator 0's replayed streams fill every issue "
               "cycle (DESIGN.md 6.3; C2's own LDS-walk stream is not replayed)")
    else:
        lim = ("the walk's steps per ray times the VALU each step issues (~160 per wave-step, the wave paying all 64 "
               "lanes' slots): fewer steps per ray paid every time (margin test, leaves of 2, light probe, DP collapse, "
               "DESIGN_LOG 6); removing vector-memory loads from the step did not (round 6: 1 and 2 of 10 loads removed "
               "with +3.7% and +12% dynamic VALU -> -3.9% and -7.0%, cycles following the VALU at an unchanged issue "
               "rate, profiles/r06_fold, r06_qnode), nor did fewer L1 lookups (-18..-37%: +-0 or worse), fewer memory-"
               "side bytes (-11.5%: +0.3%) or a sixth wave; TD busy ~0.99 counts requests in flight; VALU issue "
               "~0.26 per SIMD-cycle, at which integrator 0's replayed streams fill every issue cycle (DESIGN.md 6.3)")
    # limiter: the binding resource as one key (bench.py's roofline.bound); limiter_detail: the evidence
    kind = "lds_walk_and_f64_shading_issue" if cfg[:4] == [1024, 1024, 64, 8] else "walk_steps_x_step_valu"
    # the integrator-0 kernel on the stand-in: its VALU priced at the rate its own streams issue at alone
    # (profiles/r06_valu, tools/valu_bound.py) -- the VALU issue time of the launch against its duration
    vb_path = os.path.join(ROOT, "profiles", "r06_valu", "valu_bound.json")
    vb = json.load(open(vb_path)) if os.path.exists(vb_path) else None
    priced = (vb is not None and "SQ_INSTS_VALU" in c and kind == "walk_steps_x_step_valu"
              and "render_unidir_wf<false, 5, false>" in out["kernel"])
    if priced:
        kind = "valu_issue"
        lim = ("VALU issue: the launch's VALU instructions, priced at the rate the kernel's own instruction streams "
               "issue at when replayed alone with no memory at 5 waves per SIMD (walk step %.2f, shading %.2f SIMD-"
               "cycles per instruction; profiles/r06_valu, tools/valu_bound.py), take %s of its time -- the SIMDs "
               "issue VALU in nearly every cycle and memory latency is hidden. Consistent with every round-6 "
               "experiment: removing 1-2 of the step's 10 loads at +3.7%%/+12%% VALU lost 3.9%%/7.0%% (r06_fold, "
               "r06_qnode); fewer L1 lookups or memory-side bytes bought nothing; fewer walk steps per ray always paid"
               % (vb["cycles_per_valu_walk_replay"], vb["cycles_per_valu_shading_replay"], "%.0f%%"))
    b = {"limiter": kind, "limiter_detail": lim, "cycles_per_launch": int(cyc)}
    if priced:
        issue_ms = c["SQ_INSTS_VALU"] / 1024 * vb["cycles_per_valu_blend"] / 2.4e9 * 1e3
        b["valu_issue_ms_per_launch"] = round(issue_ms, 3)
        b["valu_issue_frac_profiled"] = round(issue_ms / kms, 4) if kms else None
        b["valu_issue_method"] = ("SQ_INSTS_VALU / 1024 SIMDs x %.4f SIMD-cycles per instruction (the walk / shading blend "
                                  "of the replayed streams, weighted as in the C3 launch) at 2.4 GHz" % vb["cycles_per_valu_blend"])
        b["limiter_detail"] = lim.replace("%.0f%%", "%.0f%%" % (100 * issue_ms / kms) if kms else "most")
    if "SQ_INSTS_VALU" in c:
        # wave64 VALU instructions per SIMD-cycle; measured ceiling ~0.25-0.3 for this kernel's mix (most
        # classes take 3.9-4.7 SIMD-cycles at >= 2 waves per SIMD, moves 2.3: profiles/r06_valu/valu_cost.txt)
        b["valu_insts_per_simd_cycle"] = round(c["SQ_INSTS_VALU"] / (1024 * cyc), 4)
    if "TD_TD_BUSY_sum" in c:
        b["td_busy"] = round(c["TD_TD_BUSY_sum"] / 256 / cyc, 4)
    if "TA_TA_BUSY_sum" in c:
        b["ta_busy"] = round(c["TA_TA_BUSY_sum"] / 256 / cyc, 4)
    if "TD_TC_STALL_sum" in c:
        b["td_tc_stall"] = round(c["TD_TC_STALL_sum"] / 256 / cyc, 4)
    if "TCP_TOTAL_CACHE_ACCESSES_sum" in c:   # L1 tag lookups (a scattered dwordx4: one per lane)
        b["l1_lookups_per_cu_cycle"] = round(c["TCP_TOTAL_CACHE_ACCESSES_sum"] / 256 / cyc, 4)
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        b["l2_hit_rate"] = round(c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1), 4)
    out["binding"] = b
if "TCC_EA0_RDREQ_DRAM_sum" in c:
    # the DRAM-request counters (profiles/r05_dram: they equal the memory-side request counters on an
    # Infinity-Cache-resident table, i.e. they count Infinity-Cache hits -- not an HBM measurement)
    out["dram_requests"] = {"rdreq": int(c.get("TCC_EA0_RDREQ_sum", 0)), "rdreq_dram": int(c["TCC_EA0_RDREQ_DRAM_sum"]),
                            "wrreq": int(c.get("TCC_EA0_WRREQ_sum", 0)), "wrreq_dram": int(c.get("TCC_EA0_WRREQ_DRAM_sum", 0))}
# one entry per (config, source hash): a new measurement replaces the entry of its config
path = os.path.join(ROOT, "profiles", "traffic.json")
try:
    tj = json.load(open(path))
except (OSError, ValueError):
    tj = {}
entries = [e for e in tj.get("entries", []) if e.get("config") != cfg]
entries.append(out)
json.dump({"entries": entries}, open(path, "w"), indent=1)
print(json.dumps(out, indent=1))
