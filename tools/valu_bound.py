#!/usr/bin/env python3
"""How much of the integrator-0 render kernel's time is VALU issue: its dynamic VALU count priced at the
rate its own instruction streams issue at when replayed alone (no memory, SALU or branches).

Inputs (all committed):
  profiles/r06_valu/walk_replay.txt   tools/gpu/micro/walk_replay at 1-5 waves per SIMD: one walk wave-step
                                      (the common path, WALK_STEP_VALU instructions) and the static code of
                                      three shading sections (sampling block, sample end, trace begin)
  profiles/r06_sections/C3.txt        section execution counts of a C3 frame (counting variant) and the
                                      walk's wave-steps
  a pmc_summary.json with SQ_INSTS_VALU (default: profiles/r06_final, the C3 bench launch)

Walk VALU = wave-steps x the replayed step's VALU; the rest of SQ_INSTS_VALU is priced at the three
sections' replay rates weighted by (static VALU x executions).  The result is the VALU issue time of one
launch at 5 waves per SIMD (the kernel's occupancy) and its fraction of the measured kernel time.

usage: tools/valu_bound.py [PMC_SUMMARY_JSON] [--json OUT]
"""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 1024            # 256 CUs x 4
REPLAY_CLOCK = 2.4e9    # walk_replay converts its event times to cycles at this clock; undone below
# static VALU per execution of the replayed shading sections (the PT_SEC_MARKERS listing, profiles/r06_sections)
STATIC = {"cosine": 428, "sample_end": 213, "begin": 852}
SEC_ORDER = ["PASS", "CHECK", "SLOW", "BOUNCE", "EMIT", "COSINE", "LIGHT", "SAMPLE_END", "START", "CAMERA", "DEAD",
             "BEGIN", "REFILL", "MEMO", "RECORD", "PROBE"]


def replay_rates(path):
    """{stream: (valu per replay, seconds per VALU per SIMD at 5 waves/SIMD)}"""
    out = {}
    for line in open(path):
        m = re.match(r"(\S+)\s+VALU\s+(\d+)\s+waves/SIMD\s+5\s+\S+ ms\s+\S+ SIMD-cycles per replay @2.4 GHz\s+(\S+) per VALU",
                     line)
        if m:
            out[m.group(1)] = (int(m.group(2)), float(m.group(3)) / REPLAY_CLOCK)
    return out


def section_counts(path):
    toks = open(path).readline().split()
    assert toks[0] == "sections"
    return dict(zip(SEC_ORDER, (int(x) for x in toks[1:])))


def walk_steps(path):
    for line in open(path):
        m = re.search(r"walk: wave-steps C2 \d+, C3 (\d+)", line)
        if m:
            return int(m.group(1))
    raise SystemExit("no C3 wave-step count in " + path)


def bound(pmc_path):
    rates = replay_rates(os.path.join(ROOT, "profiles/r06_valu/walk_replay.txt"))
    secs = section_counts(os.path.join(ROOT, "profiles/r06_sections/C3.txt"))
    steps = walk_steps(os.path.join(ROOT, "profiles/r06_sections/table.txt"))
    p = json.load(open(pmc_path))
    c = p["counters_per_launch"]
    durs = sorted(p["kernel_trace_durations_ns"])
    kernel_s = durs[len(durs) // 2] * 1e-9
    valu = c["SQ_INSTS_VALU"]
    step_valu, s_walk = rates["walk_step"]
    walk_valu = steps * step_valu
    wsum = tsum = 0.0
    for name, key in (("cosine", "COSINE"), ("sample_end", "SAMPLE_END"), ("begin", "BEGIN")):
        w = STATIC[name] * secs[key]
        wsum += w
        tsum += w * rates[name][1]
    s_shade = tsum / wsum
    shade_valu = valu - walk_valu
    t_walk = walk_valu / SIMDS * s_walk
    t_shade = shade_valu / SIMDS * s_shade
    return {
        "kernel": "render_unidir_wf<false, 5, false>",
        "pmc": os.path.relpath(pmc_path, ROOT),
        "kernel_ms": round(kernel_s * 1e3, 3),
        "valu_per_launch": int(valu),
        "walk_wave_steps": steps,
        "walk_valu_per_step_replayed": step_valu,
        "walk_valu": int(walk_valu),
        "shading_valu": int(shade_valu),
        "cycles_per_valu_walk_replay": round(s_walk * REPLAY_CLOCK, 3),
        "cycles_per_valu_shading_replay": round(s_shade * REPLAY_CLOCK, 3),
        "valu_issue_ms_walk": round(t_walk * 1e3, 3),
        "valu_issue_ms_shading": round(t_shade * 1e3, 3),
        "valu_issue_ms": round((t_walk + t_shade) * 1e3, 3),
        "valu_issue_frac": round((t_walk + t_shade) / kernel_s, 4),
        # the blended rate, for pricing other launches of the same kernel (tools/update_traffic.py)
        "cycles_per_valu_blend": round((t_walk + t_shade) * REPLAY_CLOCK / (valu / SIMDS), 4),
        "method": "SQ_INSTS_VALU of one launch priced at the replay rate (5 waves/SIMD, no memory) of the kernel's own "
                  "streams: the walk wave-step for wave-steps x its VALU, the shading sections (weighted by static VALU "
                  "x executions) for the rest; tools/valu_bound.py, profiles/r06_valu",
    }


if __name__ == "__main__":
    argv = sys.argv[1:]
    out = None
    if "--json" in argv:
        k = argv.index("--json")
        out = argv[k + 1]
        del argv[k:k + 2]
    pmc = argv[0] if argv else os.path.join(ROOT, "profiles/r06_final/pmc_summary.json")
    r = bound(pmc)
    print(json.dumps(r, indent=1))
    if out:
        json.dump(r, open(out, "w"), indent=1)
