"""bench.py's roofline blocks on CPU: every field means what its block says.

The HBM `roofline` takes its measured traffic only from the profiles/traffic.json entry of this exact
kernel source hash and config; the algorithmic bytes live in `cache_roofline` (L2 roof) and the L1
lookup rate in `l1_roofline`, marked as not the binding resource.  No field exceeds its own peak.
"""
import json
import os
import types

import bench


COUNTS = dict(node_tests=6_621_908_388, lds_node_tests=0, tri_tests=1_917_249_061, walk_lane_slots=10_493_000_000,
              leaf_steps=1_917_249_061, accel_fallbacks=195, spill_entries=0, walk_cycles=758, shade_cycles=242,
              shade_lane_slots=646_000_000, samples=1920 * 1080 * 256, rays_traced=507_000_000)


def _args(tmp_json, **kw):
    a = dict(flags=0, integrator=0, spp=256, bounces=3, sim_shards=1, traffic_json=tmp_json)
    a.update(kw)
    return types.SimpleNamespace(**a)


def test_traffic_entry_matches_hash_and_config(tmp_path):
    sha = bench.kernel_source_sha256()
    p = tmp_path / "t.json"
    e = {"config": [1920, 1080, 256, 3, 0, 1], "kernel_source_sha256": sha, "traffic_bytes_per_launch": 4e11,
         "kernel_ms": 91.0, "profile": "profiles/x", "binding": {"l1_lookups_per_cu_cycle": 0.8}}
    p.write_text(json.dumps({"entries": [e, dict(e, config=[1024, 1024, 64, 8, 0, 1], traffic_bytes_per_launch=3e10)]}))
    assert bench.traffic_entry(str(p), [1920, 1080, 256, 3, 0, 1], sha)["traffic_bytes_per_launch"] == 4e11
    assert bench.traffic_entry(str(p), [1920, 1080, 256, 3, 0, 2], sha) is None      # another shard count
    assert bench.traffic_entry(str(p), [1920, 1080, 256, 3, 0, 1], "0" * 64) is None  # another kernel
    assert bench.traffic_entry(str(tmp_path / "missing.json"), [1], sha) is None


def test_roofline_fields_stay_below_their_peaks(tmp_path):
    sha = bench.kernel_source_sha256()
    p = tmp_path / "t.json"
    p.write_text(json.dumps({"entries": [{"config": [1920, 1080, 256, 3, 0, 1], "kernel_source_sha256": sha,
                                          "traffic_bytes_per_launch": 397_000_000_000, "kernel_ms": 91.6,
                                          "profile": "profiles/x", "binding": {"l1_lookups_per_cu_cycle": 0.803}}]}))
    kms = 90.3
    roof = bench.roofline(COUNTS, kms, 1920, 1080, _args(str(p)), 1)
    assert roof["bound"] == "hbm" and roof["unit"] == "GB/s"
    assert abs(roof["achieved"] - 397e9 / (kms * 1e-3) / 1e9) < 0.01
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-4
    assert roof["achieved"] <= roof["peak"]
    assert not any(k.startswith("algorithmic") for k in roof)   # algorithmic bytes are not HBM bytes
    l1 = bench.l1_roofline(roof)
    assert l1["binding"] is False and l1["achieved"] <= l1["peak"] and l1["frac"] == 0.803
    cache = bench.cache_roofline(dict(COUNTS, spp=256), kms)
    assert cache["bound"] == "l2" and cache["achieved"] <= cache["peak"]
    alg = (COUNTS["node_tests"] * bench.NODE_BYTES + COUNTS["tri_tests"] * bench.TRI_BYTES
           + COUNTS["rays_traced"] * 64 + 1920 * 1080 * 12)
    assert abs(cache["algorithmic_bytes_per_launch"] - alg) <= 1


def test_roofline_is_null_without_a_matching_profile(tmp_path):
    roof = bench.roofline(COUNTS, 90.0, 1920, 1080, _args(str(tmp_path / "none.json")), 1)
    assert roof["frac"] is None and roof["traffic"] is None and roof["achieved"] is None
    assert bench.l1_roofline(roof) is None


def test_committed_traffic_json_covers_the_bench_configs():
    """profiles/traffic.json holds entries of the committed kernel for the default bench line (C3),
    the other BASELINE configs and the shard launches of N = 2, 4, 8."""
    path = os.path.join(bench.ROOT, "profiles", "traffic.json")
    sha = bench.kernel_source_sha256()
    for cfg in ([1920, 1080, 256, 3, 0, 1], [1024, 1024, 64, 8, 0, 1], [1920, 1080, 1024, 3, 0, 1],
                [3840, 2160, 4096, 16, 0, 1], [1920, 1080, 256, 3, 1, 1], [1920, 1080, 256, 3, 0, 2],
                [1920, 1080, 256, 3, 0, 4], [1920, 1080, 256, 3, 0, 8]):
        e = bench.traffic_entry(path, cfg, sha)
        assert e is not None, cfg
        assert e["traffic_bytes_per_launch"] / (e["kernel_ms"] * 1e-3) / 1e9 <= bench.HBM_PEAK_GBS


def test_hbm_counter_block_states_it_cannot_separate_infinity_cache_hits(tmp_path):
    """with the DRAM-request counters recorded for the launch, the roofline carries them
    beside the memory-side frac -- and says what the calibration (profiles/r05_dram) showed: they count the
    Infinity Cache's hits too, so no HBM-only bytes or frac are claimed."""
    sha = bench.kernel_source_sha256()
    p = tmp_path / "t.json"
    dr = {"rdreq": 2_097_356_374, "rdreq_dram": 2_097_356_374, "wrreq": 1_495_031_059, "wrreq_dram": 1_495_031_059}
    p.write_text(json.dumps({"entries": [{"config": [1920, 1080, 256, 3, 0, 1], "kernel_source_sha256": sha,
                                          "traffic_bytes_per_launch": 351_000_000_000, "kernel_ms": 91.7,
                                          "profile": "profiles/x", "dram_requests": dr}]}))
    roof = bench.roofline(COUNTS, 90.5, 1920, 1080, _args(str(p)), 1)
    h = roof["hbm_counter"]
    assert h["separates_infinity_cache_hits"] is False
    assert h["hbm_traffic"] is None and h["hbm_frac"] is None
    assert h["dram_share_of_memory_side_requests"] == 1.0
    assert os.path.exists(os.path.join(bench.ROOT, h["calibration"]))
    # the committed C3 entry carries the four counters (their values are a measurement: profiles/r05_dram)
    e = bench.traffic_entry(os.path.join(bench.ROOT, "profiles", "traffic.json"), [1920, 1080, 256, 3, 0, 1], sha)
    assert e is not None
    assert all(isinstance(e["dram_requests"][k], int) for k in ("rdreq", "rdreq_dram", "wrreq", "wrreq_dram"))


def test_roofline_bound_names_the_binding_limiter(tmp_path):
    """`bound` is the resource the profile's binding block names; the HBM figures stay
    (top level, as the bench contract has them, and under hbm_upper_bound) as the upper-bound utilisation."""
    sha = bench.kernel_source_sha256()
    p = tmp_path / "t.json"
    p.write_text(json.dumps({"entries": [{"config": [1920, 1080, 256, 3, 0, 1], "kernel_source_sha256": sha,
                                          "traffic_bytes_per_launch": 343_000_000_000, "kernel_ms": 90.0,
                                          "profile": "profiles/x",
                                          "binding": {"limiter": "walk_steps_x_step_valu", "limiter_detail": "..."}}]}))
    roof = bench.roofline(COUNTS, 90.0, 1920, 1080, _args(str(p)), 1)
    assert roof["bound"] == roof["binding"]["limiter"] == "walk_steps_x_step_valu"
    h = roof["hbm_upper_bound"]
    assert h["frac"] == roof["frac"] and h["achieved"] == roof["achieved"] and h["traffic"] == roof["traffic"]
    assert h["achieved"] <= h["peak"] == bench.HBM_PEAK_GBS


def test_committed_profiles_name_a_limiter():
    """Every committed traffic.json entry with a binding block names its limiter as one key."""
    tj = json.load(open(os.path.join(bench.ROOT, "profiles", "traffic.json")))
    for e in tj["entries"]:
        b = e.get("binding")
        if b:
            assert b["limiter"] in ("valu_issue", "walk_steps_x_step_valu", "lds_walk_and_f64_shading_issue"), e["config"]
            assert len(b["limiter_detail"]) > 40
            if b["limiter"] == "valu_issue":   # priced: the VALU issue time of the launch, near its duration
                assert 0.8 < b["valu_issue_frac_profiled"] < 1.1, e["config"]


def test_valu_issue_block(tmp_path):
    """A profile that prices the launch's VALU issue (tools/valu_bound.py) gives the bench line a valu_issue block
    over this run's kernel time, and bound names it."""
    sha = bench.kernel_source_sha256()
    p = tmp_path / "t.json"
    p.write_text(json.dumps({"entries": [{"config": [1920, 1080, 256, 3, 0, 1], "kernel_source_sha256": sha,
                                          "traffic_bytes_per_launch": 343_000_000_000, "kernel_ms": 90.0,
                                          "profile": "profiles/x",
                                          "binding": {"limiter": "valu_issue", "limiter_detail": "...",
                                                      "valu_issue_ms_per_launch": 88.0,
                                                      "valu_issue_method": "m"}}]}))
    roof = bench.roofline(COUNTS, 90.0, 1920, 1080, _args(str(p)), 1)
    assert roof["bound"] == "valu_issue"
    assert roof["valu_issue"]["frac"] == round(88.0 / 90.0, 4) and roof["valu_issue"]["kernel_ms"] == 90.0


def test_valu_bound_tool_reproduces_the_committed_pricing():
    """tools/valu_bound.py on the committed replay rates, section counts and C3 profile gives the blend that
    profiles/r06_valu/valu_bound.json (and so traffic.json) carries."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("valu_bound", os.path.join(bench.ROOT, "tools", "valu_bound.py"))
    vb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(vb)
    r = vb.bound(os.path.join(bench.ROOT, "profiles", "r06_final", "pmc_summary.json"))
    ref = json.load(open(os.path.join(bench.ROOT, "profiles", "r06_valu", "valu_bound.json")))
    assert r["cycles_per_valu_blend"] == ref["cycles_per_valu_blend"]
    assert 3.0 < r["cycles_per_valu_walk_replay"] < 5.0 and 3.0 < r["cycles_per_valu_shading_replay"] < 5.0


def test_plain_multi_gpu_bench_fails_loudly_without_enough_gpus():
    """`python bench.py --gpus N` with no launcher starts N rank processes itself; with RCCL
    (the default backend) and fewer visible GPUs than N it must fail before rendering, not fall back to one GPU.
    (This container has no GPU: N = 2 > 0; skipped where two GPUs are visible.)"""
    import subprocess
    import sys
    import pytest
    if bench.visible_gpus() >= 2:
        pytest.skip("two GPUs visible: the launch would succeed")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "PT_BENCH_BACKEND")}
    r = subprocess.run([sys.executable, os.path.join(bench.ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert r.stdout == ""                 # no JSON line
    assert "RCCL needs one GPU per rank" in r.stderr


def test_shard_launch_inherits_the_full_frame_limiter(tmp_path):
    """At N > 1 the shard launch's profile holds only its bytes; bound still names the full-frame launch's limiter
    (same kernel on 1/N of the tiles), without the full frame's per-launch VALU pricing."""
    sha = bench.kernel_source_sha256()
    p = tmp_path / "t.json"
    full = {"config": [1920, 1080, 256, 3, 0, 1], "kernel_source_sha256": sha, "traffic_bytes_per_launch": 343_000_000_000,
            "kernel_ms": 90.0, "profile": "profiles/full",
            "binding": {"limiter": "valu_issue", "limiter_detail": "...", "valu_issue_ms_per_launch": 88.0}}
    shard = {"config": [1920, 1080, 256, 3, 0, 8], "kernel_source_sha256": sha, "traffic_bytes_per_launch": 45_000_000_000,
             "kernel_ms": 11.7, "profile": "profiles/shard8"}
    p.write_text(json.dumps({"entries": [full, shard]}))
    roof = bench.roofline(COUNTS, 11.7, 1920, 1080, _args(str(p)), 8)
    assert roof["bound"] == "valu_issue" and roof["binding"]["inherited_from"] == "profiles/full"
    assert "valu_issue" not in roof and "valu_issue_ms_per_launch" not in roof["binding"]
