#!/usr/bin/env python3
"""Benchmark of the per-pixel path-integration hot path (BASELINE.json north star).

Workload (config C3, the default and the headline): the ~262K-triangle procedural Sponza-class
STAND-IN (Sponza is absent from this container; PT_SPONZA_OBJ=<path> uses a real file), 1920x1080,
256 spp, 3 bounces, unidirectional integrator (kernel.cu:417-515), seed 1234.  One "step" = one
full render of that image (all samples), inputs resident in HBM; for N GPUs each rank renders its
interleaved 8x8 tiles into a zero-filled fp32 framebuffer and rank 0 receives the RCCL sum (weak
scaling of the per-GPU work is NOT used: total work per step is fixed, so scaling is "strong").
--config C2 (Cornell 1024x1024, 64 spp, depth 8) / C4 (C3 at 1024 spp) / C5 (stand-in 3840x2160,
4096 spp, depth 16) measure the other BASELINE configs the same way; --integrator 1 the HEAD
integrator (kernel.cu:217-415).

Prints ONE JSON line on rank 0 (contract in the task statement), with:
  value      = Msamples/s, whole job (pixel samples per second)
  roofline   = measured memory-side bytes per launch (rocprof, calibrated; from profiles/traffic.json
               when it matches this kernel) / this run's kernel time vs 8 TB/s HBM, with the binding
               pipes beside it
  cache_roofline = the algorithmic (requested) record bytes per launch / kernel time vs the ~34.5 TB/s
               aggregate L2: caches serve most of them, so they are not an HBM figure
  cpu_baseline = the CPU oracle (same integrator) on a bounded pixel subset, host cores
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
L2_PEAK_GBS = 34500.0   # aggregate L2 bandwidth, 8 XCDs (MI355X_MICROARCH.md "L2 (per XCD)")
NODE_BYTES = 128          # one BVH4 node record (6 x float4 child boxes + uint4 children + pad)
TRI_BYTES = 48            # one triangle record {v0, e1, e2, id, rank, parent}
# the sources that define the render kernel: profiles/traffic.json is used only when it was measured
# on a build of exactly these (a stale PMC number cannot ride along)
KERNEL_SOURCES = ("cudapathtracer_amd/csrc/hip/pt_render.hip", "cudapathtracer_amd/csrc/hip/pt_device.h",
                  "cudapathtracer_amd/csrc/Makefile", "cudapathtracer_amd/csrc/host/accel_build.cpp")


def kernel_source_sha256():
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(ROOT, rel), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def host_cores():
    """Threads for the CPU baseline, as `nproc` counts them: OMP_NUM_THREADS when set, else the
    CPUs this process may run on."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.strip().isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


# BASELINE.json configs as bench workloads: scene, image, spp, bounces
CONFIGS = {
    "C2": dict(scene="cornell", width=1024, height=1024, spp=64, bounces=8),
    "C3": dict(scene="standin", width=1920, height=1080, spp=256, bounces=3),
    "C4": dict(scene="standin", width=1920, height=1080, spp=1024, bounces=3),
    "C5": dict(scene="standin", width=3840, height=2160, spp=4096, bounces=16),
}


def scene_path(cache_dir, kind="standin"):
    from cudapathtracer_amd import scenes
    if kind == "cornell":   # the build's Cornell box OBJ+MTL (ceiling light facing -y, kernel.cu:503)
        p = os.path.join(cache_dir, "models", "cornell.obj")
        if not os.path.exists(p):
            scenes.write_cornell(cache_dir)
        return p, os.path.dirname(p) + "/", "cornell (build-authored Cornell box mesh)"
    real = os.environ.get("PT_SPONZA_OBJ")
    if real:
        return real, os.path.dirname(real) + "/", "sponza (PT_SPONZA_OBJ)"
    p = os.path.join(cache_dir, "models", "sponza_standin.obj")
    if not os.path.exists(p):
        scenes.write_sponza_standin(cache_dir)
    return p, os.path.dirname(p) + "/", "sponza_standin_262k (procedural stand-in, not Sponza)"


def load(path, mtl):
    import cudapathtracer_amd as pt
    t = time.time()
    s = pt.Scene()
    s.load_obj(path, mtl_basepath=mtl)
    s.build_bvh()
    log("scene loaded + BVH built in %.2fs" % (time.time() - t))
    return s


def cpu_baseline(scene, cam_kw, width, height, spp, bounces, threads, budget_s, integrator=0):
    """Oracle (CPU restatement of the same integrator) on a bounded subset of the same image."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from cudapathtracer_amd import shard
    osc = oracle.OracleScene(scene.arrays())
    ocam = oracle.camera(cam_kw["pos"], cam_kw["dist_from_film"], cam_kw["focal_length"], cam_kw["radius"],
                         width, height)
    ntiles = shard.tiles_shape(width, height)[0] * shard.tiles_shape(width, height)[1]
    # calibrate on a spread of tiles, then size the subset (every k-th tile, full spp) to the budget
    cal_tiles = np.linspace(0, ntiles - 1, 4 * threads).astype(np.int64)
    t0 = time.time()
    oracle.render(osc, ocam, width, height, spp, bounces, integrator, 1234,
                  pixels=shard.tile_pixels(width, height, cal_tiles), threads=threads)
    dt = max(time.time() - t0, 1e-3) / len(cal_tiles)
    tiles_fit = max(1, int(budget_s / dt))
    stride = max(1, ntiles // tiles_fit)
    tiles = np.arange(stride // 2, ntiles, stride)[:tiles_fit]
    pix = shard.tile_pixels(width, height, tiles)
    t0 = time.time()
    _, cnt = oracle.render(osc, ocam, width, height, spp, bounces, integrator, 1234, pixels=pix, threads=threads)
    dt = time.time() - t0
    samples = len(pix) * spp
    return {
        "value": samples / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
        "nproc": host_cores(), "cpu_model": cpu_model(),
        "mrays_per_s": cnt["traces"] / dt / 1e6,
        "sample": "%d pixels (every %d-th 8x8 tile) x %d spp of the same %dx%d image, %.1fs"
                  % (len(pix), stride, spp, width, height, dt),
    }


def traffic_entry(path, cfg, sha):
    """The profiles/traffic.json entry measured on this kernel source and bench config, or None.
    The file holds {"entries": [...]}, one per (config, source hash)."""
    if not os.path.exists(path):
        return None
    try:
        tj = json.load(open(path))
    except (OSError, ValueError):
        return None
    for e in tj.get("entries", [tj] if "config" in tj else []):
        if e.get("config") == cfg and e.get("kernel_source_sha256") == sha:
            return e
    return None


def roofline(counts, kms, W, H, args, world):
    """The render kernel against the HBM roofline.

    achieved / frac / traffic: MEASURED memory-side bytes per launch (rocprofv3 FETCH_SIZE x2 +
    WRITE_SIZE, the x2 calibrated on this kernel's own access shapes, profiles/r02_fetch_calibration)
    from profiles/traffic.json -- used only if that profile was taken on this exact kernel source and
    config -- over this run's kernel time; null otherwise.  binding: the pipes that actually limit the
    kernel, from the same profile.  (The algorithmic bytes are cache_roofline's, against the L2 roof.)"""
    sec = kms * 1e-3
    # bound: the resource the profile names as binding (binding.limiter); "hbm" only while no profile of this
    # kernel says otherwise.  achieved / peak / frac / traffic stay the HBM-side figures (also under
    # hbm_upper_bound): the one roof this pointer-chasing kernel is priced against, an upper bound on HBM bytes.
    roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None, "traffic": None,
            "traffic_source": None,
            "kernel": KERNEL_NAME(args),
            "kernel_ms": round(kms, 3),
            "kernel_ms_note": "the integration kernel alone (HIP events around its launch on its stream), "
                              "without the seeding pre-pass and the split-pixel finalisation",
            "traffic_note": "rocprofv3 FETCH_SIZE x2 + WRITE_SIZE: bytes between L2 and the memory side (Infinity "
                            "Cache hits included), so frac is an upper bound on the HBM fraction",
            "kernel_source_sha256": kernel_source_sha256(),
            "node_fetches": int(counts["node_tests"]), "lds_node_fetches": int(counts["lds_node_tests"]),
            "tri_tests": int(counts["tri_tests"]),
            "walk_simd_util": round(counts["node_tests"] / max(counts["walk_lane_slots"], 1), 4),
            "leaf_step_frac": round(counts["leaf_steps"] / max(counts["node_tests"], 1), 4),
            "accel_fallbacks": int(counts["accel_fallbacks"]), "spill_entries": int(counts["spill_entries"]),
            "walk_phase_frac": round(counts["walk_cycles"] / max(counts["walk_cycles"] + counts["shade_cycles"], 1), 4),
            "shade_phases": int(counts["shade_lane_slots"] // 64)}
    tj = traffic_entry(args.traffic_json, [W, H, args.spp, args.bounces, args.integrator, max(world, args.sim_shards)],
                       roof["kernel_source_sha256"])
    if tj is not None:
        traffic = int(tj["traffic_bytes_per_launch"])
        roof["traffic"] = traffic
        roof["achieved"] = round(traffic / sec / 1e9, 2)
        roof["frac"] = round(traffic / sec / 1e9 / HBM_PEAK_GBS, 4)
        roof["traffic_source"] = {"profile": tj.get("profile"), "method": tj.get("method"),
                                  "kernel_ms_profiled": tj.get("kernel_ms")}
        roof["hbm_upper_bound"] = {
            "achieved": roof["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": roof["frac"], "traffic": traffic,
            "note": "memory-side bytes (L2 misses, Infinity-Cache hits included) per launch over the kernel time: the "
                    "HBM roof's utilisation at most; not what binds the kernel (see bound / binding)"}
        binding = tj.get("binding")
        shards = max(world, args.sim_shards)
        if not binding and shards > 1:
            # a shard launch's profile holds its bytes only: the limiter is the full-frame launch's (the same kernel
            # on 1/N of the tiles), without that launch's per-launch VALU pricing
            full = traffic_entry(args.traffic_json, [W, H, args.spp, args.bounces, args.integrator, 1],
                                 roof["kernel_source_sha256"])
            if full and full.get("binding"):
                binding = {k: v for k, v in full["binding"].items() if not k.startswith("valu_issue")}
                binding["inherited_from"] = full.get("profile")
        if binding:
            tj = dict(tj, binding=binding)
            roof["binding"] = tj["binding"]
            if roof["binding"].get("limiter"):
                roof["bound"] = roof["binding"]["limiter"]
            vi = roof["binding"].get("valu_issue_ms_per_launch")
            if vi:
                # the binding roof: the launch's VALU instructions priced at the rate the kernel's own streams
                # issue at alone (profiles/r06_valu, tools/valu_bound.py) against this run's kernel time
                roof["valu_issue"] = {
                    "achieved_ms": vi, "kernel_ms": round(kms, 3), "frac": round(vi / kms, 4), "unit": "ms per launch",
                    "method": roof["binding"].get("valu_issue_method"),
                    "note": "the time the SIMDs need just to issue this launch's VALU instructions (counted by "
                            "SQ_INSTS_VALU in the profile of this kernel source and config) at the rate the kernel's own "
                            "walk / shading instruction streams reach replayed alone at 5 waves per SIMD; frac ~1 means "
                            "VALU issue fills the launch and memory latency is hidden (DESIGN.md 6.3)"}
        dr = tj.get("dram_requests")
        if dr:
            roof["hbm_counter"] = {
                "counters": "TCC_EA0_RDREQ_DRAM_sum / TCC_EA0_WRREQ_DRAM_sum (rocprofv3, one --pmc pass)",
                "rdreq_dram": dr["rdreq_dram"], "rdreq": dr["rdreq"], "wrreq_dram": dr["wrreq_dram"], "wrreq": dr["wrreq"],
                "dram_share_of_memory_side_requests": round((dr["rdreq_dram"] + dr["wrreq_dram"]) /
                                                            max(dr["rdreq"] + dr["wrreq"], 1), 4),
                "separates_infinity_cache_hits": False,
                "hbm_traffic": None, "hbm_frac": None,
                "calibration": "profiles/r05_dram/dram_table.txt",
                "note": "on a 32-MiB Infinity-Cache-resident table the DRAM-request counters equal the memory-side "
                        "request counters (every L2 miss is 'destined for DRAM' whether the Infinity Cache or HBM "
                        "serves it); no counter on this pool separates them, so HBM bytes proper are unmeasured "
                        "and frac stays an upper bound"}
    return roof


L1_LINES_PER_CU_CYCLE = 1.0   # measured ceiling: tools/gpu/micro/node_gather.hip, profiles/r04_l1_lookups


def l1_roofline(roof):
    """Utilisation of the L1's cache-line lookups (profiles/r04_l1_lookups).  A scattered
    dwordx4 costs one lookup per lane (per distinct 128-B line), a node visit seven; a dependent gather loop
    of them runs at ~1 line per CU-cycle however the lines are spread over L2 / Infinity Cache / HBM (10 and
    100 MB tables alike) and however many lanes are masked or out of range.  achieved = the render kernel's
    TCP_TOTAL_CACHE_ACCESSES per CU-cycle from the same profile as `roofline`.  Not the walk's limiter: 18%
    fewer lookups left the rate unchanged (profiles/r04_topasm); the walk steps per ray are."""
    b = (roof or {}).get("binding") or {}
    x = b.get("l1_lookups_per_cu_cycle")
    if x is None:
        return None
    return {"bound": "l1_lookups", "binding": False, "achieved": x, "peak": L1_LINES_PER_CU_CYCLE, "unit": "lines/CU-cycle",
            "frac": round(x / L1_LINES_PER_CU_CYCLE, 4), "source": (roof.get("traffic_source") or {}).get("profile"),
            "peak_source": "tools/gpu/micro/node_gather.hip (profiles/r04_l1_lookups)"}


def cache_roofline(counts, kms):
    """The algorithmic bytes (records the walk and the shading pass request: node records not served by
    the LDS top, triangle records, per-ray shading reads, output) over the kernel time, against the L2
    roof (MI355X_MICROARCH.md: 8 XCDs x 4 MiB, ~34.5 TB/s aggregate).  L2 and the Infinity Cache serve
    most of these requests, so they are NOT HBM bytes and are kept out of the HBM `roofline` object."""
    npx = counts["samples"] / max(counts.get("spp", 1), 1)
    mem_nodes = counts["node_tests"] - counts["lds_node_tests"]
    alg = (mem_nodes * NODE_BYTES + counts["tri_tests"] * TRI_BYTES + counts["rays_traced"] * (16 + 48) + npx * 12)
    gbs = alg / (kms * 1e-3) / 1e9
    return {"bound": "l2", "achieved": round(gbs, 2), "peak": L2_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / L2_PEAK_GBS, 4), "algorithmic_bytes_per_launch": int(alg),
            "note": "requested record bytes (nodes x %d B + triangles x %d B + traced rays x 64 B + 12 B per "
                    "pixel) per launch / kernel time, against the aggregate L2 bandwidth" % (NODE_BYTES, TRI_BYTES)}


class FrameLoop:
    """Frames rendered back to back into a ring of framebuffers, each frame's reduce to rank 0
    issued asynchronously so that it overlaps the next frame's render (a buffer is zeroed again
    only after its reduce has completed -- `wait()` orders the stream, the host does not block).

    render(buf) -> stats dict: renders this rank's tiles into the zero-filled buf -- or, with `wait`
    given, only enqueues the render (pt_render_device_async) and wait() returns the oldest queued
    frame's stats: frame k+1 is queued before frame k's stats are collected, so the GPU never idles
    between frames (the host's return path and the next launches overlap the render).
    reduce(buf) -> work with .wait(), or None (one process, or a synchronous reduce).
    streams: optional, one (torch) stream per framebuffer: frame k's zeroing, render and reduce are issued
    on streams[k % len] (the current stream while they are issued), so consecutive frames are ordered
    only by their own dependencies -- the next frame's seeding pre-pass and render blocks start while
    this frame's render drains its last waves, and its split-pixel finalisation runs beside them.
    step() returns a frame's stats (the previous frame's when asynchronous, None for the first);
    `drain()` returns (the last frame's buffer once its reduce is ordered before whatever the caller
    does next, the stats of the frames still in flight)."""

    def __init__(self, bufs, render, reduce=None, wait=None, streams=None):
        self.bufs = list(bufs)
        self.render = render
        self.reduce = reduce
        self.wait = wait
        self.streams = list(streams) if streams else None
        self.pending = [None] * len(self.bufs)
        self.frames = 0
        self.inflight = 0

    def step(self):
        k = self.frames % len(self.bufs)
        if self.streams:
            import torch
            with torch.cuda.stream(self.streams[k % len(self.streams)]):
                st = self._issue(k)
        else:
            st = self._issue(k)
        self.frames += 1
        if self.wait is None:
            return st
        self.inflight += 1
        if self.inflight > 1:   # the previous frame's stats, with this one queued behind it
            self.inflight -= 1
            return self.wait()
        return None

    def _issue(self, k):
        if self.pending[k] is not None:
            self.pending[k].wait()
            self.pending[k] = None
        buf = self.bufs[k]
        buf.zero_()
        st = self.render(buf)
        if self.reduce is not None:
            self.pending[k] = self.reduce(buf)
        return st

    def drain(self):
        stats = []
        while self.wait is not None and self.inflight > 0:
            stats.append(self.wait())
            self.inflight -= 1
        for k, w in enumerate(self.pending):
            if w is not None:
                w.wait()
                self.pending[k] = None
        return (self.bufs[(self.frames - 1) % len(self.bufs)] if self.frames else self.bufs[0]), stats


def make_reduce(dist, backend, rank):
    """RCCL (backend nccl): an async reduce(SUM) to rank 0 on the device tensor.  gloo (rehearsal of
    the multi-process path on one GPU or on CPU): a synchronous reduce through host memory."""
    if backend == "nccl":
        return lambda buf: dist.reduce(buf, dst=0, op=dist.ReduceOp.SUM, async_op=True)

    def gloo_reduce(buf):
        host = buf.cpu() if buf.is_cuda else buf
        dist.reduce(host, dst=0, op=dist.ReduceOp.SUM)
        if rank == 0 and host is not buf:
            buf.copy_(host)
        return None
    return gloo_reduce


def make_gather(dist, backend, rank, world, width, height):
    """The framebuffer's assembly as a gather instead of a reduce: each rank sends only its own tiles' pixels
    (1/N of the image: 3.1 MB of C3's 24.9 MB at N = 8) to rank 0, which copies them into its framebuffer.  Over
    xGMI every rank has its own link to rank 0, so the N - 1 transfers run side by side, where a reduce moves the
    whole framebuffer through the ring.  The result is the same image (every pixel is exactly one rank's value;
    the reduce adds zeros to it).  RCCL: async (point-to-point sends and receives in one group), the copy into
    rank 0's framebuffer issued at wait(); gloo: synchronous through host memory."""
    import torch
    from cudapathtracer_amd import shard
    pix = [torch.from_numpy(shard.shard_pixels(width, height, j, world).astype(np.int64)) for j in range(world)]
    n = max(len(p) for p in pix)
    slots = {}   # per framebuffer: (device index tensors, send buffer, receive buffers): two frames may be in flight

    def buffers(buf):
        key = buf.data_ptr()
        if key not in slots:
            idx = [p.to(buf.device) for p in pix]
            send = torch.zeros((n, 3), dtype=buf.dtype, device=buf.device)
            recv = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
            slots[key] = (idx, send, recv)
        return slots[key]

    def unpack(flat, idx, recv):
        for j in range(1, world):
            flat.index_copy_(0, idx[j], recv[j][:len(idx[j])].to(flat.device))

    def gather(buf):
        idx, send, recv = buffers(buf)
        flat = buf.view(-1, 3)
        mine = idx[rank]
        torch.index_select(flat, 0, mine, out=send[:len(mine)])
        if backend == "nccl":
            work = dist.gather(send, recv, dst=0, async_op=True)

            class Work:
                def wait(self_inner):
                    work.wait()
                    if rank == 0:
                        unpack(flat, idx, recv)
            return Work()
        host = send.cpu()
        hrecv = [torch.empty_like(host) for _ in range(world)] if rank == 0 else None
        dist.gather(host, hrecv, dst=0)
        if rank == 0:
            unpack(flat, idx, hrecv)
        return None
    return gather


class stdout_to_stderr:
    """Route file descriptor 1 to stderr for the block: the process-group setup's own banners (RCCL's
    version lines, gloo's peer messages) are printed by C++ to stdout, which must carry rank 0's one
    JSON line only."""

    @staticmethod
    def _flush_all():
        # Python's buffer, then C stdio's (RCCL / gloo print through libc; a pipe makes stdout fully
        # buffered, so text left there would be flushed after rank 0's JSON line at exit)
        sys.stdout.flush()
        ctypes.CDLL(None).fflush(None)

    def __enter__(self):
        self._flush_all()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        self._flush_all()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def visible_gpus():
    """GPUs this process may use, counted without initialising the GPU (on this image
    `torch.cuda.device_count()` does not create a HIP context)."""
    import torch
    return torch.cuda.device_count()


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, backend, argv=None):
    """`bench.py --gpus N` with no launcher (WORLD_SIZE unset): start N fresh rank processes of this
    script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, exactly what
    `torch.distributed.run` would give them, and relay rank 0's one JSON line.  This parent never touches
    the GPU (it only counts devices) and never execs: the ranks are children, and it exits with the first
    failing rank's status (the others are then stopped by PID).  RCCL needs one device per rank, so N larger
    than the visible GPUs fails loudly; PT_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (the ranks'
    device index wraps, as under torch.distributed.run).  Returns the exit status."""
    import subprocess
    ndev = visible_gpus()
    if backend == "nccl" and n > ndev:
        log("error: --gpus %d but %d GPU(s) visible; RCCL needs one GPU per rank (no fallback to fewer GPUs; "
            "PT_BENCH_BACKEND=gloo rehearses several ranks on one GPU)" % (n, ndev))
        return 2
    argv = list(sys.argv[1:] if argv is None else argv)
    port = _free_port()
    procs = []
    for k in range(n):
        env = dict(os.environ, RANK=str(k), LOCAL_RANK=str(k), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PT_BENCH_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE if k == 0 else sys.stderr.fileno()))
    log("launched %d rank processes (%s, 127.0.0.1:%d): pids %s"
        % (n, backend, port, " ".join(str(p.pid) for p in procs)))
    import threading
    out = []   # rank 0's stdout (its one JSON line), read to EOF beside the wait so the pipe cannot fill
    reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    status = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            rc = p.poll()
            if rc is None:
                continue
            pending.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                log("rank pid %d exited with %d; stopping the other ranks" % (p.pid, rc))
                for q in pending:
                    q.kill()
        if pending:
            time.sleep(0.05)
    reader.join()
    if status == 0:
        sys.stdout.write(b"".join(out).decode())
        sys.stdout.flush()
    return status


def KERNEL_NAME(args):
    if args.flags & 1:   # PT_FLAG_REFERENCE_TRAVERSAL: the tile kernel
        return "render_tiles"
    return "render_head_wf" if args.integrator == 1 else "render_unidir_wf"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="C3", choices=sorted(CONFIGS),
                    help="BASELINE config: scene, image size, spp and bounces (overridable below)")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--bounces", type=int, default=None)
    ap.add_argument("--integrator", type=int, default=0)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--cpu-threads", type=int, default=host_cores())
    ap.add_argument("--no-count", action="store_true", help="skip the counting pass (roofline bytes)")
    ap.add_argument("--sim-shards", type=int, default=1,
                    help="diagnostic, single process only: render shard 0 of N (one GPU's share at N GPUs)")
    ap.add_argument("--sync-frames", action="store_true",
                    help="one blocking render per frame (pt_render_device) instead of frames queued back to back")
    ap.add_argument("--one-stream", action="store_true",
                    help="frames queued back to back on one stream even for shards (no overlap of consecutive frames)")
    ap.add_argument("--two-streams", action="store_true",
                    help="frames on two streams even for the whole frame (default only for shards of N > 1)")
    ap.add_argument("--collective", default="reduce", choices=["reduce", "gather"],
                    help="N > 1: assemble rank 0's image by a reduce of the zero-filled framebuffers (default) or by a "
                         "gather of each rank's own tiles (1/N of the bytes per rank, point to point; rehearsal option: "
                         "run over gloo on one GPU and as a one-rank RCCL group, never yet on two devices)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--cache-dir", default=os.path.join(tempfile.gettempdir(), "pt_bench_scene"))
    args = ap.parse_args()
    for k, v in CONFIGS[args.config].items():
        if k != "scene" and getattr(args, k) is None:
            setattr(args, k, v)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    # PT_BENCH_BACKEND=gloo rehearses the multi-process path where RCCL cannot run (several ranks
    # on one GPU: the device index wraps over the visible GPUs when there are fewer than ranks)
    backend = os.environ.get("PT_BENCH_BACKEND", "nccl")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # a plain `python bench.py --gpus N`: this process becomes the launcher of N rank processes
        sys.exit(launch_ranks(args.gpus, backend))

    import torch
    import torch.distributed as dist
    import cudapathtracer_amd as pt
    from cudapathtracer_amd import scenes

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    shards = world if world > 1 else max(1, args.sim_shards)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("note: WORLD_SIZE=%d, --gpus=%d; using WORLD_SIZE" % (world, args.gpus))
    distributed = world > 1
    ndev = torch.cuda.device_count()
    if ndev == 0:
        raise SystemExit("bench.py: no GPU visible (the render path is HIP only)")
    if local >= ndev:
        if backend == "nccl" and distributed:
            raise SystemExit("bench.py: rank %d has LOCAL_RANK %d but %d GPU(s) are visible; RCCL needs one GPU per "
                             "rank (PT_BENCH_BACKEND=gloo rehearses several ranks on one GPU)" % (rank, local, ndev))
        local = local % ndev
    torch.cuda.set_device(local)
    if distributed:
        with stdout_to_stderr():   # (communicator setup, and a first collective: no banner on stdout)
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                dist.init_process_group(backend)
            dist.barrier()

    os.makedirs(args.cache_dir, exist_ok=True)
    kind = CONFIGS[args.config]["scene"]
    path, mtl, scene_name = scene_path(args.cache_dir, kind)
    scene = load(path, mtl)
    cam_kw = dict(scenes.CORNELL_CAMERA if kind == "cornell" else scenes.SPONZA_STANDIN_CAMERA)
    W, H = args.width, args.height
    cam = pt.make_camera(width=W, height=H, **cam_kw)
    r = pt.Renderer(scene, device=local)
    # two framebuffers (and, for a shard of N > 1, two streams): frame k's RCCL reduce runs while frame
    # k+1 renders into the other one.  On two streams frame k+1's seeding pre-pass runs beside frame k's
    # last waves (its integration kernel still follows frame k's finalisation): +1.3% on the 1/8 C3 shard,
    # +-0 on the whole frame, -9% on C2's 10-ms frames (the cross-stream wait), so shards only by default
    overlap = not args.sync_frames and not args.one_stream and (args.two_streams or shards > 1)
    fbs = [torch.zeros((H, W, 3), dtype=torch.float32, device="cuda") for _ in range(2 if (distributed or overlap) else 1)]

    def render(buf, flags=0):
        return r.render_device(cam, buf.data_ptr(), W, H, args.spp, bounces=args.bounces, integrator=args.integrator,
                               flags=args.flags | flags, shard_index=rank, shard_count=shards,
                               stream_ptr=torch.cuda.current_stream().cuda_stream)

    def render_async(buf):
        r.render_device_async(cam, buf.data_ptr(), W, H, args.spp, bounces=args.bounces, integrator=args.integrator,
                              flags=args.flags, shard_index=rank, shard_count=shards,
                              stream_ptr=torch.cuda.current_stream().cuda_stream)

    red = None
    if distributed:
        red = make_reduce(dist, backend, rank) if args.collective == "reduce" else make_gather(dist, backend, rank, world, W, H)
    if args.sync_frames:
        loop = FrameLoop(fbs, render, red)
    else:
        loop = FrameLoop(fbs, render_async, red, wait=r.wait,
                         streams=[torch.cuda.Stream() for _ in fbs] if overlap else None)

    # counting pass (same inputs, counting variant): algorithmic bytes of the render kernel
    counts = None
    if not args.no_count:
        fbs[0].zero_()
        counts = render(fbs[0], pt.PT_FLAG_COUNT)
    for _ in range(args.warmup):
        loop.step()
    loop.drain()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_ms = []
    stats = []
    for _ in range(args.steps):
        st = loop.step()
        if st is not None:
            stats.append(st)
    fb, rest = loop.drain()
    stats += rest
    kernel_ms = [st["kernel_ms"] for st in stats]
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    dev = "cuda" if backend == "nccl" else "cpu"
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    tot = torch.tensor([sum(s["samples"] for s in stats), sum(s["rays_traced"] for s in stats),
                        sum(s["rays_reference"] for s in stats)], dtype=torch.float64, device=dev)
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    elapsed = float(t.item())
    samples, traced, refrays = [float(v) for v in tot.tolist()]

    if rank == 0:
        img = fb.cpu().numpy()
        finite = bool(np.isfinite(img).all())
        ms_step = elapsed / args.steps * 1e3
        kms = float(np.mean(kernel_ms))
        roof = roofline(counts, kms, W, H, args, world) if counts is not None else None
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(scene, cam_kw, W, H, args.spp, args.bounces, args.cpu_threads, args.cpu_budget,
                               args.integrator)
        out = {
            "metric": "Mrays/sec + Msamples/sec, Sponza 1080p 256spp, 1/2/4/8 GPU",
            "value": round(samples / elapsed / 1e6, 3),
            "unit": "Msamples/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32 geometry / f64 radiance",
            "data": "synthetic",
            "config": {"workload": "%s %s %dx%d %dspp %d bounces integrator=%d" % (
                args.config, scene_name, W, H, args.spp, args.bounces, args.integrator),
                "scene": scene_name, "width": W, "height": H, "spp": args.spp, "bounces": args.bounces,
                "integrator": "unidirectional" if args.integrator == 0 else "head", "seed": 1234,
                "parallelism": ("image tiles %dx, %s %s" % (world, "RCCL" if backend == "nccl" else backend, args.collective)
                                if distributed else
                                "1 GPU" if shards == 1 else "1 GPU rendering shard 0 of %d (diagnostic)" % shards),
                "rank_launcher": (None if not distributed else
                                  "bench.py (one child process per rank)" if os.environ.get("PT_BENCH_LAUNCHED")
                                  else "external (WORLD_SIZE set, e.g. torch.distributed.run)")},
            "mrays_per_s_traced": round(traced / elapsed / 1e6, 3),
            "reference_equiv_not_traced": {
                "mrays_per_s": round(refrays / elapsed / 1e6, 3),
                "note": "trace() calls the reference integrator would make for the same samples; NOT rays traced "
                        "here (the primary-hit memo and the dead-path skip are exact shortcuts): never a throughput"},
            "mrays_per_s_nominal": round(samples * (args.bounces + 1) / elapsed / 1e6, 3),
            "image_finite": finite,
            "roofline": roof,
            "cache_roofline": cache_roofline(dict(counts, spp=args.spp), kms) if counts is not None else None,
            "l1_roofline": l1_roofline(roof),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    r.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
