#!/usr/bin/env python3
"""Does a small kernel on a second stream run while the persistent render kernel occupies the GPU?
(bench.py's FrameLoop issues frame k's RCCL reduce on RCCL's stream and then frame
k+1's render; the render launches blocks up to full residency on every CU.)

On one GPU (run under `rocprofv3 --kernel-trace`, GPU box, repo root): frames of the C3 1/8 shard (the
8-GPU job's per-GPU work) rendered back to back as FrameLoop does, and after each render a stand-in for
the reduce kernel on a second stream -- torch.cuda._sleep (one wave spinning ~SLEEP_US) or a 24.9 MB
device copy (the reduce's memory traffic) -- launched before the next render.  Prints per-frame wall
times for: no side kernel / sleep / copy.  The kernel trace gives each kernel's start and end, so
tools/gpu/overlap_report.py can tell whether the side kernel ran inside the next render's span."""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import torch  # noqa: E402
import cudapathtracer_amd as pt  # noqa: E402
from cudapathtracer_amd import scenes  # noqa: E402

W, H, SPP, B = 1920, 1080, 256, 3
SHARDS = int(os.environ.get("SHARDS", "8"))
FRAMES = int(os.environ.get("FRAMES", "6"))
SLEEP_US = float(os.environ.get("SLEEP_US", "500"))
cache = os.path.join(tempfile.gettempdir(), "pt_bench_scene")
os.makedirs(cache, exist_ok=True)
path, mtl, _ = bench.scene_path(cache)
s = bench.load(path, mtl)
cam = pt.make_camera(width=W, height=H, **scenes.SPONZA_STANDIN_CAMERA)
r = pt.Renderer(s, device=0)
fbs = [torch.zeros((H, W, 3), dtype=torch.float32, device="cuda") for _ in range(2)]
dst = torch.zeros_like(fbs[0])
main = torch.cuda.current_stream()
side = torch.cuda.Stream()
# cycles for SLEEP_US: the wall-clock rate of s_memrealtime is 100 MHz; _sleep counts shader clocks
clk_hz = 2.4e9


def run(mode):
    times = []
    for f in range(FRAMES):
        buf = fbs[f % 2]
        t0 = time.perf_counter()
        buf.zero_()
        r.render_device(cam, buf.data_ptr(), W, H, SPP, bounces=B, shard_index=0, shard_count=SHARDS,
                        stream_ptr=main.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(main)
        side.wait_event(ev)
        with torch.cuda.stream(side):   # frame f's "reduce", issued before frame f+1's render
            if mode == "sleep":
                torch.cuda._sleep(int(SLEEP_US * 1e-6 * clk_hz))
            elif mode == "copy":
                dst.copy_(buf)
        times.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    return times


out = {}
for mode in ("none", "sleep", "copy", "none2"):
    run(mode)                      # warm-up pass of this mode
    t = run(mode)
    out[mode] = {"ms_per_frame_median": round(sorted(t)[len(t) // 2] * 1e3, 3), "frames_ms": [round(x * 1e3, 3) for x in t]}
print(json.dumps({"shards": SHARDS, "sleep_us": SLEEP_US, "modes": out}))
r.close()
