#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer entry points against pt_render_device on the same C3 inputs:
  pt_render        render into device memory, one DMA into the context's pinned staging buffer, a
                   parallel host copy into the caller's array (fresh array per frame, and reused);
  pt_render_group  the same through a 1-device group (its RCCL reduce, then the same copy-out).
Prints one JSON line (GPU box, repo root)."""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
import cudapathtracer_amd as pt  # noqa: E402
from cudapathtracer_amd import scenes  # noqa: E402

W, H, SPP, B, K = 1920, 1080, 256, 3, 3
cache = os.path.join(tempfile.gettempdir(), "pt_bench_scene")
os.makedirs(cache, exist_ok=True)
path, mtl, _ = bench.scene_path(cache)
s = bench.load(path, mtl)
cam = pt.make_camera(width=W, height=H, **scenes.SPONZA_STANDIN_CAMERA)
r = pt.Renderer(s, device=0)
fb = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
r.render(cam, W, H, SPP, bounces=B)   # warm-up (builds the per-context tables and the staging buffer)
torch.cuda.synchronize()


def timed(fn):
    t0 = time.perf_counter()
    for _ in range(K):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K


fresh_s = timed(lambda: r.render(cam, W, H, SPP, bounces=B))
keep = np.zeros((H, W, 3), dtype=np.float32)
reuse_s = timed(lambda: r.render(cam, W, H, SPP, bounces=B, out=keep))


def dev_frame():
    fb.zero_()
    r.render_device(cam, fb.data_ptr(), W, H, SPP, bounces=B, stream_ptr=stream)


dev_s = timed(dev_frame)
g = pt.Group([r])
g.render(cam, W, H, SPP, bounces=B, out=keep)
group_fresh_s = timed(lambda: g.render(cam, W, H, SPP, bounces=B))
group_reuse_s = timed(lambda: g.render(cam, W, H, SPP, bounces=B, out=keep))
g.close()
samples = W * H * SPP


def rate(sec):
    return round(samples / sec / 1e6, 1)


print(json.dumps({
    "device_buffer_msamples_per_s": rate(dev_s), "device_ms_per_frame": round(dev_s * 1e3, 3),
    "host_buffer_fresh_msamples_per_s": rate(fresh_s), "host_fresh_ms_per_frame": round(fresh_s * 1e3, 3),
    "host_buffer_reused_msamples_per_s": rate(reuse_s), "host_reused_ms_per_frame": round(reuse_s * 1e3, 3),
    "group1_fresh_msamples_per_s": rate(group_fresh_s), "group1_fresh_ms_per_frame": round(group_fresh_s * 1e3, 3),
    "group1_reused_msamples_per_s": rate(group_reuse_s), "group1_reused_ms_per_frame": round(group_reuse_s * 1e3, 3),
    "group1_reused_of_device": round(dev_s / group_reuse_s, 4),
    "host_fresh_of_device": round(dev_s / fresh_s, 4),
    "image_bytes": W * H * 12,
    "host_threads_env": os.environ.get("OMP_NUM_THREADS")}))
r.close()
