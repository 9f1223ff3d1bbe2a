#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer entry point (pt_render: render into device memory, then
one device-to-host copy of the W*H*3 fp32 image) against pt_render_device on the same C3 inputs.
Prints one JSON line (GPU box, repo root)."""
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

W, H, SPP, B, K = 1920, 1080, 256, 3, 3
cache = os.path.join(tempfile.gettempdir(), "pt_bench_scene")
os.makedirs(cache, exist_ok=True)
path, mtl, _ = bench.scene_path(cache)
s = bench.load(path, mtl)
cam = pt.make_camera(width=W, height=H, **scenes.SPONZA_STANDIN_CAMERA)
r = pt.Renderer(s, device=0)
fb = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
r.render(cam, W, H, SPP, bounces=B)   # warm-up (builds the per-context tables)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    img, st = r.render(cam, W, H, SPP, bounces=B)
host_s = (time.perf_counter() - t0) / K
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    fb.zero_()
    r.render_device(cam, fb.data_ptr(), W, H, SPP, bounces=B, stream_ptr=stream)
torch.cuda.synchronize()
dev_s = (time.perf_counter() - t0) / K
samples = W * H * SPP
print(json.dumps({"host_buffer_msamples_per_s": round(samples / host_s / 1e6, 1),
                  "device_buffer_msamples_per_s": round(samples / dev_s / 1e6, 1),
                  "host_ms_per_frame": round(host_s * 1e3, 3), "device_ms_per_frame": round(dev_s * 1e3, 3),
                  "image_bytes": W * H * 12}))
r.close()
