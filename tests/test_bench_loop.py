"""bench.py's multi-process frame loop, without a GPU.

The render is a stub that writes this rank's 8x8 tiles (cudapathtracer_amd.shard, the kernel's
assignment) with values that depend on the frame number, so a reduce of a stale or half-zeroed
buffer shows up; the loop, the ring of framebuffers and the reduce are bench.py's own
(FrameLoop, make_reduce).  world_size 2 over gloo on CPU tensors, as the GPU job runs them over RCCL."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402
from cudapathtracer_amd import shard  # noqa: E402

W, H = 40, 24


def frame_image(frame):
    """What the full single-process render of `frame` would hold (a stub integrand)."""
    pix = np.arange(W * H, dtype=np.float32)
    img = np.stack([pix + 1, pix * 0.5 + frame, np.full_like(pix, 3.0 + frame)], axis=1)
    return img.reshape(H, W, 3)


def stub_render(rank, world, counter):
    full = {}

    def render(buf):
        frame = counter[0]
        counter[0] += 1
        if frame not in full:
            full[frame] = torch.from_numpy(frame_image(frame))
        pix = torch.from_numpy(shard.shard_pixels(W, H, rank, world).astype(np.int64))
        flat = buf.view(-1, 3)
        assert float(flat.abs().sum()) == 0.0, "the loop must hand the renderer a zeroed buffer"
        flat[pix] = full[frame].view(-1, 3)[pix]
        return {"samples": len(pix), "rays_traced": 2 * len(pix), "rays_reference": 3 * len(pix), "kernel_ms": 1.0}
    return render


def async_stub(render):
    """render as pt_render_device_async / pt_render_wait present it: enqueue (here: do) the frame, hand
    its stats out later, oldest first, at most two in flight."""
    queue = []

    def enqueue(buf):
        assert len(queue) < 2, "at most two renders in flight per context"
        queue.append(render(buf))

    def wait():
        return queue.pop(0)
    return enqueue, wait


class LazyReduce:
    """An async 'collective' that only lands at wait(): catches a loop that reuses a buffer before
    its reduce completed or returns a buffer whose reduce is still pending."""

    def __init__(self, log):
        self.log = log

    def __call__(self, buf):
        snap = buf.clone()
        log = self.log

        class Work:
            def wait(self_inner):
                log.append(float(snap.sum()))
                buf.copy_(snap * 2)   # 'sum over two identical ranks'
        return Work()


@pytest.mark.parametrize("asynchronous", [False, True])
def test_frame_loop_orders_buffers_and_reduces(asynchronous):
    counter = [0]
    log = []
    bufs = [torch.zeros((H, W, 3)) for _ in range(2)]
    if asynchronous:
        enqueue, wait = async_stub(stub_render(0, 1, counter))
        loop = bench.FrameLoop(bufs, enqueue, LazyReduce(log), wait=wait)
    else:
        loop = bench.FrameLoop(bufs, stub_render(0, 1, counter), LazyReduce(log))
    stats = [loop.step() for _ in range(5)]
    out, rest = loop.drain()
    stats = [st for st in stats if st is not None] + rest
    assert len(stats) == 5 and all(st["samples"] == W * H for st in stats)
    assert counter[0] == 5 and len(log) == 5
    np.testing.assert_array_equal(out.numpy(), 2 * frame_image(4))
    # each reduce saw a complete frame: frame k's buffer was not zeroed under it
    # (drain() completes the outstanding reduces in buffer order, not frame order)
    want = sorted(float(frame_image(k).sum()) for k in range(5))
    assert sorted(log) == pytest.approx(want, rel=1e-6)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, frames, outdir, asynchronous=False, collective="reduce"):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench as b
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    counter = [0]
    bufs = [torch.zeros((H, W, 3)) for _ in range(2)]
    red = b.make_reduce(dist, "gloo", rank) if collective == "reduce" else b.make_gather(dist, "gloo", rank, world, W, H)
    if asynchronous:
        enqueue, wait = async_stub(stub_render(rank, world, counter))
        loop = b.FrameLoop(bufs, enqueue, red, wait=wait)
    else:
        loop = b.FrameLoop(bufs, stub_render(rank, world, counter), red)
    stats = [loop.step() for _ in range(frames)]
    fb, rest = loop.drain()
    stats = [st for st in stats if st is not None] + rest
    tot = torch.tensor([sum(s["samples"] for s in stats), sum(s["rays_traced"] for s in stats)], dtype=torch.float64)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    if rank == 0:
        np.save(os.path.join(outdir, "fb.npy"), fb.numpy())
        np.save(os.path.join(outdir, "tot.npy"), tot.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,asynchronous,collective", [(2, False, "reduce"), (3, False, "reduce"), (2, True, "reduce"),
                                                           (2, False, "gather"), (3, True, "gather")])
def test_gloo_frame_loop_assembles_every_frame(tmp_path, world, asynchronous, collective):
    frames = 3
    mp.spawn(_worker, args=(world, _free_port(), frames, str(tmp_path), asynchronous, collective), nprocs=world, join=True)
    fb = np.load(str(tmp_path / "fb.npy"))
    np.testing.assert_array_equal(fb, frame_image(frames - 1))
    tot = np.load(str(tmp_path / "tot.npy"))
    assert tot[0] == frames * W * H and tot[1] == 2 * frames * W * H
