"""Multi-process image-tile sharding on CPU: world_size-2 `gloo`.

Each rank asks libptamd which pixels its interleaved tiles hold (pt_shard_pixels: the kernels' own
slot -> pixel function, run on the host), renders them with the CPU oracle into a zero-filled
framebuffer; one reduce(SUM) assembles the image on rank 0, which must equal the single-process
render bit for bit.  The GPU job does the same with the kernel and RCCL (bench.py)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

from cudapathtracer_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, w, h, spp, outdir, tw=0, th=0):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle
    from conftest import load_scene
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = load_scene("cornell_blob")
    osc = oracle.OracleScene(s.arrays())
    cam = oracle.camera((0.0, 1.0, 3.0), 1.0, 3.0, 0.0, w, h)
    pix = shard.shard_pixels_lib(w, h, rank, world, tw, th)
    assert np.array_equal(pix, shard.shard_pixels(w, h, rank, world, tw, th))
    img, cnt = oracle.render(osc, cam, w, h, spp, 3, 0, 1234, pixels=pix, threads=2)
    fb = torch.from_numpy(img.astype(np.float32))
    dist.reduce(fb, dst=0, op=dist.ReduceOp.SUM)
    n = torch.tensor([len(pix)], dtype=torch.int64)
    dist.all_reduce(n)
    if rank == 0:
        np.save(os.path.join(outdir, "assembled.npy"), fb.numpy())
        np.save(os.path.join(outdir, "count.npy"), n.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_shards_partition_the_image():
    for w, h in ((40, 24), (1920, 1080), (13, 7)):
        for n in (1, 2, 3, 8):
            allp = np.concatenate([shard.shard_pixels_lib(w, h, k, n) for k in range(n)])
            assert len(allp) == w * h
            assert len(np.unique(allp)) == w * h


def test_library_tile_map_equals_python_mirror():
    """pt_shard_pixels (the kernels' unit_pixel, host-side) == cudapathtracer_amd.shard, incl. tile sizes."""
    for w, h in ((40, 24), (333, 97), (8, 8)):
        for tw, th in ((0, 0), (16, 8), (24, 40), (64, 64)):
            for n in (1, 3, 8):
                for k in range(n):
                    assert np.array_equal(shard.shard_pixels_lib(w, h, k, n, tw, th),
                                          shard.shard_pixels(w, h, k, n, tw, th))


@pytest.mark.timeout(300)
def test_gloo_two_rank_render_equals_single(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from conftest import load_scene
    w, h, spp = 40, 24, 2
    mp.spawn(_worker, args=(2, _free_port(), w, h, spp, str(tmp_path), 16, 8), nprocs=2, join=True)
    assembled = np.load(str(tmp_path / "assembled.npy"))
    assert int(np.load(str(tmp_path / "count.npy"))[0]) == w * h
    s = load_scene("cornell_blob")
    osc = oracle.OracleScene(s.arrays())
    full, _ = oracle.render(osc, oracle.camera((0.0, 1.0, 3.0), 1.0, 3.0, 0.0, w, h), w, h, spp, 3, 0, 1234)
    assert assembled.tobytes() == full.astype(np.float32).tobytes()
