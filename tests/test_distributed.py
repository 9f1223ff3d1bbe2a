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


def _gpu_worker(rank, world, port, objpath, w, h, spp, outdir):
    """One rank of the GPU multi-process test: libptamd renders this rank's tile shard on GPU 0 (both
    integrators; integrator 0 through the host-buffer entry point, integrator 1 into a torch device
    tensor as bench.py does), gloo sums the shards on rank 0, which also renders the whole frame."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import cudapathtracer_amd as pt
    from cudapathtracer_amd import scenes
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = pt.Scene()
    s.load_obj(objpath, mtl_basepath=os.path.dirname(objpath) + "/")
    s.build_bvh()
    cam = pt.make_camera(width=w, height=h, **scenes.SPONZA_STANDIN_CAMERA)
    with pt.Renderer(s, 0) as r:
        for integ in (pt.PT_INTEGRATOR_UNIDIR, pt.PT_INTEGRATOR_HEAD):
            if integ == pt.PT_INTEGRATOR_UNIDIR:
                img, st = r.render(cam, w, h, spp, bounces=3, integrator=integ, seed=1234,
                                   shard_index=rank, shard_count=world)
                fb = torch.from_numpy(img.copy())
            else:
                d = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda:0")
                st = r.render_device(cam, d.data_ptr(), w, h, spp, bounces=3, integrator=integ, seed=1234,
                                     shard_index=rank, shard_count=world,
                                     stream_ptr=torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                fb = d.cpu()
            np.save(os.path.join(outdir, "shard_%d_r%d.npy" % (integ, rank)), fb.numpy())
            dist.reduce(fb, dst=0, op=dist.ReduceOp.SUM)
            n = torch.tensor([st["samples"]], dtype=torch.int64)
            dist.all_reduce(n)
            if rank == 0:
                full, _ = r.render(cam, w, h, spp, bounces=3, integrator=integ, seed=1234)
                np.save(os.path.join(outdir, "assembled_%d.npy" % integ), fb.numpy())
                np.save(os.path.join(outdir, "full_%d.npy" % integ), full)
                np.save(os.path.join(outdir, "samples_%d.npy" % integ), n.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_gpu_two_rank_libptamd_shards_reduce_to_full_frame(tmp_path):
    """SURVEY 8e on the GPU, across processes: two freshly spawned rank processes
    (the spawn start method: each a new interpreter; this file runs before any in-process GPU test)
    render their interleaved 8x8-tile shards of a 320x180 stand-in frame with libptamd on GPU 0, and a
    gloo reduce(SUM) assembles rank 0's image.  It must equal libptamd's single-process render of the
    whole frame bit for bit, for both integrators; each shard is zero outside its own tiles and the
    sample counts add up to W*H*spp.  (RCCL refuses two ranks on one device, so the reduce is gloo's;
    bench.py's RCCL leg differs only in the transport.)"""
    from cudapathtracer_amd import scenes
    d = tmp_path / "scene"
    d.mkdir()
    objpath = scenes.write_sponza_standin(str(d))
    w, h, spp, world = 320, 180, 16, 2
    mp.start_processes(_gpu_worker, args=(world, _free_port(), objpath, w, h, spp, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    for integ in (0, 1):
        assembled = np.load(str(tmp_path / ("assembled_%d.npy" % integ)))
        full = np.load(str(tmp_path / ("full_%d.npy" % integ)))
        assert assembled.shape == full.shape == (h, w, 3)
        assert int(np.load(str(tmp_path / ("samples_%d.npy" % integ)))[0]) == w * h * spp
        assert np.count_nonzero(full) > 0
        assert assembled.view(np.uint32).tobytes() == full.view(np.uint32).tobytes(), integ
        for k in range(world):
            sh = np.load(str(tmp_path / ("shard_%d_r%d.npy" % (integ, k)))).reshape(-1, 3)
            mine = np.zeros(w * h, dtype=bool)
            mine[shard.shard_pixels(w, h, k, world)] = True
            assert not np.any(sh[~mine]), (integ, k)
            assert sh[mine].view(np.uint32).tobytes() == full.reshape(-1, 3)[mine].view(np.uint32).tobytes()


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_gpu_plain_bench_gpus2_launches_its_own_ranks():
    """a plain `bench.py --gpus 2` (no torch.distributed.run, WORLD_SIZE unset) starts two
    rank processes itself and prints rank 0's one JSON line with n_gpus 2 and a finite image.  On the 1-GPU box
    the two ranks share GPU 0 over gloo (PT_BENCH_BACKEND=gloo; RCCL refuses two ranks on one device): the same
    launcher, FrameLoop, shard and reduce path the 8-GPU run takes with RCCL."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["PT_BENCH_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=380)
    sys.stderr.write(r.stderr[-3000:])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["image_finite"] is True
    assert d["config"]["rank_launcher"].startswith("bench.py")
    assert d["value"] > 0 and d["steps"] == 1


_NCCL_WORLD1 = r'''
import os, sys, json
sys.path.insert(0, %r)
import numpy as np
import torch
import torch.distributed as dist
import bench
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, init_method="tcp://127.0.0.1:%d", device_id=torch.device("cuda", 0))
W, H = 40, 24
out = {}
for kind in ("reduce", "gather"):
    fn = bench.make_reduce(dist, "nccl", 0) if kind == "reduce" else bench.make_gather(dist, "nccl", 0, 1, W, H)
    buf = torch.arange(H * W * 3, dtype=torch.float32, device="cuda").reshape(H, W, 3) / 7.0
    ref = buf.clone()
    work = fn(buf)
    assert work is not None          # RCCL: asynchronous
    work.wait()
    torch.cuda.synchronize()
    out[kind] = bool(torch.equal(buf, ref))
dist.destroy_process_group()
print(json.dumps(out))
'''


@pytest.mark.gpu
@pytest.mark.timeout(200)
def test_gpu_rccl_reduce_and_gather_world1():
    """bench.py's RCCL legs (make_reduce's async reduce, make_gather's async gather with the unpack done at
    wait()) run on a CUDA tensor in a one-rank RCCL group -- the asynchronous Work.wait() path the 8-GPU run takes --
    and leave rank 0's framebuffer exactly as rendered (with one rank the gather unpacks nothing and the reduce adds
    nothing).  Multi-device behaviour stays unmeasured here (1-GPU boxes)."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-c", _NCCL_WORLD1 % (ROOT, _free_port())], env=env, capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert res == {"reduce": True, "gather": True}
