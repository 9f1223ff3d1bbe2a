"""Randomised parity sweep: random triangle soups (tests/test_gpu_random_scenes.py's generator: duplicates, fans,
axis-aligned and zero-area triangles), each rendered with random image size, samples, depth, integrator, lens radius,
camera position and seed on the wavefront kernel, against the oracle, bit for bit (kernel.cu:417-515 / :217-415), plus
a batch of random rays through pt_trace against the oracle's `trace` (kernel.cu:112-161).

PT_PARITY_SWEEP=N sets the number of cases (default 8, a few seconds); a long sweep is run as
`PT_PARITY_SWEEP=200 PT_PARITY_SWEEP_LOG=path python -m pytest tests/test_gpu_parity_sweep.py -m gpu`, and the log
(one JSON line per case) is kept under profiles/.
"""
import json
import os

import numpy as np
import pytest

import cudapathtracer_amd as pt
from test_gpu_random_scenes import write_soup

pytestmark = pytest.mark.gpu

N_CASES = int(os.environ.get("PT_PARITY_SWEEP", "8"))


def case_params(k):
    rng = np.random.default_rng(7000 + k)
    return dict(
        soup=int(1000 + k),
        w=int(rng.integers(4, 41)), h=int(rng.integers(4, 33)),
        spp=int(rng.integers(1, 7)), bounces=int(rng.integers(1, 9)),
        integrator=int(rng.integers(0, 2)),
        radius=float(rng.choice([0.0, 0.0, 0.03, 0.2])),
        pos=tuple(float(x) for x in (rng.uniform(-0.6, 0.6), 1.0 + rng.uniform(-0.5, 0.5), 3.0 + rng.uniform(-0.8, 0.8))),
        focal=float(rng.choice([2.0, 3.0, 5.0])),
        seed=int(rng.integers(1, 2**31 - 1)),
    )


@pytest.mark.parametrize("k", range(N_CASES))
def test_random_case_matches_the_oracle(k, tmp_path):
    import oracle
    c = case_params(k)
    p = write_soup(str(tmp_path), c["soup"])
    s = pt.Scene()
    s.load_obj(p, mtl_basepath=str(tmp_path) + "/")
    s.build_bvh()
    osc = oracle.OracleScene(s.arrays())
    with pt.Renderer(s, 0) as r:
        cam = pt.make_camera(pos=c["pos"], dist_from_film=1.0, focal_length=c["focal"], radius=c["radius"],
                             width=c["w"], height=c["h"])
        img, st = r.render(cam, c["w"], c["h"], c["spp"], bounces=c["bounces"], integrator=c["integrator"],
                           seed=c["seed"])
        ocam = oracle.camera(c["pos"], 1.0, c["focal"], c["radius"], c["w"], c["h"])
        ref, cnt = oracle.render(osc, ocam, c["w"], c["h"], c["spp"], c["bounces"], c["integrator"], c["seed"])
        diff = int(np.count_nonzero(img.view(np.uint32) != ref.astype(np.float32).view(np.uint32)))
        rng = np.random.default_rng(9000 + k)
        n = 4000
        o = rng.uniform(-2.5, 2.5, (n, 3)).astype(np.float32)
        d = rng.normal(0, 1, (n, 3))
        d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
        gt, gtt = r.trace(o, d)
    rt, rtt = oracle.trace_batch(osc, o, d)
    tdiff = int(np.count_nonzero(gt != rt)) + int(np.count_nonzero(gtt.view(np.uint32) != rtt.view(np.uint32)))
    log = os.environ.get("PT_PARITY_SWEEP_LOG")
    if log:
        with open(log, "a") as fh:
            fh.write(json.dumps(dict(case=k, **c, pixel_diffs=diff, trace_diffs=tdiff,
                                     rays_traced=int(st["rays_traced"]), rays_reference=int(st["rays_reference"]),
                                     nonzero=int(np.count_nonzero(img)))) + "\n")
    assert diff == 0, (c, diff)
    assert st["rays_reference"] == cnt["traces"], c
    assert tdiff == 0, (c, tdiff)
