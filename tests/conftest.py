import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
MODELS = os.path.join(GOLD, "scenes", "models")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# (obj, origin, scale, flip) load lists, as kernel.cu:590-599 calls loadOBJ
SCENE_SETS = {
    "cornell": [("cornell.obj", (0, 0, 0), 1.0, 0)],
    "cornell_blob": [("cornell.obj", (0, 0, 0), 1.0, 0), ("blob.obj", (0.35, 0.6, 0.3), 0.75, 0)],
    "quirks": [("quirks.obj", (0, 0, 0), 1.0, 0)],
    "blob_flip": [("blob.obj", (0.1, -0.2, 0.3), 1.5, 1)],
    "nomtl": [("nomtl.obj", (0, 0, 0), 1.0, 0)],
    "quad": [("quad.obj", (0, 0, 0), 1.0, 0)],
}


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


def _build_once():
    lib = os.path.join(ROOT, "cudapathtracer_amd", "libptamd.so")
    olib = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(ROOT, "cudapathtracer_amd", "csrc")])
    if not os.path.exists(olib):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


_build_once()


def load_scene(name, build_bvh=True):
    import cudapathtracer_amd as pt
    s = pt.Scene()
    for obj, origin, scale, flip in SCENE_SETS[name]:
        s.load_obj(os.path.join(MODELS, obj), origin, scale, flip, mtl_basepath=MODELS + "/")
    if build_bvh:
        s.build_bvh()
    return s


@pytest.fixture(scope="session")
def standin_scene(tmp_path_factory):
    """The ~262K-triangle stand-in (cudapathtracer_amd.scenes), loaded once per session."""
    import cudapathtracer_amd as pt
    from cudapathtracer_amd import scenes
    d = tmp_path_factory.mktemp("standin")
    p = scenes.write_sponza_standin(str(d))
    s = pt.Scene()
    s.load_obj(p, mtl_basepath=os.path.dirname(p) + "/")
    s.build_bvh()
    return s


@pytest.fixture(scope="session")
def scene_cache():
    return {}


def golden(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
