"""The C-ABI library: loads without a GPU, exports every entry point include/pt/pt.h declares,
and fails loudly (error code + message, no exit) where a GPU or valid input is required."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT, load_scene

import cudapathtracer_amd as pt
from cudapathtracer_amd import _lib


def _declared_functions():
    txt = open(os.path.join(ROOT, "include", "pt", "pt.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pt_[a-z0-9_]+)\s*\(", txt)))


def test_exports_every_declared_symbol():
    names = _declared_functions()
    assert len(names) >= 18
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    exported = set(re.findall(r" T (pt_[a-z0-9_]+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    assert set(names) == set(_lib.SIGNATURES), "ctypes table out of sync with pt.h"
    # and nothing beyond the declared C surface leaks out with C linkage
    assert exported == set(names)


def test_abi_version_and_error_channel():
    L = _lib.lib()
    assert L.pt_abi_version() == 6
    rc = L.pt_render(None, None, None, None, None)
    assert rc == _lib.PT_E_INVALID
    assert b"null" in L.pt_last_error()


def test_create_without_gpu_fails_cleanly():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    s = load_scene("cornell")
    with pytest.raises(pt.PtError) as e:
        pt.Renderer(s, 0)
    assert e.value.code in (_lib.PT_E_NODEV, _lib.PT_E_HIP)


def test_create_rejects_bad_scenes():
    L = _lib.lib()
    v = _lib.SceneView()
    err = C.c_int(0)
    h = L.pt_create(C.byref(v), 0, C.byref(err))
    assert not h and err.value == _lib.PT_E_INVALID
    s = load_scene("cornell")
    v = s.view()
    v.bvh_size = 3                      # inconsistent with num_tris - 1
    h = L.pt_create(C.byref(v), 0, C.byref(err))
    assert not h and err.value == _lib.PT_E_SCENE


def test_no_cpu_fallback_in_product():
    """The product package never imports or links the oracle (test infrastructure)."""
    pkg = os.path.join(ROOT, "cudapathtracer_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dp, f), errors="ignore").read()
                assert "import oracle" not in txt and "pt_oracle" not in txt and "liboracle" not in txt, f
    out = subprocess.check_output(["ldd", _lib.LIB_PATH]).decode()
    assert "oracle" not in out


def test_group_entry_points_reject_bad_arguments():
    """pt_group_* / pt_render_multi (one process, N GPUs, RCCL reduce) validate before touching a
    device: no contexts, a null context, null buffers."""
    L = _lib.lib()
    err = C.c_int(0)
    assert not L.pt_group_create(None, 0, C.byref(err)) and err.value == _lib.PT_E_INVALID
    arr = (C.c_void_p * 2)(None, None)
    assert not L.pt_group_create(arr, 2, C.byref(err)) and err.value == _lib.PT_E_INVALID
    assert b"null" in L.pt_last_error()
    assert L.pt_render_group(None, None, None, None, None) == _lib.PT_E_INVALID
    assert L.pt_render_multi(None, 0, None, None, None, None) == _lib.PT_E_INVALID
    assert L.pt_group_size(None) == 0
    L.pt_group_destroy(None)
    assert L.pt_tri_counts(None, None, 0) == _lib.PT_E_INVALID
    assert L.pt_trace_counts(None, 1, None, None, None, 0, None, None) == _lib.PT_E_INVALID
