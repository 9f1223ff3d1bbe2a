"""Gap between this build's arithmetic spec and the reference's own CUDA binary, CPU only.

The GPU image is bit-exact to the oracle; the oracle fixes three choices the reference's nvcc binary
makes differently or unknowably (FMA contraction, kernel.cu:68,86-87 cosf/sinf, curand_uniform's
rounding at kernel.cu:58).  oracle/Makefile builds one sensitivity variant of the oracle per choice;
tools/parity/ref_gap.py measures them at the C2/C3 configurations (profiles/r04_ref_gap).  These tests
pin the budget on a small fixture render (Cornell + blob, 64x64, 16 spp, depth 8, seed 1234; pixel 0
excluded as in SURVEY 8a d1) so that a change to the oracle or the variants that moves it is caught.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, load_scene

import oracle

sys.path.insert(0, os.path.join(ROOT, "tools", "parity"))
import ref_gap  # noqa: E402

W = H = 64
SPP, BOUNCES = 16, 8


@pytest.fixture(scope="module")
def fixture_render():
    if not all(os.path.exists(os.path.join(ROOT, "oracle", "variants", "liboracle_%s.so" % v)) for v in oracle.VARIANTS):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "variants"])
    osc = oracle.OracleScene(load_scene("cornell_blob").arrays())
    cam = oracle.camera((0.0, 1.0, 3.0), 1.0, 3.0, 0.0, W, H)
    pix = np.arange(1, W * H, dtype=np.uint32)
    ref, _ = oracle.render(osc, cam, W, H, SPP, BOUNCES, 0, 1234, pixels=pix)
    tri0, t0 = ref_gap.primary_hits(osc, cam, W, pix, None)

    def measure(variant):
        img, _ = oracle.render(osc, cam, W, H, SPP, BOUNCES, 0, 1234, pixels=pix, variant=variant)
        tri1, t1 = ref_gap.primary_hits(osc, cam, W, pix, variant)
        return ref_gap.gap(ref, img, pix, (tri0 != tri1) | (t0 != t1), tri0 != tri1)
    return measure


def test_unfused_uniform_is_bit_identical(fixture_render):
    """curand_uniform fused or rounded twice is the same float for every draw: (float)x * 2^-32 is exact
    (a power-of-two scaling of a 24-bit significand), so only the addition rounds.  The spec's choice
     therefore cannot matter."""
    g = fixture_render("unfused")
    assert g["pixels_differing_fp32"] == 0 and g["rmse_tonemapped"] == 0.0
    # and directly, on a spread of 32-bit draws: the double-precision sum of the exact product and 2^-33,
    # rounded once to float (the fused form), equals the twice-rounded float form
    x = np.unique(np.concatenate([np.random.default_rng(5).integers(0, 2**32, 200000, dtype=np.uint64),
                                  np.array([0, 1, 2**24 - 1, 2**24 + 1, 2**31, 2**32 - 1], dtype=np.uint64)]))
    xf = x.astype(np.float32)
    prod = (xf * np.float32(2.3283064e-10)).astype(np.float32)
    assert np.array_equal(prod.astype(np.float64), xf.astype(np.float64) * np.float64(np.float32(2.3283064e-10)))
    twice = (prod + np.float32(2.3283064e-10 / 2)).astype(np.float32)
    fused = (xf.astype(np.float64) * np.float64(np.float32(2.3283064e-10)) +
             np.float64(np.float32(2.3283064e-10 / 2))).astype(np.float32)
    assert np.array_equal(twice.view(np.uint32), fused.view(np.uint32))


@pytest.mark.parametrize("variant", ["libm", "ulp1", "ulp2"])
def test_sincos_choice_within_budget(fixture_render, variant):
    """glibc sinf/cosf, or det_sincos moved by up to CUDA's documented 2 ulp: no camera ray changes and the
    image stays far inside the north-star RMSE 1e-4 (measured 1.9e-10 / 1.7e-9 / 3.2e-9 here)."""
    g = fixture_render(variant)
    assert g["primary_hit_flips"] == 0
    assert g["rmse_tonemapped"] <= 1e-6


def test_fma_contraction_open_parity_risk_is_camera_ray_triangle_changes(fixture_render):
    """OPEN PARITY RISK (not expected behaviour; DESIGN.md 5 "Gap to the reference binary"): the reference's
    compile.bat builds with nvcc's default -fmad=true, and contracting triIntersect's dot/cross products
    changes which triangle some camera rays hit where they pass within rounding of an edge (exact-edge
    pixels of the axis-aligned fixture); those pixels' paths diverge completely and the image RMSE exceeds
    the north-star 1e-4 (8.0e-3 here; C2 1e-3..2e-3 and C3 6.0e-4 at full size, profiles/r04_ref_gap,
    profiles/r05_ref_gap).  This pins WHERE the risk lives -- only there: the rest of the image stays far
    inside 1e-4, and without the triangle test contracted the whole image does -- so that a change that
    widens it is caught.  It cannot be closed here (no nvcc; which products get fused is the compiler's
    choice, see the next test)."""
    g = fixture_render("fma")
    assert g["rmse_tonemapped"] > 1e-4
    assert 0 < g["primary_triangle_flips"] < 0.05 * g["pixels"]
    assert g["rmse_tonemapped_no_primary_triangle_flips"] <= 1e-5
    g2 = fixture_render("fma_notri")
    assert g2["primary_triangle_flips"] == 0
    assert g2["rmse_tonemapped"] <= 1e-6


def test_fma_contraction_shape_matters_as_much_as_contraction():
    """Why the spec stays uncontracted ("pick the spec from that evidence"): triIntersect with
    the contraction spelled out -- the left product of each a*b +- c*d fused (LLVM's DAG-combiner order,
    oracle variant fmal_tri) or the right one (fmar_tri) -- gives images that differ from EACH OTHER by about
    as much as either differs from the uncontracted spec (C2 full frame: 2.0e-3 / 2.4e-3 against the spec,
    1.95e-3 between the two shapes; profiles/r05_ref_gap), through the same camera-ray edge flips.  GCC's own
    choice (fma_tri) matches neither shape bit for bit.  So adopting a contracted spec would only be closer
    to the nvcc binary if it guessed nvcc's (and ptxas's) fused shapes exactly; the uncontracted IEEE spec is
    the compiler-independent one."""
    osc = oracle.OracleScene(load_scene("cornell_blob").arrays())
    cam = oracle.camera((0.0, 1.0, 3.0), 1.0, 3.0, 0.0, W, H)
    pix = np.arange(1, W * H, dtype=np.uint32)
    imgs, hits = {}, {}
    for v in (None, "fmal_tri", "fmar_tri", "fma_tri"):
        imgs[v], _ = oracle.render(osc, cam, W, H, SPP, BOUNCES, 0, 1234, pixels=pix, variant=v)
        hits[v] = ref_gap.primary_hits(osc, cam, W, pix, v)[0]

    def g(a, b):
        return ref_gap.gap(imgs[a], imgs[b], pix, hits[a] != hits[b], hits[a] != hits[b])
    lr, l0, r0 = g("fmal_tri", "fmar_tri"), g(None, "fmal_tri"), g(None, "fmar_tri")
    assert lr["primary_triangle_flips"] > 0 and lr["rmse_tonemapped"] > 1e-4
    assert lr["rmse_tonemapped"] > 0.5 * min(l0["rmse_tonemapped"], r0["rmse_tonemapped"])
    # outside the camera-ray triangle changes the shapes agree to far inside the budget
    assert lr["rmse_tonemapped_no_primary_triangle_flips"] <= 1e-5
    # GCC's own contraction matches neither spelled-out shape bit for bit (both inequalities asserted)
    assert not np.array_equal(imgs["fma_tri"], imgs["fmal_tri"])
    assert not np.array_equal(imgs["fma_tri"], imgs["fmar_tri"])
