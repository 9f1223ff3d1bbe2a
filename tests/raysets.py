"""Ray sets for the ray-level parity tests and the trace() goldens (tools/make_golden.py).

What the integrator produces (camera rays, rays leaving surfaces at t - 0.001) plus the edge
cases of the slab test (axis-parallel rays, zero direction components, origins on box planes
and vertices, tiny components that leave the Markstein range, rays from outside the scene)."""
import numpy as np


def _unit(v):
    return (v / np.linalg.norm(v, axis=1)[:, None]).astype(np.float32)


def ray_sets(arrays, n, seed):
    """Dict of named (origins, directions) float32 arrays over the scene's bounds."""
    rng = np.random.default_rng(seed)
    v = arrays["verts"]
    P = np.stack([v["x"], v["y"], v["z"]], axis=1).astype(np.float64)
    lo, hi = P.min(0), P.max(0)
    ext = hi - lo
    out = {}
    o = rng.uniform(lo + 0.05 * ext, hi - 0.05 * ext, (n, 3))
    out["interior"] = (o.astype(np.float32), _unit(rng.normal(size=(n, 3))))
    d = rng.normal(size=(n, 3))
    axis = rng.integers(0, 3, n)
    zero = rng.integers(0, 3, n)
    d[np.arange(n), zero] = 0.0                     # one zero component
    d[: n // 3] = 0.0
    d[np.arange(n // 3), axis[: n // 3]] = rng.choice([-1.0, 1.0], n // 3)   # axis-parallel
    out["axis"] = (o.astype(np.float32), _unit(d))
    # origins on vertices and on their coordinate planes
    pick = P[rng.integers(0, len(P), n)]
    o2 = pick.copy()
    o2[n // 2:, 0] = rng.uniform(lo[0], hi[0], n - n // 2)
    out["vertex_planes"] = (o2.astype(np.float32), _unit(rng.normal(size=(n, 3))))
    # tiny components: outside the Markstein preconditions (exact slow path)
    d3 = rng.normal(size=(n, 3))
    d3[:, 1] = rng.choice([1e-31, -1e-36, 3e-39, 1e-20], n)
    out["tiny"] = (o.astype(np.float32), _unit(d3))
    # from outside: aimed at the scene
    c = 0.5 * (lo + hi)
    far = c + _unit(rng.normal(size=(n, 3))) * (2.0 * np.linalg.norm(ext) + 1.0)
    tgt = rng.uniform(lo, hi, (n, 3))
    out["outside"] = (far.astype(np.float32), _unit(tgt - far))
    return out


def bounce_rays(arrays, o, d, tri, t, seed):
    """Rays leaving the surfaces hit by (o, d) the way the integrator builds them
    (kernel.cu:455-470: pos = o + d * (float)(t - 0.001))."""
    rng = np.random.default_rng(seed)
    hit = tri >= 0
    tt = (t[hit].astype(np.float64) - 0.001).astype(np.float32)
    pos = (o[hit] + d[hit] * tt[:, None]).astype(np.float32)
    return pos, _unit(rng.normal(size=(len(pos), 3)))
